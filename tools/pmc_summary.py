#!/usr/bin/env python3
"""Summarise rocprofv3 outputs of tools/gpu_round.sh: per kernel the launch
count and average duration (kernel trace) and the average HBM bytes per launch
(FETCH_SIZE x 2 on gfx950, WRITE_SIZE as is -- MI355X_MICROARCH.md, HBM
section), plus the L2 hit rate.

  python tools/pmc_summary.py gpurun_out/TAG [--json out.json]
"""
import argparse
import csv
import json
import os
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    m = re.match(r"(?:void )?([A-Za-z_][\w:]*(?:<[^()]*>)?)", name)
    return m.group(1) if m else name[:60]


BY_GRID = False


def key(name, grid):
    return f"{short(name)} [{grid}]" if BY_GRID else short(name)


def read_counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return acc
    with open(path) as f:
        for r in csv.DictReader(f):
            acc[key(r["Kernel_Name"], int(r["Grid_Size"]))][r["Counter_Name"]].append(
                float(r["Counter_Value"]))
    return acc


def read_trace(path):
    durs = defaultdict(list)
    if not os.path.exists(path):
        return durs
    with open(path) as f:
        for r in csv.DictReader(f):
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            durs[key(r["Kernel_Name"], g)].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    return durs


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dir")
    p.add_argument("--json")
    p.add_argument("--by-grid", action="store_true", help="separate launches by grid size")
    p.add_argument("--top", type=int, default=25)
    a = p.parse_args()
    global BY_GRID
    BY_GRID = a.by_grid
    durs = read_trace(os.path.join(a.dir, "prof", "run_kernel_trace.csv"))
    cnt = {}
    for i in range(1, 10):
        f = os.path.join(a.dir, f"pmc{i}", "run_counter_collection.csv")
        for k, d in read_counters(f).items():
            cnt.setdefault(k, {}).update(d)
    out = {}
    names = sorted(set(durs) | set(cnt), key=lambda k: -sum(durs.get(k, [0])))[:a.top]
    print(f"{'kernel':70s} {'n':>5s} {'avg ms':>9s} {'tot ms':>9s} {'rd MB':>9s} {'wr MB':>9s} "
          f"{'GB/s':>8s} {'L2 hit':>7s}")
    for k in names:
        d = durs.get(k, [])
        c = cnt.get(k, {})
        avg = sum(d) / len(d) if d else float("nan")
        rd = 2 * 1024 * sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) if "FETCH_SIZE" in c else None
        wr = 1024 * sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"]) if "WRITE_SIZE" in c else None
        hit = None
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            h, m = sum(c["TCC_HIT_sum"]), sum(c["TCC_MISS_sum"])
            hit = h / max(h + m, 1)
        bw = (rd or 0) + (wr or 0)
        gbs = bw / (avg * 1e-3) / 1e9 if d and bw else None
        out[k] = {"launches": len(d), "avg_ms": avg, "total_ms": sum(d), "hbm_read_bytes": rd,
                  "hbm_write_bytes": wr, "hbm_GBs": gbs, "l2_hit": hit}
        f = lambda v, s=1e6: f"{v / s:9.2f}" if v is not None else f"{'-':>9s}"
        print(f"{k[:70]:70s} {len(d):5d} {avg:9.3f} {sum(d):9.1f} {f(rd)} {f(wr)} "
              f"{(f'{gbs:8.0f}' if gbs else '       -')} {(f'{hit:7.3f}' if hit is not None else '      -')}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
