#!/usr/bin/env python3
"""L2 -> L1 line traffic of the bench's k_local_fused launches, from one
rocprofv3 --pmc pass over `bench.py --steps 1 --warmup 0 --no-extras`
(tools/gpu_r03j.sh): TCP_TCC_READ_REQ (L1 -> L2 read requests, one 128-B
line each), TCP_TOTAL_CACHE_ACCESSES, TCC_HIT / TCC_MISS per dispatch, in
launch order (= phase order).  bench.py prices the kernel's line traffic
against the L2 bandwidth with it.

  python tools/l2_lines.py gpurun_out/TAG/pmc_lines profiles/r03_l2_lines.json
"""
import csv
import json
import os
import re
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    rows = {}
    for root, _, files in os.walk(src):
        for fn in files:
            if not fn.endswith("counter_collection.csv"):
                continue
            with open(os.path.join(root, fn)) as f:
                for r in csv.DictReader(f):
                    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
                    if "k_local_fused" not in name or int(r["Grid_Size"]) != 12500 * 512:
                        continue
                    d = rows.setdefault(int(r["Dispatch_Id"]),
                                        {"_nostage": re.search(r"false, false>", name) is not None,
                                         "_staged": re.search(r"<0, false, 1, false, true>", name)
                                         is not None})
                    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # a routed phase is two or three dispatches (the staged kernel, the
    # box-less one, the y-pair one; those not chosen exit at entry): a staged
    # dispatch opens a phase, the others add to it
    phases, cur = [], None
    for k in sorted(rows):
        d = rows[k]
        d.pop("_nostage")
        staged = d.pop("_staged")
        if staged or cur is None:
            if cur is not None:
                phases.append(cur)
            cur = dict(d)
            continue
        for c, v in d.items():
            cur[c] = cur.get(c, 0.0) + v
    if cur is not None:
        phases.append(cur)
    if not phases:
        sys.exit("no k_local_fused dispatches at the bench grid")
    keys = sorted(phases[0])
    mean = {k: sum(p.get(k, 0.0) for p in phases) / len(phases) for k in keys}
    res = {"source": f"rocprofv3 --pmc over bench.py --steps 1 --warmup 0 ({src})",
           "kernel": "k_local_fused, grid 12500 x 512 (one launch per phase)",
           "line_bytes": 128, "per_phase": phases, "mean": mean}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(mean, indent=1))


if __name__ == "__main__":
    main()
