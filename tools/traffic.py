#!/usr/bin/env python3
"""HBM traffic per launch of the two roofline kernels, from the rocprofv3 PMC
passes of tools/gpu_round.sh (pmc1 = FETCH_SIZE, pmc2 = WRITE_SIZE, both run
on `bench.py --steps 1 --warmup 0`).

A "launch" is the whole launch sequence the bench times with HIP events
(local_bench: the single k_local_fused<0> dispatch of a bench phase):
  scan  : k_prep_aconst .. k_scan_combine_bf of one thx_global_scan call whose
          k_scan_split grid is the 4096-image grid (bench.scan_roofline);
  local : one thx_local_phase call of bench.local_roofline (full resolution,
          512 images, grid 512 x 512): per cloud (1.5, 2, 3 degrees, uniform)
          four launches (timed_events: one warm-up + 3) in each layout, in the
          order half-complex (k_local_fused<0>, not routed: one dispatch),
          cells (k_local_fused<1>), y-pair (k_local_fused<2>) -- sliced per
          cloud and layout so each by_cloud time of the bench pairs with the
          traffic of the same dispatches;
  local_bench : the bench step's routed phase (k_local_fused<0> staged
          variant, exits at entry, + k_local_fused<2>) over 12 500 images.
Bytes: FETCH_SIZE is 64 B per memory-side read request (TCC_EA0_RDREQ x 64),
whatever the request's size.  profiles/r02_fetch_calibration.json measured
what that means per access shape on gfx950: wide coalesced reads (128-B
requests: streaming loads, LDS DMA, the staged box rows) are counted at half
their bytes (x2), 64-B cell gathers exactly (x1), and 16-B pieces on separate
rows (the half-complex interp_ft taps) as one 64-B request each -- 64 B
moved per piece, so x1 is the HBM traffic there too.  Each summary carries the
factor of its dominant access shape plus the two bounds (x1 .. x2) when the
launch mixes shapes; WRITE_SIZE x 1024 is exact for streaming stores
(MI355X_MICROARCH.md, HBM section).  When a pmc3 pass with TCC_EA0_RDREQ and
TCC_EA0_RDREQ_128B (if the box lists it) exists, the split is exact:
64 B x (RDREQ - RDREQ_128B) + 128 B x RDREQ_128B.

  python tools/traffic.py gpurun_out/TAG profiles/rNN_traffic.json
"""
import csv
import json
import os
import re
import sys


def dispatches(path, counter):
    rows = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            d = int(r["Dispatch_Id"])
            name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
            e = rows.setdefault(d, [name, int(r["Grid_Size"]), 0.0])
            e[2] += float(r["Counter_Value"])
    return [rows[d] for d in sorted(rows)]


def groups(disp, start, end):
    out, cur = [], None
    for name, grid, val in disp:
        if start in name:
            cur = []
        if cur is not None:
            cur.append((name, grid, val))
            if end in name:
                out.append(cur)
                cur = None
    return out


def _entry(fetch_kib, write_kib, factor, launches, kernels, shape):
    r = fetch_kib * 1024 * factor
    w = write_kib * 1024
    return {"read_bytes": r, "write_bytes": w, "traffic_bytes": r + w, "launches": launches,
            "fetch_factor": factor, "access_shape": shape,
            "traffic_bytes_bounds": [fetch_kib * 1024 + w, fetch_kib * 2048 + w],
            "kernels": kernels}


def summarise(rd, wr, start, end, pick, factor, shape, first=None):
    gr = [g for g in groups(rd, start, end) if pick(g)][:first]
    gw = [g for g in groups(wr, start, end) if pick(g)][:first]
    if not gr or not gw:
        return None
    f = sum(sum(v for _, _, v in g) for g in gr) / len(gr)
    w = sum(sum(v for _, _, v in g) for g in gw) / len(gw)
    return _entry(f, w, factor, len(gr), [n.split("(")[0] for n, _, _ in gr[-1]], shape)


def single(rd, wr, name, grid, factor, shape, per=1):
    """Average bytes per launch of one kernel at one grid size; `per`
    consecutive dispatches make one launch (a routed phase dispatches the
    staged and the box-less variant, one of them exits at entry)."""
    r = [v for n, g, v in rd if name in n and g == grid]
    w = [v for n, g, v in wr if name in n and g == grid]
    if not r or not w:
        return None
    return _entry(sum(r) / len(r) * per, sum(w) / len(w) * per, factor, len(r) // per, [name],
                  shape)


def routed_phase(rd, wr, grid, factor, shape):
    """Bytes per routed bench phase: its staged half-complex dispatch
    (k_local_fused<0>) plus, with a y-pair copy, the pair-form dispatch
    (k_local_fused<2>, LAYOUT_YPAIR2) or, without, the box-less <0> variant;
    the kernel not chosen exits at entry."""
    r0 = [v for n, g, v in rd if "k_local_fused<0," in n and g == grid]
    w0 = [v for n, g, v in wr if "k_local_fused<0," in n and g == grid]
    r2 = [v for n, g, v in rd if "k_local_fused<2," in n and g == grid]
    w2 = [v for n, g, v in wr if "k_local_fused<2," in n and g == grid]
    if not r0 or not w0:
        return None
    nph = len(r2) if r2 else len(r0) // 2
    return _entry((sum(r0) + sum(r2)) / nph, (sum(w0) + sum(w2)) / nph, factor, nph,
                  ["k_local_fused<0,", "k_local_fused<2,"], shape)


def sliced(rd, wr, name, grid, k, per, factor, shape, pair=1):
    """Average bytes per launch of the k-th run of `per` consecutive launches
    of one kernel at one grid (bench.local_roofline: 1 + reps launches per
    cloud and layout); `pair` dispatches make one launch (routed phases)."""
    n0, n1 = k * per * pair, (k + 1) * per * pair
    r = [v for n, g, v in rd if name in n and g == grid][n0:n1]
    w = [v for n, g, v in wr if name in n and g == grid][n0:n1]
    if not r or not w:
        return None
    return _entry(sum(r) / len(r) * pair, sum(w) / len(w) * pair, factor, len(r) // pair, [name],
                  shape)


def exact_split(tag, name, grid, k=None, per=None):
    """64 B x (RDREQ - RDREQ_128B) + 128 B x RDREQ_128B per dispatch, from a
    pmc3 pass, or None; k / per: the k-th run of `per` dispatches only."""
    p = os.path.join(tag, "pmc3", "run_counter_collection.csv")
    if not os.path.exists(p):
        return None
    req = [v for n, g, v in dispatches(p, "TCC_EA0_RDREQ_sum") if name in n and g == grid]
    big = [v for n, g, v in dispatches(p, "TCC_EA0_RDREQ_128B_sum") if name in n and g == grid]
    if k is not None:
        req, big = req[k * per:(k + 1) * per], big[k * per:(k + 1) * per]
    if not req or not big:
        return None
    a, b = sum(req) / len(req), sum(big) / len(big)
    return {"read_bytes": 64 * (a - b) + 128 * b, "requests": a, "requests_128B": b}


CLOUDS = ("1.5", "2.0", "3.0", "uniform")          # bench.local_roofline spreads
LAYOUTS = (("halfcomplex", "k_local_fused<0,", 2, "staged box rows (128-B requests) + 16-B row taps"),
           ("cells", "k_local_fused<1,", 1, "64-B cell gathers"),
           ("ypair", "k_local_fused<2,", 1, "32-B / 64-B y-pair pieces"))


def local_fullres(tag, rd, wr):
    """Per cloud and layout: bytes per launch of the full-resolution phase, the
    FETCH_SIZE factor of the dominant access shape, and the exact 64 / 128-B
    split where the pmc3 pass has it (then read_bytes is exact)."""
    out = {}
    for k, cl in enumerate(CLOUDS):
        row = {}
        for lay, name, factor, shape in LAYOUTS:
            e = sliced(rd, wr, name, 512 * 512, k, 4, factor, shape)
            if e is None:
                continue
            ex = exact_split(tag, name, 512 * 512, k, 4)
            if ex:
                e["exact_read"] = ex
                e["read_bytes"] = ex["read_bytes"]
                e["traffic_bytes"] = ex["read_bytes"] + e["write_bytes"]
            row[lay] = e
        out[cl] = row
    return out


def main():
    tag, out = sys.argv[1], sys.argv[2]
    rd = dispatches(os.path.join(tag, "pmc1", "run_counter_collection.csv"), "FETCH_SIZE")
    wr = dispatches(os.path.join(tag, "pmc2", "run_counter_collection.csv"), "WRITE_SIZE")
    # the bf16x6 scan kernel's grid at 4096 images, nR 2000 (64-image tiles x
    # 250 blocks of 8 rotations, 512 threads each)
    scan_grid = (4096 // 64) * 250 * 512
    res = {
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py ({tag}), "
                  "FETCH_SIZE x2 on gfx950",
        "scan_4096": summarise(rd, wr, "k_prep_aconst", "k_scan_combine_bf",
                               lambda g: any("k_scan_split" in n and gr == scan_grid
                                             for n, gr, _ in g), 2, "streaming (128-B requests)"),
        # bench.local_roofline, every cloud and layout (not routed: one
        # dispatch per launch)
        "local_fullres_512": local_fullres(tag, rd, wr),
        # the bench step's dominant kernel: one k_local_fused<0> launch per
        # phase over the whole 12 500-image batch (grid 12500 x 1 x 1 of 512)
        "local_bench": routed_phase(rd, wr, 12500 * 512, 2,
                                    "16-B row taps / 32-B y-pair pieces"),
    }
    ex = exact_split(tag, "k_local_fused<2,", 12500 * 512)
    if ex and res["local_bench"]:
        res["local_bench"]["exact_read_ypair"] = ex
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
