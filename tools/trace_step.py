"""Timeline of one bench step from a rocprofv3 kernel trace (diagnostic).

tools/gpu_round.sh prof writes prof/run_kernel_trace.csv for `bench.py
--steps 3 --warmup 1`; this prints, for the last expectation call (the last
k_scan_split dispatch to the end of its last phase), every dispatch with its
start offset, duration and stream, the busy time of the main stream's
k_scan / k_local kernels, and the gaps on the path between them -- the time
the particle-filter chain keeps the local phases waiting.
  python tools/trace_step.py gpurun_out/TAG/prof/run_kernel_trace.csv [--all]
"""
import csv
import re
import sys


def short(name):
    m = re.search(r"(k_[A-Za-z0-9_]+)(<[^>(]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name.split("(")[0][-40:]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                  r["Queue_Id"]) for r in rows), key=lambda e: e[0])
    scans = [i for i, e in enumerate(ev) if e[2].startswith("k_scan_split")]
    i0 = scans[-1]
    # back to the prep kernels of this scan
    while i0 > 0 and ev[i0 - 1][2].startswith(("k_prep", "k_scan_bias", "k_project3d", "k_rotmat",
                                              "k_trans_table")):
        i0 -= 1
    locs = [i for i, e in enumerate(ev) if e[2].startswith("k_local_fused") and i > i0]
    # phases: the routed pair, the y-pair one does the work
    i1 = max(locs)
    while i1 + 1 < len(ev) and ev[i1 + 1][2].startswith(("k_pf", "k_gather", "k_top", "k_resample")):
        i1 += 1
    t0 = ev[i0][0]
    seg = ev[i0:i1 + 1]
    if "--all" in sys.argv:
        for s, e, n, q in seg:
            print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} q{q} {n}")
    span = (seg[-1][1] - t0) / 1e6
    work = {}
    for s, e, n, q in seg:
        work.setdefault(n, [0, 0.0])
        work[n][0] += 1
        work[n][1] += (e - s) / 1e6
    print(f"step span {span:.2f} ms ({len(seg)} dispatches)")
    for n, (c, t) in sorted(work.items(), key=lambda kv: -kv[1][1]):
        print(f"  {t:8.3f} ms {c:4d} x {n}")
    # gaps between consecutive heavy kernels (scan / local of the y-pair route)
    heavy = [x for x in seg if x[2].startswith(("k_scan_split", "k_local_fused<2"))]
    gaps = [(heavy[k + 1][0] - heavy[k][1]) / 1e6 for k in range(len(heavy) - 1)]
    busy = sum((e - s) for s, e, *_ in heavy) / 1e6
    print(f"heavy kernels busy {busy:.2f} ms; gaps between them: " + ", ".join(f"{g:.3f}" for g in gaps))
    print(f"time outside scan + local: {span - busy:.2f} ms")


if __name__ == "__main__":
    main()
