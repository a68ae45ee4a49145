#!/usr/bin/env python3
"""inferACG fixed-point iterations of the perturbation mean on the bench's
particle clouds: the C3 workload (bench.make_workload) run for k = 1 .. 10
phases; the resampled clouds after phase k are the next phase's k_pf_mean
input.  Prints one JSON line per k: the iteration histogram and the
k_pf_mean time, and the median number of runs of equal particles (distinct
ancestors, as k_gather stores copies together) over all and over capped clouds."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from thunder_amd import expectation as ex, ops, synth  # noqa: E402
from thunder_amd._lib import check, lib  # noqa: E402

dev = torch.device("cuda", 0)
n = int(os.environ.get("PF_ITERS_N", "4096"))
# the bench's C3 workload (bench.main): box 256, pf 2, rU 24, nR 2000, nT 151
vol = synth.projectee(synth.blob_volume(256, seed=1, device=dev), 2)
_, nR, nT = ops.global_sample_sizes(2000)
gset = tuple(x.cpu().numpy() for x in ops.global_sample_set(nR, nT, 10.0, 2, dev))
px, dat, ctf, sig, _, _ = bench.make_stack(256, 2, 24, 1, n, dev, seed=5, vol=vol)
st = torch.cuda.current_stream(dev)
for k in range(1, 11):
    e = ex.Expectation(vol, px, gset, n_phase=k, seed=7)
    quat = e.run(dat, ctf, sig)[0]
    mq = torch.empty(n, 4, dtype=torch.float64, device=dev)
    it = torch.empty(n, dtype=torch.int32, device=dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    check(lib().thx_pf_acg_mean(n, quat.shape[1], ops._ptr(quat), 100, ops._ptr(mq), ops._ptr(it),
                                ctypes.c_void_p(st.cuda_stream)), "thx_pf_acg_mean")
    b.record(st)
    torch.cuda.synchronize()
    h = it.cpu().numpy()
    q = quat.cpu().numpy()
    runs = (q[:, 1:] != q[:, :-1]).any(-1).sum(1) + 1
    print(json.dumps({"phase": k, "ms": a.elapsed_time(b), "p50": float(np.median(h)),
                      "p90": float(np.percentile(h, 90)), "p99": float(np.percentile(h, 99)),
                      "max": int(h.max()), "capped": int((h >= 100).sum()), "n": n,
                      "runs_p50": float(np.median(runs)),
                      "runs_capped_p50": float(np.median(runs[h >= 100])) if (h >= 100).any() else None,
                      "runs_capped_p90": float(np.percentile(runs[h >= 100], 90)) if (h >= 100).any() else None,
                      "capped_runs_ge_64": int(((h >= 100) & (runs >= 64)).sum()),
                      # a wave's pass costs its heaviest lane: runs per lane of 8 lanes
                      "waves_cost_model": float(np.sum(np.max((h * np.ceil(runs / 8.0))[:n // 8 * 8]
                                                               .reshape(-1, 8), axis=1)))}), flush=True)
