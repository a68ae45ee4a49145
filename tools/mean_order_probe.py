#!/usr/bin/env python3
"""Does the order of the images in k_pf_mean's waves matter?  A wave holds
GROUP = 8 images and runs until its slowest fixed point ends; the capped
images (acgIters iterations) are spread over most waves.  On the bench's
particle clouds after k phases (as tools/pf_iters.py makes them), times
thx_pf_acg_mean on the clouds in index order and sorted by their own
iteration count (longest first, an upper bound for any predicted order).
    python tools/mean_order_probe.py     (PF_ITERS_N images, default 12500)"""
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
n = int(os.environ.get("PF_ITERS_N", "12500"))
vol = synth.projectee(synth.blob_volume(256, seed=1, device=dev), 2)
_, nR, nT = ops.global_sample_sizes(2000)
gset = tuple(x.cpu().numpy() for x in ops.global_sample_set(nR, nT, 10.0, 2, dev))
px, dat, ctf, sig, _, _ = bench.make_stack(256, 2, 24, 1, n, dev, seed=5, vol=vol)
st = torch.cuda.current_stream(dev)


def mean(q, reps=5):
    mq = torch.empty(n, 4, dtype=torch.float64, device=dev)
    it = torch.empty(n, dtype=torch.int32, device=dev)
    call = lambda: check(lib().thx_pf_acg_mean(n, q.shape[1], ops._ptr(q), 100, ops._ptr(mq),
                                               ops._ptr(it), ctypes.c_void_p(st.cuda_stream)),
                         "thx_pf_acg_mean")
    call()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        call()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps, it.cpu().numpy(), mq


prev = None
for k in range(1, 11):
    e = ex.Expectation(vol, px, gset, n_phase=k, seed=7)
    quat = e.run(dat, ctf, sig)[0].contiguous()
    ms, it, mq = mean(quat)
    order = np.argsort(-it, kind="stable")
    qs = quat[torch.as_tensor(order, device=dev)].contiguous()
    ms_sorted, it_s, mq_s = mean(qs)
    same = bool(torch.equal(mq_s, mq[torch.as_tensor(order, device=dev)]))
    row = {"phase": k, "n": n, "ms_index_order": round(ms, 4), "ms_sorted_by_iters": round(ms_sorted, 4),
           "capped": int((it >= 100).sum()), "p50": float(np.median(it)), "means_identical": same}
    if prev is not None:    # the previous phase's counts as the predictor
        po = np.argsort(-prev, kind="stable")
        ms_pred, _, _ = mean(quat[torch.as_tensor(po, device=dev)].contiguous())
        row["ms_sorted_by_prev_phase_iters"] = round(ms_pred, 4)
        row["capped_also_capped_before"] = int(((it >= 100) & (prev >= 100)).sum())
    prev = it
    print(json.dumps(row), flush=True)
