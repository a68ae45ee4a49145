#!/usr/bin/env python3
"""The staged perturbation mean against a library with the one-launch
k_pf_mean (thunder_amd/ab/lib_cv.so, loaded beside the product library):
the same clouds, bitwise comparison of means and iteration counts, and the
staged mean run twice.   python tools/mean_stage_check.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from thunder_amd import expectation as ex, ops, synth  # noqa: E402
from thunder_amd._lib import lib  # noqa: E402

dev = torch.device("cuda", 0)
n = 4096
vol = synth.projectee(synth.blob_volume(256, seed=1, device=dev), 2)
_, nR, nT = ops.global_sample_sizes(2000)
gset = tuple(x.cpu().numpy() for x in ops.global_sample_set(nR, nT, 10.0, 2, dev))
px, dat, ctf, sig, _, _ = bench.make_stack(256, 2, 24, 1, n, dev, seed=5, vol=vol)
old = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                               "thunder_amd", "ab", "lib_cv.so"))
st = torch.cuda.current_stream(dev)
for k in (1, 3):
    quat = ex.Expectation(vol, px, gset, n_phase=k, seed=7).run(dat, ctf, sig)[0].contiguous()
    outs = []
    for L in (lib(), lib(), old):
        mq = torch.full((n, 4), float("nan"), dtype=torch.float64, device=dev)
        it = torch.full((n,), -1, dtype=torch.int32, device=dev)
        assert L.thx_pf_acg_mean(n, quat.shape[1], ctypes.c_void_p(quat.data_ptr()), 100,
                                 ctypes.c_void_p(mq.data_ptr()), ctypes.c_void_p(it.data_ptr()),
                                 ctypes.c_void_p(st.cuda_stream)) == 0
        torch.cuda.synchronize()
        outs.append((mq.cpu().numpy(), it.cpu().numpy()))
    (a, ia), (b, ib), (c, ic) = outs
    bad = np.nonzero(~np.all(a == c, axis=1))[0]
    print(json.dumps({"phase": k, "staged_repeat_identical": bool(np.array_equal(a, b) and np.array_equal(ia, ib)),
                      "staged_vs_one_launch_identical": bool(np.array_equal(a, c) and np.array_equal(ia, ic)),
                      "n_differ": int(len(bad)), "iters_of_differing": ia[bad][:10].tolist(),
                      "old_iters_of_differing": ic[bad][:10].tolist(),
                      "max_abs_diff": float(np.nanmax(np.abs(a - c))) if len(bad) else 0.0}), flush=True)
