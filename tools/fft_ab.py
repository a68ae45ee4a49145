#!/usr/bin/env python3
"""A/B of the 3D transforms of the reconstruction (thx_fft3d): hipFFT's 3D
plans (method 1) against the LDS column passes + batched 1D x transform
(method 2), forward and inverse, per vdim; one JSON line each."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from thunder_amd import ops  # noqa: E402
from thunder_amd._lib import check, lib  # noqa: E402

dev = torch.device("cuda", 0)
for vdim in (256, 512):
    rl = torch.randn(vdim, vdim, vdim, device=dev)
    C = torch.empty(vdim, vdim, vdim // 2 + 1, dtype=torch.complex64, device=dev)
    ws = ops.workspace(lib().thx_fft3d_workspace(vdim), dev)
    for method in (1, 2):
        for inv in (0, 1):
            f = lambda: check(lib().thx_fft3d(ops._ptr(C), ops._ptr(rl), vdim, inv, method,
                                              ops._ptr(ws), ws.numel(), None), "thx_fft3d")
            f()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                f()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / 5
            gb = 2 * (rl.numel() * 4 + C.numel() * 8) / 1e9
            print(json.dumps({"vdim": vdim, "method": ["", "hipfft3d", "columns"][method],
                              "dir": "c2r" if inv else "r2c", "ms": ms,
                              "GBps_2rw": gb / ms * 1e3}), flush=True)
