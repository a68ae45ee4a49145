#!/usr/bin/env python3
"""Time of the particle filter's resampling kernel (thx_pf_resample) at the
bench's shapes: the reseed's 2000 global rotations -> 125 particles (shared
prior, per-image marginals) and a phase's 125 -> 125, with and without the
support shuffle, 12 500 images.  One JSON line per case.
    python tools/resample_probe.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from thunder_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
n = 12500
rng = np.random.default_rng(5)
st = torch.cuda.current_stream(dev)
for nIn, nOut, shared in ((2000, 125, True), (125, 125, False), (9, 9, False)):
    u = torch.as_tensor((rng.exponential(1.0, (n, nIn)) ** 4).astype(np.float32), device=dev)
    w = torch.as_tensor(rng.uniform(0.5, 1.0, nIn if shared else (n, nIn)), device=dev)
    for shuffle in (True, False):
        f = lambda: ops.pf_resample(w, u, nOut, seed=3, shuffle=shuffle)
        f()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(5):
            f()
        b.record(st)
        torch.cuda.synchronize()
        print(json.dumps({"lib": os.path.basename(os.environ.get("THX_LIB", "prod")), "nIn": nIn,
                          "nOut": nOut, "shuffle": shuffle, "ms": round(a.elapsed_time(b) / 5, 4)}),
              flush=True)
