#!/usr/bin/env python3
"""Every output of thx_pf_resample (ancestors, priors, iMax, perm, u0) for a
set of support sizes and seeds, saved as .npy under DIR, to compare two
libraries bit for bit (tools/cmp_dump.py).
    python tools/resample_dump.py DIR"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from thunder_amd import ops  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
dev = torch.device("cuda", 0)
for nIn, nOut in ((9, 9), (33, 20), (64, 64), (125, 125), (128, 125), (200, 125), (257, 100),
                  (1000, 125), (2000, 125), (2048, 125)):
    rng = np.random.default_rng(nIn)
    n = 300
    u = torch.as_tensor((rng.exponential(1.0, (n, nIn)) ** 4).astype(np.float32), device=dev)
    w = torch.as_tensor(rng.uniform(0.5, 1.0, nIn), device=dev)
    for seed in (3, 17):
        res = ops.pf_resample(w, u, nOut, seed=seed, shuffle=True)
        for name, x in zip(("anc", "wout", "imax", "perm", "u0"), res):
            np.save(os.path.join(out, f"n{nIn}_s{seed}_{name}.npy"), x.cpu().numpy())
print("ok")
