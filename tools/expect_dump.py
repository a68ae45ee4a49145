#!/usr/bin/env python3
"""Every output of the expectation driver (quat, trans, pR, pT, score, cls,
nPhase) on a reduced C3 workload -- box 256, rU 24, the 2000 x 151 global
set, 512 images, 1 / 3 / 10 phases, fixed seeds -- saved as .npy under DIR, to
compare two libraries bit for bit (tools/cmp_dump.py).
    python tools/expect_dump.py DIR"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from thunder_amd import expectation as ex, ops, synth  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
dev = torch.device("cuda", 0)
n = 512
vol = synth.projectee(synth.blob_volume(256, seed=1, device=dev), 2)
_, nR, nT = ops.global_sample_sizes(2000)
gset = tuple(x.cpu().numpy() for x in ops.global_sample_set(nR, nT, 10.0, 2, dev))
px, dat, ctf, sig, _, _ = bench.make_stack(256, 2, 24, 1, n, dev, seed=5, vol=vol)
names = ("quat", "trans", "pR", "pT", "score", "cls", "nphase")
for k in (1, 3, 10):
    for conv in (False, True):
        e = ex.Expectation(vol, px, gset, n_phase=k, seed=7, converge=conv)
        res = e.run(dat, ctf, sig)
        for name, x in zip(names, res):
            np.save(os.path.join(out, f"k{k}_c{int(conv)}_{name}.npy"), x.cpu().numpy())
print("ok")
