#!/usr/bin/env python3
"""Determinism / library comparison of the expectation driver: a small
global search (1024 images, 4 phases) run twice in this process with the
library THX_LIB names; prints whether the two runs agree bitwise and saves
the first run's outputs to OUT.npz for a comparison across libraries.
    THX_LIB=... python tools/driver_det_check.py OUT.npz"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from thunder_amd import expectation as ex, ops, synth  # noqa: E402

dev = torch.device("cuda", 0)
vol = synth.projectee(synth.blob_volume(256, seed=1, device=dev), 2)
_, nR, nT = ops.global_sample_sizes(2000)
gset = tuple(x.cpu().numpy() for x in ops.global_sample_set(nR, nT, 10.0, 2, dev))
px, dat, ctf, sig, _, _ = bench.make_stack(256, 2, 24, 1, 1024, dev, seed=77, vol=vol)
runs = []
for _ in range(2):
    e = ex.Expectation(vol, px, gset, n_phase=4, seed=13)
    runs.append([x.clone().cpu().numpy() for x in e.run(dat, ctf, sig)])
same = all(np.array_equal(a, b) for a, b in zip(*runs))
names = ["quat", "trans", "pR", "pT", "score", "cls", "nph"]
np.savez(sys.argv[1], **dict(zip(names, runs[0])))
if len(sys.argv) > 2 and os.path.exists(sys.argv[2]):
    ref = np.load(sys.argv[2])
    diff = {k: int(np.sum(~np.isclose(ref[k], v, rtol=0, atol=0)) if v.dtype.kind == "f"
                   else np.sum(ref[k] != v)) for k, v in zip(names, runs[0])}
else:
    diff = None
print(json.dumps({"lib": os.path.basename(os.environ.get("THX_LIB", "prod")), "repeat_identical": same,
                  "entries_differing_from_ref": diff}), flush=True)
