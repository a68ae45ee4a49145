"""Diagnostic: global-scan algorithms 1-3 against the direct algorithm 0 at
the metric configuration (baseline and argmax of wR per image)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_stack  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402

DEV = torch.device("cuda", 0)
N, pf = 256, 2
vol = synth.projectee(synth.blob_volume(N, seed=1, device=DEV), pf)
px, dat, ctf, sig, qtrue, ttrue = make_stack(N, pf, 24, 1, 64, DEV, seed=9, vol=vol)
for nr, nt in ((64, 30), (64, 60), (64, 100), (64, 151), (2000, 151)):
    q, t, pR, pT = synth.global_sample_set(nr, seed=2)
    t, pT = t[:nt], pT[:nt] / pT[:nt].sum()
    rotP = ops.project3d(vol, ops.rotmat(torch.as_tensor(q, device=DEV)), px)
    traP = ops.trans_table(torch.as_tensor(np.ascontiguousarray(t), device=DEV), px)
    pRd, pTd = torch.as_tensor(pR, device=DEV), torch.as_tensor(pT, device=DEV)
    res = {a: [x.cpu().numpy() for x in ops.global_scan(rotP, traP, dat, ctf, sig, pRd, pTd, algo=a)]
           for a in (0, 1, 2, 3)}
    for a in (1, 2, 3):
        d = np.abs(res[a][3] - res[0][3])
        print(nr, nt, a, "base maxdiff %.3g" % d.max(), "imgs>1e-3:", np.nonzero(d > 1e-3)[0][:12])
