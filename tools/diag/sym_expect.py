"""Diagnostic: pose recovery on a C4 map with and without the symmetric search."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import symmetry as osym  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402

DEV = torch.device("cuda", 0)
T_ = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=DEV)


def err_mod(q, qt, Q):
    best = abs(float(q @ qt))
    for s in Q:
        best = max(best, abs(float(q @ osym.quat_mul(s, qt))))
    return np.degrees(2 * np.arccos(min(1.0, best)))


N, pf, sym = 64, 2, "C4"
R, Q = ops.symmetry(sym)
vol = synth.projectee(synth.blob_volume(N, n_blobs=int(os.environ.get("NB", 10)), seed=4, sym_R=R, device=DEV), pf)
px = ops.PixelSet(N, pf, int(os.environ.get("RU", 20)), 1, device=DEV)
rng = np.random.default_rng(6)
nImg = 96
qt = synth.uniform_quaternions(nImg, rng)
tt = rng.standard_normal((nImg, 2)) * 2
ctf = ops.ctf(T_(synth.ctf_attrs(nImg, seed=7)), px)
sig = ctf * ops.project3d(vol, ops.rotmat(T_(qt)), px) * ops.trans_table(T_(tt), px)
dat, sigRcp = synth.noisy_images(sig, px.iSig, N // 2 + 1, snr=20.0, seed=8)
# is the map symmetric?  projections at q and s q
p1 = ops.project3d(vol, ops.rotmat(T_(qt[:4])), px)
p2 = ops.project3d(vol, ops.rotmat(T_(np.stack([osym.quat_mul(Q[0], q) for q in qt[:4]]))), px)
print("proj sym rel diff", float((p1 - p2).abs().max() / p1.abs().max()))
for use_sym, nphase in ((None, 10), (sym, 10), (sym, 1), (None, 1)):
    mS, nR, nT = ops.global_sample_sizes(1500, n_sym_elem=len(Q) if use_sym else 0)
    gq, gt, gpR, gpT = ops.global_sample_set(nR, nT, 10.0, 5, DEV, sym=use_sym)
    gset = tuple(x.cpu().numpy() for x in (gq, gt, gpR, gpT))
    e = ex.Expectation(vol, px, gset, n_phase=nphase, seed=3, sym=use_sym)
    quat = e.run(dat, ctf, sigRcp)[0]
    mode = ex.cloud_mode(quat).cpu().numpy()
    err = np.array([err_mod(mode[l], qt[l], Q) for l in range(nImg)])
    print(use_sym, nphase, nR, "median", np.median(err), "frac>15", np.mean(err > 15))
