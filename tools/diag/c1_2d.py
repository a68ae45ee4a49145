"""Diagnostic: the C1 two-iteration test's first iteration, with class counts."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import test_gpu_reconstruct2d as t  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402

DEV, T_, N1, PF1, K1 = t.DEV, t.T_, t.N1, t.PF1, t.K1
imgs = t._class_images(K1, 81)
cl = t._projectee2d(imgs)
px = ops.PixelSet(N1, PF1, 16, 1, device=DEV)
mS, nR, nT = ops.global_sample_sizes(100, mode=0)
gset = [x.cpu().numpy() for x in ops.global_sample_set2d(nR, nT, 10.0, 83, DEV)]
n = 400
rng = np.random.default_rng(82)
cls_true = rng.integers(0, K1, n)
q, tr = gset[0], gset[1]
th = np.arctan2(q[:, 1], q[:, 0])[rng.integers(0, len(q), n)]
near = np.argsort(np.linalg.norm(tr, axis=1))[:40]
tt = tr[near[rng.integers(0, len(near), n)]]
ctf = ops.ctf(T_(synth.ctf_attrs(n, seed=84)), px)
P = torch.empty(n, px.n, dtype=torch.complex64, device=DEV)
for l in range(n):
    P[l] = ops.project2d(cl[cls_true[l]].contiguous(), T_(np.array([[np.cos(th[l]), np.sin(th[l])]])), px)[0]
dat, sig = synth.noisy_images(ctf * P * ops.trans_table(T_(tt), px), px.iSig, N1 // 2 + 1, snr=10.0, seed=85)
e = ex.Expectation(cl, px, gset, n_phase=10, seed=9, mode="2d")
rot, trans, pR, pT, score, cls, nph = e.run(dat, ctf, sig)
c = cls.cpu().numpy()
print("rot", tuple(rot.shape), "trans", tuple(trans.shape), "cls", tuple(cls.shape), cls.dtype)
print("true hist", np.bincount(cls_true, minlength=K1))
print("got hist ", np.bincount(c, minlength=K1))
print("acc", np.mean(c == cls_true))
qd, td = ex.draw_insert_samples(rot, trans, 4, seed=30)
print("qd", tuple(qd.shape), "td", tuple(td.shape))
print("rot[0,:3]", rot[0, :3].cpu().numpy())
print("qd[0]", qd[0].cpu().numpy())
print("true th0", th[0], np.cos(th[0]), np.sin(th[0]), "tt0", tt[0])
# the test's insert -> prepare -> reconstruct, per-class statistics
pxi = ops.PixelSet(N1, PF1, N1 // 2 - 2, 0, device=DEV)
ctfi = ops.ctf(T_(synth.ctf_attrs(n, seed=84)), pxi)
Pi = torch.empty(n, pxi.n, dtype=torch.complex64, device=DEV)
for l in range(n):
    Pi[l] = ops.project2d(cl[cls_true[l]].contiguous(), T_(np.array([[np.cos(th[l]), np.sin(th[l])]])), pxi)[0]
dati, _ = synth.noisy_images(ctfi * Pi * ops.trans_table(T_(tt), pxi), pxi.iSig, N1 // 2 + 1, snr=10.0, seed=86)
print("dati finite", bool(torch.isfinite(dati).all()), "ctfi finite", bool(torch.isfinite(ctfi).all()))
rot2 = qd[..., :2].contiguous()
nc = cls.view(n, 1).expand(n, 4).contiguous().to(torch.int32)
hm = ops.HalfMap2D(N1 * PF1, K1, DEV)
ops.insert2d(hm, dati, ctfi, rot2, td.contiguous(), torch.zeros(n, 2, dtype=torch.float64, device=DEV),
             torch.full((n,), 0.25, dtype=torch.float32, device=DEV), pxi, nc=nc)
F = hm.F.cpu().numpy(); T = hm.T.cpu().numpy()
for k in range(K1):
    print("class", k, "T00", T[k, 0, 0], "Tsum", T[k].sum(), "Ffinite", np.isfinite(F[k]).all(), "Tfinite", np.isfinite(T[k]).all(),
          "counter", int(hm.counter[k]), "T<0", int((T[k] < 0).sum()))
ops.prepare_tf2d(hm)
T = hm.T.cpu().numpy()
print("after prepare: finite per class", [bool(np.isfinite(T[k]).all()) for k in range(K1)])
out, its = ops.reconstruct2d(hm, N1, PF1)
o = out.cpu().numpy()
print("its", its, "finite per class", [bool(np.isfinite(o[k]).all()) for k in range(K1)], "std", [float(o[k].std()) for k in range(K1)])
