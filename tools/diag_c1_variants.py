"""Diagnostic: the C1 two-iteration pipeline of tests/test_gpu_reconstruct2d.py
under a few variants; prints the second expectation's class histogram and
the reconstructed classes' correlation with the generating ones."""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import test_gpu_reconstruct2d as t  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402

DEV, T_, N1, PF1, K1 = t.DEV, t.T_, t.N1, t.PF1, t.K1


def run(snr=10.0, n=400, m_reco=4, fsc=None, ru_search=16, white=False, lp=None):
    imgs = t._class_images(K1, 81)
    cl = t._projectee2d(imgs)
    px = ops.PixelSet(N1, PF1, ru_search, 1, device=DEV)
    mS, nR, nT = ops.global_sample_sizes(100, mode=0)
    gset = [x.cpu().numpy() for x in ops.global_sample_set2d(nR, nT, 10.0, 83, DEV)]
    rng = np.random.default_rng(82)
    cls_true = rng.integers(0, K1, n)
    q, tr = gset[0], gset[1]
    th = np.arctan2(q[:, 1], q[:, 0])[rng.integers(0, len(q), n)]
    near = np.argsort(np.linalg.norm(tr, axis=1))[:40]
    tt = tr[near[rng.integers(0, len(near), n)]]
    attr = T_(synth.ctf_attrs(n, seed=84))
    def images(pxs, seed):
        c = ops.ctf(attr, pxs)
        P = torch.empty(n, pxs.n, dtype=torch.complex64, device=DEV)
        for l in range(n):
            P[l] = ops.project2d(cl[cls_true[l]].contiguous(),
                                 T_(np.array([[np.cos(th[l]), np.sin(th[l])]])), pxs)[0]
        d, s = synth.noisy_images(c * P * ops.trans_table(T_(tt), pxs), pxs.iSig, N1 // 2 + 1, snr=snr,
                                  seed=seed, white=white)
        return d, c, s
    dat, ctf, sig = images(px, 85)
    pxi = ops.PixelSet(N1, PF1, N1 // 2 - 2, 0, device=DEV)
    dati, ctfi, _ = images(pxi, 86)
    refs = cl
    out = []
    gen = t._centre_crop(imgs, N1)
    for it in range(2):
        e = ex.Expectation(refs, px, gset, n_phase=10, seed=9 + it, mode="2d")
        rot, trans, pR, pT, score, cls, nph = e.run(dat, ctf, sig)
        hist = np.bincount(cls.cpu().numpy(), minlength=K1)
        acc = float(np.mean(cls.cpu().numpy() == cls_true))
        qd, td = ex.draw_insert_samples(rot, trans, m_reco, seed=30 + it)
        nc = cls.view(n, 1).expand(n, m_reco).contiguous().to(torch.int32)
        hm = ops.HalfMap2D(N1 * PF1, K1, DEV)
        ops.insert2d(hm, dati, ctfi, qd[..., :2].contiguous(), td.contiguous(),
                     torch.zeros(n, 2, dtype=torch.float64, device=DEV),
                     torch.full((n,), 1.0 / m_reco, dtype=torch.float32, device=DEV), pxi, nc=nc)
        ops.prepare_tf2d(hm)
        o, its = ops.reconstruct2d(hm, N1, PF1, fsc=fsc)
        rec = o.cpu().numpy()
        if lp is not None:      # the references low-passed to shell lp (as a resolution limit)
            fy = np.fft.fftfreq(N1)[:, None] * N1
            fx = np.fft.fftfreq(N1)[None, :] * N1
            rec = np.fft.ifft2(np.fft.fft2(rec) * (np.hypot(fy, fx) <= lp)).real
        rec = np.fft.fftshift(rec, axes=(-2, -1))
        corr = [round(float(np.corrcoef(rec[k].ravel(), gen[k].ravel())[0, 1]), 3) for k in range(K1)]
        out.append((it, acc, hist.tolist(), corr, [round(float(rec[k].std() * N1 * PF1 / gen[k].std()), 3)
                                                   for k in range(K1)]))
        pad = np.zeros_like(imgs)
        oo = (N1 * PF1 - N1) // 2
        pad[:, oo:oo + N1, oo:oo + N1] = rec * (N1 * PF1)
        refs = t._projectee2d(pad)
    return out


for kw in ({"white": True}, {"white": True, "snr": 3.0}, {"white": True, "snr": 1.0},
           {"white": True, "ru_search": 24}, {"lp": 10}, {"lp": 12}):
    for row in run(**kw):
        print(kw if not isinstance(kw.get("fsc"), np.ndarray) else "fsc", row)
