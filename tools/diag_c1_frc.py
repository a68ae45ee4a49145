"""Diagnostic: the C1 pipeline's first reconstruction against the generating
classes, per Fourier shell (FRC, power ratio, phase slope = residual shift),
and the second expectation under swapped references (true classes with the
second seed, reconstructed ones, reconstructed ones low-passed)."""
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
n = 400
imgs = t._class_images(K1, 81)
cl = t._projectee2d(imgs)
px = ops.PixelSet(N1, PF1, 16, 1, device=DEV)
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
    d, s = synth.noisy_images(c * P * ops.trans_table(T_(tt), pxs), pxs.iSig, N1 // 2 + 1, snr=10.0,
                              seed=seed)
    return d, c, s


dat, ctf, sig = images(px, 85)
pxi = ops.PixelSet(N1, PF1, N1 // 2 - 2, 0, device=DEV)
dati, ctfi, _ = images(pxi, 86)


def expect(refs, seed):
    e = ex.Expectation(refs, px, gset, n_phase=10, seed=seed, mode="2d")
    rot, trans, pR, pT, score, cls, nph = e.run(dat, ctf, sig)
    c = cls.cpu().numpy()
    return rot, trans, c, float(np.mean(c == cls_true)), np.bincount(c, minlength=K1).tolist()


rot, trans, cls0, acc0, h0 = expect(cl, 9)
print("it0 true refs seed 9", acc0, h0)
print("it1 true refs seed 10", expect(cl, 10)[3:])
m_reco = 4
qd, td = ex.draw_insert_samples(rot, trans, m_reco, seed=30)
nc = torch.as_tensor(cls0, device=DEV).view(n, 1).expand(n, m_reco).contiguous().to(torch.int32)
hm = ops.HalfMap2D(N1 * PF1, K1, DEV)
ops.insert2d(hm, dati, ctfi, qd[..., :2].contiguous(), td.contiguous(),
             torch.zeros(n, 2, dtype=torch.float64, device=DEV),
             torch.full((n,), 1.0 / m_reco, dtype=torch.float32, device=DEV), pxi, nc=nc)
ops.prepare_tf2d(hm)
T00 = hm.T[:, 0, :4].cpu().numpy()
o, its = ops.reconstruct2d(hm, N1, PF1)
rec = np.fft.fftshift(o.cpu().numpy(), axes=(-2, -1))
gen = t._centre_crop(imgs, N1)
print("its", its, "T row0", np.round(T00, 3).tolist())
# shells on the N x N crops
fy = np.fft.fftfreq(N1)[:, None] * N1
fx = np.fft.rfftfreq(N1)[None, :] * N1
shell = np.rint(np.sqrt(fy ** 2 + fx ** 2)).astype(int)
for k in range(K1):
    A = np.fft.rfft2(np.fft.ifftshift(rec[k]))
    B = np.fft.rfft2(np.fft.ifftshift(gen[k]))
    frc, pr, ph = [], [], []
    for s in (2, 4, 8, 12, 16, 20, 24, 28):
        m = shell == s
        num = np.sum(A[m] * np.conj(B[m]))
        frc.append(round(float(num.real / np.sqrt(np.sum(abs(A[m]) ** 2) * np.sum(abs(B[m]) ** 2))), 3))
        pr.append(round(float(np.sqrt(np.sum(abs(A[m]) ** 2) / np.sum(abs(B[m]) ** 2)) * N1 * PF1), 3))
        ph.append(round(float(np.angle(num)), 3))
    # residual shift from the cross power peak
    xc = np.fft.irfft2(A * np.conj(B), s=(N1, N1))
    iy, ix = np.unravel_index(np.argmax(xc), xc.shape)
    print("class", k, "frc", frc, "amp", pr, "phase", ph, "peak", (int(iy), int(ix)))
pad = np.zeros_like(imgs)
oo = (N1 * PF1 - N1) // 2
pad[:, oo:oo + N1, oo:oo + N1] = rec * (N1 * PF1)
refs = t._projectee2d(pad)
print("it1 rec refs seed 10", expect(refs, 10)[3:])
print("it1 rec refs seed 9", expect(refs, 9)[3:])
# true refs cropped to N and band-limited like the solve
padg = np.zeros_like(imgs)
padg[:, oo:oo + N1, oo:oo + N1] = gen
print("it1 cropped true refs seed 10", expect(t._projectee2d(padg), 10)[3:])
# the reference amplitudes against the true ones on the search pixel set
rp = ops.project2d(refs[0].contiguous(), T_(np.array([[1.0, 0.0]])), px)[0].cpu().numpy()
tp = ops.project2d(cl[0].contiguous(), T_(np.array([[1.0, 0.0]])), px)[0].cpu().numpy()
print("px ref/true power", float(np.sum(abs(rp) ** 2) / np.sum(abs(tp) ** 2)),
      "corr", float(abs(np.vdot(rp, tp)) / np.linalg.norm(rp) / np.linalg.norm(tp)))
