"""f1, MODE_2D: thx_reconstruct2d (the 2D branches of Reconstructor::reconstruct,
src/Reconstructor.cpp:1136-1589) against the float64 restatement
(oracle/reconstruct.py reconstruct2d), and config C1 closing two iterations
on the GPU: expectation2d -> InsertI2D (thx_insert2d) -> prepareTF (2D
normalisation) -> reconstruct2d -> the class images as the next references ->
expectation2d again.  Tolerances: class images 1e-4 of max (as the 3D
solve); iterations per class equal."""
import numpy as np
import pytest
import torch

from oracle import reconstruct as orc_rc
from thunder_amd import expectation as ex
from thunder_amd import ops, synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def T_(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


@pytest.mark.parametrize("grid_corr,map_", [(True, False), (False, False), (True, True)])
def test_reconstruct2d_matches_restatement(grid_corr, map_):
    N, pf, nK = 64, 2, 3
    vdim = N * pf
    rng = np.random.default_rng(12)
    quad = orc_rc._ft_quad2(vdim).astype(np.float64)
    Fs, Ts = [], []
    for k in range(nK):
        X = np.fft.rfftn(rng.standard_normal((vdim, vdim)))
        T = (20.0 * (k + 1) / (1.0 + np.sqrt(quad))) * rng.uniform(0.8, 1.2, quad.shape)
        Fs.append(X * T)
        Ts.append(T)
    hm = ops.HalfMap2D(vdim, nK, DEV)
    hm.F.copy_(T_(np.stack(Fs).astype(np.complex64)))
    hm.T.copy_(T_(np.stack(Ts).astype(np.float32)))
    fsc = np.stack([np.linspace(0.99, 0.1 + 0.1 * k, N // 2 + 1) for k in range(nK)]) if map_ else None
    got, its = ops.reconstruct2d(hm, N, pf, grid_corr=grid_corr, fsc=fsc)
    got = got.cpu().numpy()
    for k in range(nK):
        ref, rit, _ = orc_rc.reconstruct2d(Fs[k].astype(np.complex64), Ts[k].astype(np.float32), N, pf,
                                           grid_corr=grid_corr, fsc=None if fsc is None else fsc[k])
        assert its[k] == rit
        assert np.max(np.abs(got[k] - ref)) <= 1e-4 * np.max(np.abs(ref)), k


def test_prepare_tf2d_normalises_each_class():
    vdim, nK = 64, 4
    rng = np.random.default_rng(2)
    hm = ops.HalfMap2D(vdim, nK, DEV)
    F = (rng.standard_normal((nK, vdim, vdim // 2 + 1)) +
         1j * rng.standard_normal((nK, vdim, vdim // 2 + 1))).astype(np.complex64)
    T = rng.uniform(0.5, 3.0, (nK, vdim, vdim // 2 + 1)).astype(np.float32)
    hm.F.copy_(T_(F))
    hm.T.copy_(T_(T))
    ops.prepare_tf2d(hm)
    sf = (1.0 / T[:, 0, 0]).astype(np.float32)[:, None, None]
    assert np.allclose(hm.T.cpu().numpy(), T * sf, rtol=1e-6)
    assert np.allclose(hm.F.cpu().numpy(), F * sf, rtol=1e-6)


# --------------------------------------------------- C1: two iterations
N1, PF1, K1 = 64, 2, 8


def _class_images(nK, seed):
    """[nK, vdim, vdim] real blob images centred in the padded box."""
    vdim = N1 * PF1
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[:vdim, :vdim] - vdim // 2
    out = np.zeros((nK, vdim, vdim))
    for k in range(nK):
        for _ in range(6):
            cx, cy = rng.uniform(-N1 / 3, N1 / 3, 2)
            w = rng.uniform(2, 5)
            out[k] += rng.uniform(0.5, 1.5) * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * w * w))
    return out


def _projectee2d(imgs):
    """Padded real images (centred) -> half-complex 2D projectees (as the tests' references)."""
    vdim = imgs.shape[-1]
    return T_(np.stack([np.fft.rfft2(np.fft.ifftshift(i)) / vdim for i in imgs]).astype(np.complex64))


def _centre_crop(padded, N):
    vdim = padded.shape[-1]
    o = (vdim - N) // 2
    return padded[..., o:o + N, o:o + N]


def test_c1_two_iterations_on_gpu():
    """Config C1 (box 64, 8 classes): expectation2d against the generating
    classes, the particles' samples inserted per class, the 2D normalisation
    and solve, the class images as the next references, a second
    expectation2d.  The reconstructed classes correlate > 0.9 with the
    generating ones and the second iteration keeps the class assignment."""
    imgs = _class_images(K1, 81)
    cl = _projectee2d(imgs)
    px = ops.PixelSet(N1, PF1, 16, 1, device=DEV)
    mS, nR, nT = ops.global_sample_sizes(100, mode=0)
    gset = [t.cpu().numpy() for t in ops.global_sample_set2d(nR, nT, 10.0, 83, DEV)]
    n = 400
    rng = np.random.default_rng(82)
    cls_true = rng.integers(0, K1, n)
    q, t = gset[0], gset[1]
    th = np.arctan2(q[:, 1], q[:, 0])[rng.integers(0, len(q), n)]
    near = np.argsort(np.linalg.norm(t, axis=1))[:40]
    tt = t[near[rng.integers(0, len(near), n)]]
    ctf = ops.ctf(T_(synth.ctf_attrs(n, seed=84)), px)
    P = torch.empty(n, px.n, dtype=torch.complex64, device=DEV)
    for l in range(n):
        P[l] = ops.project2d(cl[cls_true[l]].contiguous(), T_(np.array([[np.cos(th[l]), np.sin(th[l])]])),
                             px)[0]
    # white noise (one sigma^2 over the pixel set, as in a micrograph): the
    # high shells are noise-dominated, so the second expectation weighs the
    # reconstructed classes' noisy high shells by their real reliability
    # (per-shell SNR noise would trust them 10:1 and classify on the solve's
    # high-frequency residue -- tools/diag_c1_frc.py)
    dat, sig = synth.noisy_images(ctf * P * ops.trans_table(T_(tt), px), px.iSig, N1 // 2 + 1, snr=3.0,
                                  seed=85, white=True)
    # the full-resolution pixel set for the insert (rU = N / 2 - 2, the
    # reconstruction's maxRadius) and the images there
    pxi = ops.PixelSet(N1, PF1, N1 // 2 - 2, 0, device=DEV)
    ctfi = ops.ctf(T_(synth.ctf_attrs(n, seed=84)), pxi)
    Pi = torch.empty(n, pxi.n, dtype=torch.complex64, device=DEV)
    for l in range(n):
        Pi[l] = ops.project2d(cl[cls_true[l]].contiguous(),
                              T_(np.array([[np.cos(th[l]), np.sin(th[l])]])), pxi)[0]
    dati, _ = synth.noisy_images(ctfi * Pi * ops.trans_table(T_(tt), pxi), pxi.iSig, N1 // 2 + 1,
                                 snr=3.0, seed=86, white=True)
    refs = cl
    classes = []
    for it in range(2):
        e = ex.Expectation(refs, px, gset, n_phase=10, seed=9 + it, mode="2d")
        rot, trans, pR, pT, score, cls, nph = e.run(dat, ctf, sig)
        classes.append(cls.cpu().numpy())
        # Particle::rand samples of each image's final clouds, its drawn class
        m_reco = 4
        qd, td = ex.draw_insert_samples(rot, trans, m_reco, seed=30 + it)
        rot2 = qd[..., :2].contiguous()
        nc = cls.view(n, 1).expand(n, m_reco).contiguous().to(torch.int32)
        hm = ops.HalfMap2D(N1 * PF1, K1, DEV)
        ops.insert2d(hm, dati, ctfi, rot2, td.contiguous(),
                     torch.zeros(n, 2, dtype=torch.float64, device=DEV),
                     torch.full((n,), 1.0 / m_reco, dtype=torch.float32, device=DEV), pxi, nc=nc)
        ops.prepare_tf2d(hm)
        out, its = ops.reconstruct2d(hm, N1, PF1)
        rec = np.fft.fftshift(out.cpu().numpy(), axes=(-2, -1))       # centred N x N
        assert all(1 <= i <= 30 for i in its)
        gen = _centre_crop(imgs, N1)
        corr = [np.corrcoef(rec[k].ravel(), gen[k].ravel())[0, 1] for k in range(K1)]
        info = (it, its, [bool(np.isfinite(rec[k]).all()) for k in range(K1)],
                [float(np.nanstd(rec[k])) for k in range(K1)], np.bincount(cls.cpu().numpy(), minlength=K1))
        assert np.all(np.isfinite(corr)) and min(corr) > 0.9, (corr, info)
        # the next references: the reconstructed classes at the references'
        # scale -- the solve returns irfft2 of F / T (FFT::bw's 1 / size), i.e.
        # the generating images / vdim under _projectee2d's 1 / vdim
        pad = np.zeros_like(imgs)
        o = (N1 * PF1 - N1) // 2
        pad[:, o:o + N1, o:o + N1] = rec * (N1 * PF1)
        refs = _projectee2d(pad)
    assert np.mean(classes[0] == cls_true) >= 0.9
    assert np.mean(classes[1] == cls_true) >= 0.9
