"""f1 on the GPU: thx_reconstruct (Reconstructor::reconstruct with hipFFT)
against the float64 restatement (oracle/reconstruct.py), and the north-star
parity chain end to end -- insert of two half-stacks (GPU vs the C
restatement), reconstruction of both half-maps, FSC of the reconstructed maps
(FSC, src/Functions/Spectrum.cpp:302-337) within 1e-4."""
import numpy as np
import pytest
import torch

from oracle import reconstruct as orc_rc
from stacks import small_stack
from thunder_amd import ops, synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def T_(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


def _halfmap(F, T):
    hm = ops.HalfMap(F.shape[0], DEV)
    hm.F.copy_(T_(F.astype(np.complex64)))
    hm.T.copy_(T_(T.astype(np.float32)))
    return hm


@pytest.mark.parametrize("grid_corr,map_", [(True, False), (False, False), (True, True)])
def test_reconstruct_matches_restatement(grid_corr, map_):
    N, pf = 32, 2
    vdim = N * pf
    rng = np.random.default_rng(11)
    vol = synth.projectee(synth.blob_volume(N, n_blobs=6, seed=3), pf).numpy()
    # T: a smooth positive sampling density like an insert's, F = T x the projectee
    quad = orc_rc._ft_quad(vdim).astype(np.float64)
    T = (50.0 / (1.0 + np.sqrt(quad))) * rng.uniform(0.8, 1.2, quad.shape)
    F = vol.astype(np.complex128) * T
    fsc = np.linspace(0.99, 0.2, N // 2 + 1) if map_ else None
    hm = _halfmap(F, T)
    got, gft, it, diffs = ops.reconstruct(hm, N, pf, grid_corr=grid_corr, fsc=fsc)
    ref, rit, rdiffs = orc_rc.reconstruct(F.astype(np.complex64), T.astype(np.float32), N, pf,
                                          grid_corr=grid_corr, fsc=fsc)
    got = got.cpu().numpy()
    assert it == rit
    if grid_corr:
        assert np.allclose(diffs, rdiffs, rtol=1e-3, atol=1e-5)
    assert np.max(np.abs(got - ref)) <= 1e-4 * np.max(np.abs(ref))
    # the map's transform for the FSC
    assert np.allclose(gft.cpu().numpy(), np.fft.rfftn(got), atol=1e-3 * np.abs(np.fft.rfftn(got)).max())


def test_halfmap_fsc_end_to_end(orc):
    """Two half-stacks -> insert -> reconstruct -> FSC: GPU (tiled insert,
    thx_reconstruct, thx_fsc) against the restatement (orc.insert_batch,
    oracle/reconstruct.py, orc.fsc) -- the north-star 'reconstructed half-map
    FSC within 1e-4' on a seeded synthetic stack."""
    s = small_stack(orc, N=32, nImg=4, nR=4, nT=3, seed=21, snr=2.0)
    N, pf, vdim = s["N"], s["pf"], s["vdim"]
    # full-resolution pixel set for the insert (rU = N/2 - 2, Reconstructor's maxRadius)
    pxh = orc.pixel_set(N, pf, N // 2 - 2, 0)
    px = ops.PixelSet(N, pf, N // 2 - 2, 0, device=DEV)
    rng = np.random.default_rng(22)
    nImg, mReco = 600, 8     # 300 images per half: every shell well sampled
    # images at random poses (recompute at the full-resolution pixel set)
    qt = synth.uniform_quaternions(nImg, rng)
    dat = np.stack([orc.project3d(s["vol"], vdim, pf, orc.rotate3d(q), pxh) for q in qt])
    dat = (dat + 0.05 * (rng.standard_normal(dat.shape) + 1j * rng.standard_normal(dat.shape))
           ).astype(np.complex64)
    ctf = np.ones((nImg, pxh.n), np.float32)
    quat = synth.clustered_quaternions(nImg, mReco, 1.0, rng)
    quat[:, 0] = qt
    trans = rng.standard_normal((nImg, mReco, 2)) * 0.3
    off = np.zeros((nImg, 2))
    w = np.full(nImg, 1.0 / mReco, np.float32)
    maps_g, maps_r = [], []
    for h in (0, 1):
        sel = np.arange(h, nImg, 2)
        hm = ops.HalfMap(vdim, DEV)
        ops.insert3d(hm, T_(dat[sel]), T_(ctf[sel]), T_(quat[sel]), T_(trans[sel]), T_(off[sel]),
                     T_(w[sel]), px)
        F, Tm, O, cnt = orc.insert_batch(vdim, pf, dat[sel], ctf[sel], quat[sel], trans[sel],
                                         off[sel], w[sel], pxh, N)
        F = F.reshape(vdim, vdim, vdim // 2 + 1)
        Tm = Tm.reshape(vdim, vdim, vdim // 2 + 1)
        _, gft, it, _ = ops.reconstruct(hm, N, pf)
        ref, rit, _ = orc_rc.reconstruct(F, Tm, N, pf)
        maps_g.append(gft)
        maps_r.append(np.fft.rfftn(ref).astype(np.complex64))
    got = ops.fsc(maps_g[0], maps_g[1], N // 2).cpu().numpy()
    ref = orc.fsc(maps_r[0], maps_r[1], N, N // 2)
    assert np.all(np.isfinite(got)) and got[2] > 0.5
    # relative to the FSC value, on the shells the half-maps cover
    rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-3)
    assert np.max(rel[1:]) < 1e-4, rel


@pytest.mark.parametrize("vdim", [64, 128, 512])
def test_fft3d_column_passes_match_numpy_and_hipfft(vdim):
    """thx_fft3d: the LDS column passes (method 2) against numpy's rfftn /
    irfftn (float64) and against hipFFT's 3D plans (method 1) on the same
    input, both directions (FFT::fw / FFT::bw conventions: unnormalised)."""
    import ctypes
    from thunder_amd._lib import check, lib
    rng = np.random.default_rng(vdim)
    x = rng.standard_normal((vdim, vdim, vdim)).astype(np.float32)
    X = np.fft.rfftn(x.astype(np.float64)) if vdim <= 128 else None
    ws = ops.workspace(lib().thx_fft3d_workspace(vdim), DEV)
    out = {}
    for method in (1, 2):
        rl = torch.as_tensor(x, device=DEV).contiguous()
        C = torch.empty(vdim, vdim, vdim // 2 + 1, dtype=torch.complex64, device=DEV)
        check(lib().thx_fft3d(ops._ptr(C), ops._ptr(rl), vdim, 0, method, ops._ptr(ws), ws.numel(),
                              None), "thx_fft3d")
        out[(method, "fw")] = C.cpu().numpy()
        back = torch.empty_like(rl)
        check(lib().thx_fft3d(ops._ptr(C), ops._ptr(back), vdim, 1, method, ops._ptr(ws), ws.numel(),
                              None), "thx_fft3d")
        out[(method, "bw")] = back.cpu().numpy()
    scale = np.abs(out[(1, "fw")]).max()
    assert np.max(np.abs(out[(2, "fw")] - out[(1, "fw")])) <= 2e-6 * scale
    if X is not None:
        assert np.max(np.abs(out[(2, "fw")] - X)) <= 2e-6 * np.abs(X).max()
    # bw(fw(x)) = vdim^3 x
    n3 = float(vdim) ** 3
    for m in (1, 2):
        assert np.max(np.abs(out[(m, "bw")] / n3 - x)) <= 2e-5 * np.abs(x).max()
    assert np.max(np.abs(out[(2, "bw")] - out[(1, "bw")])) <= 2e-6 * np.abs(out[(1, "bw")]).max()


def _reconstruct_f64_torch(F, T, N, pf, a=1.9, alpha=15.0):
    """oracle/reconstruct.py's reconstruct (grid correction, no MAP) restated
    line for line in float64 torch on the GPU, so the restatement runs at the
    bench's 512^3 padded box in seconds (torch's double-precision FFTs; the
    kernel table from the oracle's MKB closed forms)."""
    vdim = pf * N
    dev = F.device
    maxR = N // 2 - int(np.ceil(a))
    i = torch.arange(vdim // 2 + 1, device=dev, dtype=torch.float64)
    j = torch.fft.fftfreq(vdim, 1.0 / vdim, device=dev, dtype=torch.float64)
    quad = j[:, None, None] ** 2 + j[None, :, None] ** 2 + i[None, None, :] ** 2
    inside = quad < (maxR * pf) ** 2
    del quad
    T = torch.clamp(T.double(), min=1e-25)
    W = inside.double()
    tab = torch.as_tensor(orc_rc.mkb_rl_r2(np.arange(orc_rc.TAB_N + 1) * 1e-5, a, alpha)
                          .astype(np.float32).astype(np.float64), device=dev)
    nf = float(orc_rc.mkb_rl_r2(np.array([0.0]), a, alpha)[0])
    c = torch.fft.fftfreq(vdim, 1.0 / vdim, device=dev, dtype=torch.float64)
    rq = c[:, None, None] ** 2 + c[None, :, None] ** 2 + c[None, None, :] ** 2
    idx = torch.clamp(torch.round((rq / float(vdim * vdim)) / 1e-5).long(), max=orc_rc.TAB_N)
    kern = tab[idx] / nf
    del rq, idx
    diff_prev = diff = float(np.finfo(np.float32).max)
    n_no, m = 0, 0
    for m in range(30):
        C = T * W
        cr = torch.fft.irfftn(C.to(torch.complex128), s=(vdim, vdim, vdim)) * kern
        C = torch.fft.rfftn(cr)
        del cr
        a_ = C.abs()
        del C
        W = torch.where(inside, W / torch.clamp(a_, min=1e-6), W)
        diff_prev, diff = diff, float((a_[inside] - 1).abs().max())
        del a_
        n_no = n_no + 1 if diff > diff_prev * 0.95 else 0
        if diff < 1e-2 or (m >= 10 and n_no == 2):
            m += 1
            break
    else:
        m = 30
    pad = torch.where(inside, F.to(torch.complex128) * W, torch.zeros((), dtype=torch.complex128,
                                                                        device=dev))
    rl = torch.fft.irfftn(pad, s=(vdim, vdim, vdim))
    del pad
    cN = torch.fft.fftfreq(N, 1.0 / N, device=dev).long() % vdim
    box = rl[cN][:, cN][:, :, cN]
    cc = torch.fft.fftfreq(N, 1.0 / N, device=dev, dtype=torch.float64)
    r = torch.sqrt(cc[:, None, None] ** 2 + cc[None, :, None] ** 2 + cc[None, None, :] ** 2) / vdim
    x = np.pi * r
    j0 = torch.where(x == 0, torch.ones_like(x), torch.sin(x) / torch.where(x == 0, torch.ones_like(x), x))
    return (box / (j0 * j0)).cpu().numpy(), m


def test_reconstruct_at_the_bench_box_matches_f64():
    """The bench's solve (box 256, 512^3 padded -- the even half-grid
    balancing) against the float64 restatement at the same size: map within
    1e-4 of its maximum, the same iteration count."""
    N, pf = 256, 2
    vdim = N * pf
    vol = synth.projectee(synth.blob_volume(N, n_blobs=12, seed=3, device=DEV), pf)
    i = torch.arange(vdim // 2 + 1, device=DEV, dtype=torch.float32)
    j = torch.fft.fftfreq(vdim, 1.0 / vdim, device=DEV).float()
    quad = j[:, None, None] ** 2 + j[None, :, None] ** 2 + i[None, None, :] ** 2
    g = torch.Generator(device=DEV).manual_seed(5)
    T = (50.0 / (1.0 + quad.sqrt())) * (0.8 + 0.4 * torch.rand(quad.shape, generator=g, device=DEV))
    del quad
    F = vol * T
    del vol
    ref, rit = _reconstruct_f64_torch(F, T, N, pf)
    hm = ops.HalfMap(vdim, DEV)
    hm.F.copy_(F)
    hm.T.copy_(T)
    del F, T
    got, _, it, _ = ops.reconstruct(hm, N, pf, want_ft=False)
    got = got.cpu().numpy()
    assert it == rit
    assert np.max(np.abs(got - ref)) <= 1e-4 * np.max(np.abs(ref))
