"""The reconstruction half of the drop-in (Interface.h:320-528 through the
C-ABI adapters of thunder_amd/csrc/recon_iface.hip), called with host arrays
through ctypes exactly as the INTEGRATION.md forwards call them.

Reconstructor::reconstructG (src/Reconstructor.cpp:1835-2346) is replayed
step by step -- ExposePT (MAP), the split-step balancing AllocDevicePoint /
HostDeviceInit / {ExposeC, host backward FFT, ExposeForConvC, host forward
FFT, ExposeWC} / FreeDevHostPoint with the reference's stopping rule,
ExposePFW, the host backward FFT and VOL_EXTRACT_RL, ExposeCorrF -- with
numpy standing in for THUNDER's FFTW calls (forward unnormalised, backward
scaled by 1 / size, src/FFT.cpp:362-370), and the map is held against the
float64 restatement of Reconstructor::reconstruct (oracle/reconstruct.py) at
1e-4 of its maximum, iterations equal; likewise the 2D branch
(ExposePT2D, ExposeWT2D, ExposePF2D, IMG_EXTRACT_RL, ExposeCorrF2D) against
reconstruct2d.  PrepareTF against oracle/symmetry.py's prepare_tf; TranslateI
/ 2D, ReMask and GCTFinit against their closed forms and restatements."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import preprocess as opp
from oracle import reconstruct as orc_rc
from oracle import symmetry as osym
from thunder_amd import ops, synth
from thunder_amd._lib import check, lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
GPU = 0
A, ALPHA = 1.9, 15.0
TAB_N = 100000


def P(a):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def _kernel_table():
    """_kernelRL (MKB_RL_R2 on [0, 1], 1e5 steps, src/Reconstructor.cpp:77-88)
    and nf = MKB_RL(0) (:1939-1945), as float32 like RFLOAT."""
    tab = orc_rc.mkb_rl_r2(np.arange(TAB_N + 1) * 1e-5, A, ALPHA).astype(np.float32)
    nf = float(orc_rc.mkb_rl_r2(np.array([0.0]), A, ALPHA)[0])
    return tab, np.float32(1e-5), np.float32(nf)


def _tik_table(dim, padSize, nd):
    """mkbRL of reconstructG with the trilinear kernel: TIK_RL(NORM(i, j[, k]) / padSize)
    over [0, dim/2]^nd (src/Reconstructor.cpp:2194-2212, 2291-2310)."""
    h = np.arange(dim // 2 + 1, dtype=np.float64)
    if nd == 3:
        r = np.sqrt(h[:, None, None] ** 2 + h[None, :, None] ** 2 + h[None, None, :] ** 2)
    else:
        r = np.sqrt(h[:, None] ** 2 + h[None, :] ** 2)
    x = np.pi * r / padSize
    j0 = np.where(x == 0, 1.0, np.sin(x) / np.where(x == 0, 1.0, x))
    return np.ascontiguousarray((j0 * j0).astype(np.float32))


def _inputs3d(N, pf, seed):
    vdim = N * pf
    rng = np.random.default_rng(seed)
    vol = synth.projectee(synth.blob_volume(N, n_blobs=6, seed=3), pf).numpy()
    quad = orc_rc._ft_quad(vdim).astype(np.float64)
    T = ((50.0 / (1.0 + np.sqrt(quad))) * rng.uniform(0.8, 1.2, quad.shape)).astype(np.float32)
    F = (vol.astype(np.complex128) * T).astype(np.complex64)
    return F, T


def _balance_split_step(T, maxR, pf, N):
    """reconstructG's 3D grid-correction loop (src/Reconstructor.cpp:1962-2087)
    through the split-step adapters; returns (W, iterations)."""
    L = lib()
    vdim = T.shape[0]
    tab, step, nf = _kernel_table()
    dC, dW, dT, dTab, dDiff, dMax, dCount = (ctypes.c_void_p() for _ in range(7))
    streams = (ctypes.c_void_p * 3)()
    check(L.thx_AllocDevicePoint(GPU, *(ctypes.addressof(x) for x in (dC, dW, dT, dTab, dDiff, dMax,
                                                                          dCount)),
                                 streams, 3, TAB_N, vdim), "AllocDevicePoint")
    assert dDiff.value is None and dCount.value is None and streams[0]
    W = np.zeros_like(T)
    try:
        check(L.thx_HostDeviceInit(GPU, P(T), P(tab), dW, dT, dTab, streams, 3, TAB_N, maxR, pf,
                                   vdim), "HostDeviceInit")
        C = np.zeros(T.shape, np.complex64)
        diffC, diffCPrev, noDec = np.float32(3.402823466e38), None, 0
        m = 0
        for m in range(30):                                          # MAX_N_ITER_BALANCE
            check(L.thx_ExposeC(GPU, P(C), dC, dT, dW, streams, 3, vdim), "ExposeC")
            c = np.ascontiguousarray(np.fft.irfftn(C, s=(vdim,) * 3).astype(np.float32))   # bwExecutePlan
            check(L.thx_ExposeForConvC(GPU, P(c), dC, dTab, streams, step, TAB_N, nf, 3, pf, N, vdim),
                  "ExposeForConvC")
            C = np.ascontiguousarray(np.fft.rfftn(c).astype(np.complex64))   # fwExecutePlan
            diffCPrev = diffC
            d = ctypes.c_float()
            check(L.thx_ExposeWC(GPU, P(C), dC, dW, dMax, streams, ctypes.byref(d), 3, maxR, pf,
                                 vdim), "ExposeWC")
            diffC = np.float32(d.value)
            noDec = noDec + 1 if diffC > diffCPrev * np.float32(0.95) else 0
            if diffC < 1e-2 or (m >= 10 and noDec == 2):
                break
        iters = m + 1
    finally:
        check(L.thx_FreeDevHostPoint(GPU, *(ctypes.addressof(x) for x in (dC, dW, dT, dTab, dDiff,
                                                                              dMax, dCount)),
                                     streams, P(W), 3, vdim), "FreeDevHostPoint")
    assert dC.value is None and streams[0] is None
    return W, iters


@pytest.mark.parametrize("map_", [False, True])
def test_reconstructG_3d_through_adapters(map_):
    L = lib()
    N, pf = 32, 2
    vdim = N * pf
    maxR = N // 2 - 2                                   # N / 2 - ceil(a)
    F, T = _inputs3d(N, pf, 11)
    fsc = np.linspace(0.99, 0.2, N // 2 + 1) if map_ else None
    Th = np.ascontiguousarray(T.copy())
    if map_:
        fs = fsc.astype(np.float32)
        check(L.thx_ExposePT(GPU, P(Th), maxR, pf, vdim, P(fs), len(fs), 0, 5), "ExposePT")
    W, iters = _balance_split_step(Th, maxR, pf, N)
    # the in-library loop (ExposeWT with the table) balances to the same W
    tab, step, nf = _kernel_table()
    W2 = np.zeros_like(Th)
    n2 = ctypes.c_int()
    check(L.thx_ExposeWT(GPU, P(Th), P(W2), P(tab), step, TAB_N, nf, maxR, pf, vdim, 30, 10, N,
                         ctypes.byref(n2)), "ExposeWT")
    assert n2.value == iters
    assert np.max(np.abs(W2 - W)) <= 1e-4 * np.max(np.abs(W))
    pad = np.zeros_like(F)
    check(L.thx_ExposePFW(GPU, P(pad), P(F), P(W), maxR, pf, vdim, vdim), "ExposePFW")
    rl = np.fft.irfftn(pad, s=(vdim,) * 3)                               # fft.bw(padDst)
    c = np.fft.fftfreq(N, 1.0 / N).astype(np.int64)
    dst = np.ascontiguousarray(rl[np.ix_(c % vdim, c % vdim, c % vdim)].astype(np.float32))
    check(L.thx_ExposeCorrF(GPU, P(dst), P(_tik_table(N, vdim, 3)), 0.0, N), "ExposeCorrF")
    ref, rit, _ = orc_rc.reconstruct(F, T, N, pf, fsc=fsc)
    assert iters == rit
    assert np.max(np.abs(dst - ref)) <= 1e-4 * np.max(np.abs(ref))
    # ExposePF (pad + backward transform on device) and the two-volume ExposeCorrF
    padR = np.zeros((vdim,) * 3, np.float32)
    check(L.thx_ExposePF(GPU, P(padR), P(F), P(W), maxR, pf, vdim, vdim), "ExposePF")
    assert np.max(np.abs(padR - rl)) <= 1e-5 * np.max(np.abs(rl))
    dstN = np.ascontiguousarray(rl[np.ix_(c % vdim, c % vdim, c % vdim)].astype(np.float32))
    ft = np.zeros((N, N, N // 2 + 1), np.complex64)
    check(L.thx_ExposeCorrFT(GPU, P(dstN), P(ft), P(_tik_table(N, vdim, 3)), 0.0, N), "ExposeCorrFT")
    rft = np.fft.rfftn(ref)
    assert np.max(np.abs(ft - rft)) <= 1e-4 * np.max(np.abs(rft))


def test_no_grid_correction_weights():
    L = lib()
    N, pf = 32, 2
    vdim = N * pf
    maxR = N // 2 - 2
    F, T = _inputs3d(N, pf, 12)
    W = np.full_like(T, 7.0)
    check(L.thx_ExposeWT_T(GPU, P(T), P(W), maxR, pf, vdim), "ExposeWT_T")
    inside = orc_rc._ft_quad(vdim) < (maxR * pf) ** 2
    assert np.allclose(W[inside], 1.0 / np.maximum(np.abs(T[inside]), 1e-6), rtol=1e-6)
    assert np.all(W[~inside] == 7.0)                    # kernel_CalculateW leaves the outside
    pad = np.zeros_like(F)
    check(L.thx_ExposePFW(GPU, P(pad), P(F), P(W), maxR, pf, vdim, vdim), "ExposePFW")
    rl = np.fft.irfftn(pad, s=(vdim,) * 3)
    c = np.fft.fftfreq(N, 1.0 / N).astype(np.int64)
    dst = np.ascontiguousarray(rl[np.ix_(c % vdim, c % vdim, c % vdim)].astype(np.float32))
    check(L.thx_ExposeCorrF(GPU, P(dst), P(_tik_table(N, vdim, 3)), 0.0, N), "ExposeCorrF")
    ref, _, _ = orc_rc.reconstruct(F, T, N, pf, grid_corr=False)
    assert np.max(np.abs(dst - ref)) <= 1e-4 * np.max(np.abs(ref))


@pytest.mark.parametrize("grid_corr,map_", [(True, False), (False, False), (True, True)])
def test_reconstructG_2d_through_adapters(grid_corr, map_):
    L = lib()
    N, pf = 64, 2
    vdim = N * pf
    maxR = N // 2 - 2
    rng = np.random.default_rng(5)
    quad = orc_rc._ft_quad2(vdim).astype(np.float64)
    X = np.fft.rfftn(rng.standard_normal((vdim, vdim)))
    T = ((30.0 / (1.0 + np.sqrt(quad))) * rng.uniform(0.8, 1.2, quad.shape)).astype(np.float32)
    F = (X * T).astype(np.complex64)
    fsc = np.linspace(0.99, 0.15, N // 2 + 1) if map_ else None
    Th = T.copy()
    if map_:
        fs = fsc.astype(np.float32)
        check(L.thx_ExposePT2D(GPU, P(Th), maxR, pf, vdim, P(fs), len(fs), 0, 5), "ExposePT2D")
    W = np.zeros_like(Th)
    if grid_corr:
        tab, step, nf = _kernel_table()
        it = ctypes.c_int()
        check(L.thx_ExposeWT2D(GPU, P(Th), P(W), P(tab), step, TAB_N, nf, maxR, pf, vdim, 30, 10, N,
                               ctypes.byref(it)), "ExposeWT2D")
    else:
        check(L.thx_ExposeWT2D_T(GPU, P(Th), P(W), maxR, pf, vdim), "ExposeWT2D_T")
    padR = np.zeros((vdim, vdim), np.float32)
    check(L.thx_ExposePF2D(GPU, P(padR), P(F), P(W), maxR, pf, vdim, vdim), "ExposePF2D")
    c = np.fft.fftfreq(N, 1.0 / N).astype(np.int64)
    img = np.ascontiguousarray(padR[np.ix_(c % vdim, c % vdim)])          # IMG_EXTRACT_RL
    ft = np.zeros((N, N // 2 + 1), np.complex64)
    check(L.thx_ExposeCorrF2D(GPU, P(img), P(ft), P(_tik_table(N, vdim, 2)), 0.0, N), "ExposeCorrF2D")
    ref, rit, _ = orc_rc.reconstruct2d(F, T, N, pf, grid_corr=grid_corr, fsc=fsc)
    if grid_corr:
        assert it.value == rit
    rft = np.fft.rfft2(ref)
    assert np.max(np.abs(ft - rft)) <= 1e-4 * np.max(np.abs(rft))


@pytest.mark.parametrize("sym", ["C1", "C4", "D2"])
def test_prepare_tf_adapter(sym):
    """PrepareTF with symMat packed as prepareTFG packs it (Eigen column-major)."""
    L = lib()
    vdim, maxR, pf = 32, 6, 2
    rng = np.random.default_rng(3)
    F = np.fft.rfftn(rng.standard_normal((vdim,) * 3)).astype(np.complex64)
    T = np.abs(np.fft.rfftn(rng.standard_normal((vdim,) * 3))).astype(np.float32) + 0.5
    R, _ = osym.elements(sym)
    symMat = np.ascontiguousarray(np.stack([r.T for r in R]) if len(R) else np.zeros((1, 3, 3)))
    Fh, Th = F.copy(), T.copy()
    check(L.thx_PrepareTF(GPU, P(Fh), P(Th), P(symMat), len(R), maxR, pf, vdim), "PrepareTF")
    rF, rT = osym.prepare_tf(F, T, R, maxR, pf)
    # the shell the radius test decides by rounding can differ (the same
    # voxels tests/test_gpu_symmetry.py masks); compare the decided voxels
    i = np.arange(vdim // 2 + 1)
    j = np.fft.fftfreq(vdim, 1.0 / vdim)
    K, J, I = np.meshgrid(j, j, i, indexing="ij")
    r2 = (maxR * pf + 1) ** 2
    ok = np.ones(F.shape, bool)
    for M in R:
        q2 = ((M @ np.stack([I.ravel(), J.ravel(), K.ravel()])) ** 2).sum(0).reshape(F.shape)
        ok &= np.abs(q2 - r2) > 1e-3
    assert np.max(np.abs(Fh - rF)[ok]) <= 1e-5 * np.abs(rF).max()
    assert np.max(np.abs(Th - np.maximum(rT, 1e-25))[ok]) <= 1e-5 * np.abs(rT).max()


def test_translate_adapters():
    L = lib()
    dim, r = 32, 12
    rng = np.random.default_rng(8)
    V = (rng.standard_normal((dim, dim, dim // 2 + 1)) +
         1j * rng.standard_normal((dim, dim, dim // 2 + 1))).astype(np.complex64)
    ox, oy, oz = -1.7, 2.25, 0.6
    got = V.copy()
    check(L.thx_TranslateI(GPU, P(got), ox, oy, oz, r, dim), "TranslateI")
    i = np.arange(dim // 2 + 1)
    j = np.fft.fftfreq(dim, 1.0 / dim)
    K, J, I = np.meshgrid(j, j, i, indexing="ij")
    ph = 2 * np.pi * (I * ox + J * oy + K * oz) / dim
    ref = np.where(I ** 2 + J ** 2 + K ** 2 < r * r, V * np.exp(-1j * ph), V)
    assert np.max(np.abs(got - ref)) <= 2e-5 * np.abs(ref).max()
    img = V[0].copy()
    check(L.thx_TranslateI2D(GPU, P(img), ox, oy, r, dim), "TranslateI2D")
    J2, I2 = np.meshgrid(j, i, indexing="ij")
    ref2 = np.where(I2 ** 2 + J2 ** 2 < r * r, V[0] * np.exp(-2j * np.pi * (I2 * ox + J2 * oy) / dim), V[0])
    assert np.max(np.abs(img - ref2)) <= 2e-5 * np.abs(ref2).max()


def test_remask_and_gctf_adapters():
    L = lib()
    N, n = 64, 5
    rng = np.random.default_rng(9)
    imgs = [np.fft.rfft2(rng.standard_normal((N, N))).astype(np.complex64) for _ in range(n)]
    before = [x.copy() for x in imgs]
    arr = (ctypes.c_void_p * n)(*[x.ctypes.data for x in imgs])
    mask_a, pix, ew = 80.0, 2.5, 6.0
    check(L.thx_ReMask(arr, mask_a, pix, ew, N, n), "ReMask")
    for b, x in zip(before, imgs):
        rr = opp.remask(b.astype(np.complex128), N, mask_a / pix, ew)
        assert np.max(np.abs(x - rr)) <= 2e-5 * np.abs(rr).max()
    # GCTFinit: (CTF, 0) over the whole grid, CTFAttr rows of 7 floats
    attr8 = synth.ctf_attrs(n, seed=3)                    # {pixelSize, voltage, dU, dV, theta, Cs, ampC, ps}
    ctfa = np.ascontiguousarray(attr8[:, 1:].astype(np.float32))
    out = [np.zeros((N, N // 2 + 1), np.complex64) for _ in range(n)]
    arr = (ctypes.c_void_p * n)(*[x.ctypes.data for x in out])
    check(L.thx_GCTFinit(arr, P(ctfa), float(attr8[0, 0]), N, n), "GCTFinit")
    a8 = attr8.astype(np.float32).copy()
    a8[:, 0] = attr8[0, 0]
    px = ops.PixelSet(N, 2, N // 4, 1, device=DEV)
    ref = ops.ctf(torch.as_tensor(a8, device=DEV), px).cpu().numpy()
    for l in range(n):
        assert np.all(out[l].imag == 0)
        assert np.allclose(out[l].reshape(-1).real[px.iPxl], ref[l], rtol=0, atol=1e-6)
