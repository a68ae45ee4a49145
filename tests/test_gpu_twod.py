"""f4 on the GPU: the 2D classification path (MODE_2D) against the C
restatement -- thx_project2d vs orc.project2d, the 2D global scan over nK
classes (thx_ExpectGlobal2D, gpu/interface/Interface.h:176-197) vs
orc.project2d + orc.logdatavs + orc.weights_global(kIdx, nK), one 2D
particle-filter phase (thx_local_phase2d, the 2D branch of
src/Optimiser.cpp:1183-1402) vs the restated direct likelihood, and the 2D
insert with per-sample classes (thx_insert2d / thx_InsertI2D, Interface.h:
239-265) vs orc.insert2d_batch."""
import ctypes

import numpy as np
import pytest
import torch

from thunder_amd import ops
from thunder_amd._lib import lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
vp = ctypes.c_void_p


def T_(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


def P(a):
    return a.ctypes.data_as(vp)


def _classes(nK, N, pf, seed):
    """nK half-complex class images [nK, vdim, vdim/2+1] (smooth blobs)."""
    vdim = N * pf
    rng = np.random.default_rng(seed)
    out = np.empty((nK, vdim, vdim // 2 + 1), np.complex64)
    yy, xx = np.mgrid[:vdim, :vdim] - vdim // 2
    for k in range(nK):
        img = np.zeros((vdim, vdim))
        for _ in range(5):
            cx, cy = rng.uniform(-N / 4, N / 4, 2)
            img += rng.uniform(0.5, 1.5) * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * rng.uniform(2, 5) ** 2))
        out[k] = np.fft.rfft2(np.fft.ifftshift(img)) / vdim
    return out


def _rot(th):
    return np.stack([np.cos(th), np.sin(th)], -1)


def _stack(orc, N=32, pf=2, rU=12, nImg=6, nK=3, seed=0):
    vdim = N * pf
    px = orc.pixel_set(N, pf, rU, 1)
    cl = _classes(nK, N, pf, seed)
    rng = np.random.default_rng(seed + 1)
    k = rng.integers(0, nK, nImg)
    th = rng.uniform(0, 2 * np.pi, nImg)
    t = rng.standard_normal((nImg, 2))
    dat = np.stack([orc.project2d(cl[k[l]], vdim, pf, _rot(th[l]), px) * orc.translate(px, *t[l], N)
                    for l in range(nImg)])
    dat = (dat + 0.3 * (rng.standard_normal(dat.shape) + 1j * rng.standard_normal(dat.shape))
           ).astype(np.complex64)
    ctf = rng.uniform(0.3, 1.0, (nImg, px.n)).astype(np.float32)
    sig = rng.uniform(0.5, 2.0, (nImg, px.n)).astype(np.float32)
    return dict(N=N, pf=pf, vdim=vdim, px=px, cl=cl, dat=dat, ctf=ctf, sig=sig, k=k, th=th, t=t,
                gpx=ops.PixelSet(N, pf, rU, 1, device=DEV), rng=rng)


def test_project2d_matches_restatement(orc):
    s = _stack(orc)
    th = s["rng"].uniform(0, 2 * np.pi, 37)
    got = ops.project2d(T_(s["cl"][1]), T_(_rot(th)), s["gpx"]).cpu().numpy()
    ref = np.stack([orc.project2d(s["cl"][1], s["vdim"], s["pf"], _rot(a), s["px"]) for a in th])
    assert np.max(np.abs(got - ref)) <= 1e-5 * np.abs(ref).max()


def test_expect_global2d_matches_restatement(orc):
    s = _stack(orc, nImg=4, nK=3)
    N, pf, vdim, px = s["N"], s["pf"], s["vdim"], s["px"]
    nK, nR, nT, nImg = 3, 24, 9, 4
    rot = _rot(np.arange(nR) * 2 * np.pi / nR)
    g = np.linspace(-1.5, 1.5, 3)
    trans = np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2)
    pR = np.full(nR, 1.0 / nR)
    pT = np.full(nT, 1.0 / nT)
    state = None
    dvps = []
    for k in range(nK):
        dvp = np.empty((nImg, nR, nT), np.float32)
        for r in range(nR):
            pri = orc.project2d(s["cl"][k], vdim, pf, rot[r], px)
            for t in range(nT):
                pt = (orc.translate(px, *trans[t], N) * pri).astype(np.complex64)
                for l in range(nImg):
                    dvp[l, r, t] = orc.logdatavs(s["dat"][l], pt, s["ctf"][l], s["sig"][l])
        dvps.append(dvp)
        state = orc.weights_global(dvp, pR, pT, k, nK, state)
    rC, rR, rT, rb = state
    wC = np.zeros(nImg * nK, np.float32)
    wR = np.zeros(nImg * nK * nR, np.float32)
    wT = np.zeros(nImg * nK * nT, np.float32)
    cl = np.ascontiguousarray(s["cl"]).view(np.float32)
    dat = np.ascontiguousarray(s["dat"]).view(np.float32)
    ctf, sig = np.ascontiguousarray(s["ctf"]), np.ascontiguousarray(s["sig"])
    rc = lib().thx_ExpectGlobal2D(P(cl), P(dat), P(ctf), P(sig), P(trans), P(wC), P(wR), P(wT),
                                  P(pR), P(pT), P(rot), P(px.iCol), P(px.iRow), nK, nR, nT, pf, 1,
                                  N, vdim, px.n, nImg)
    assert rc == 0, lib().thx_last_error()
    # the GPU scan keeps its running baseline across classes exactly like the
    # restatement; marginals agree to the FP32 likelihood's rounding
    best = np.max([d.reshape(nImg, -1).max(1) for d in dvps], axis=0)
    assert np.all(np.abs(rb - best) <= 1e-6 * np.abs(best))
    for got, want in ((wC, rC), (wR, rR), (wT, rT)):
        m = want >= 1e-4 * want.max()
        assert np.max(np.abs(got - want)[m] / want[m]) < 2e-3


def test_local_phase2d_matches_restatement(orc):
    s = _stack(orc, nImg=5, nK=2, seed=4)
    N, pf, vdim, px = s["N"], s["pf"], s["vdim"], s["px"]
    nImg, mR, mT = 5, 20, 6
    rng = s["rng"]
    th = s["th"][:, None] + rng.standard_normal((nImg, mR)) * 0.05
    rot = _rot(th)
    trans = s["t"][:, None, :] + rng.standard_normal((nImg, mT, 2)) * 0.5
    pC = np.full(nImg, 0.8)
    pR = rng.uniform(0.5, 1.5, (nImg, mR))
    pR /= pR.sum(1, keepdims=True)
    pT = np.full((nImg, mT), 1.0 / mT)
    cls = s["k"].astype(np.int32)
    wC, wR, wT, base, d = ops.local_phase2d(T_(s["cl"]), T_(rot), T_(trans), T_(pC), T_(pR), T_(pT),
                                            T_(s["dat"]), T_(s["ctf"]), T_(s["sig"]), s["gpx"],
                                            cls=T_(cls), want_dvp=True)
    d = d.cpu().numpy()
    wR, wT, wC = wR.cpu().numpy(), wT.cpu().numpy(), wC.cpu().numpy()
    for l in range(nImg):
        ref = np.empty((mR, mT), np.float32)
        for r in range(mR):
            pri = orc.project2d(s["cl"][cls[l]], vdim, pf, rot[l, r], px)
            for t in range(mT):
                pt = (orc.translate(px, *trans[l, t], N) * pri).astype(np.complex64)
                ref[r, t] = orc.logdatavs(s["dat"][l], pt, s["ctf"][l], s["sig"][l])
        assert np.max(np.abs(d[l] - ref)) <= 1e-5 * np.abs(ref).max()
        # the restatement's marginals (src/Optimiser.cpp:1302-1340, nD = 1)
        base_l = ref.max()
        e = np.exp((ref - base_l).astype(np.float64))
        rR = (e * pT[l][None, :]).sum(1) * pC[l]
        rT = (e * pR[l][:, None]).sum(0) * pC[l]
        rC = (e * pR[l][:, None] * pT[l][None, :]).sum()
        tol = max(1e-3, 2.5 * float(np.max(np.abs(d[l] - ref))))
        for got, want in ((wR[l], rR), (wT[l], rT)):
            m = want >= 1e-4 * want.max()
            assert np.max(np.abs(got - want)[m] / want[m]) < tol
        assert abs(wC[l] - rC) <= tol * rC


@pytest.mark.parametrize("nK", [1, 3])
def test_insert2d_matches_restatement(orc, nK):
    N, pf = 32, 2
    vdim = N * pf
    px = orc.pixel_set(N, pf, N // 2 - 2, 0)
    gpx = ops.PixelSet(N, pf, N // 2 - 2, 0, device=DEV)
    rng = np.random.default_rng(7 + nK)
    nImg, mReco = 9, 5
    dat = (rng.standard_normal((nImg, px.n)) + 1j * rng.standard_normal((nImg, px.n))).astype(np.complex64)
    ctf = rng.uniform(-1, 1, (nImg, px.n)).astype(np.float32)
    rot = _rot(rng.uniform(0, 2 * np.pi, (nImg, mReco)))
    trans = rng.standard_normal((nImg, mReco, 2))
    off = rng.standard_normal((nImg, 2)) * 0.2
    w = rng.uniform(0.1, 0.3, nImg).astype(np.float32)
    nc = rng.integers(0, nK, (nImg, mReco)).astype(np.int32) if nK > 1 else None
    F, T, O, cnt = orc.insert2d_batch(vdim, pf, dat, ctf, rot, trans, off, w, nc, px, N, nK=nK)
    hm = ops.HalfMap2D(vdim, nK, DEV)
    ops.insert2d(hm, T_(dat), T_(ctf), T_(rot), T_(trans), T_(off), T_(w), gpx,
                 nc=T_(nc) if nc is not None else None)
    gF = hm.F.cpu().numpy().reshape(-1)
    gT = hm.T.cpu().numpy().reshape(-1)
    assert np.max(np.abs(gF - F)) <= 1e-5 * np.abs(F).max()
    assert np.max(np.abs(gT - T)) <= 1e-5 * np.abs(T).max()
    assert np.allclose(hm.O.cpu().numpy().reshape(-1), O, rtol=1e-12, atol=1e-12)
    assert np.array_equal(hm.counter.cpu().numpy(), cnt.astype(np.int32))
    # the host adapter (InsertI2D): read-modify-write of host buffers
    hF = np.zeros(2 * F.size, np.float32)
    hT = np.zeros(T.size, np.float32)
    hO = np.zeros(2 * nK)
    hc = np.zeros(nK, np.int32)
    ncl = nc if nc is not None else np.zeros((nImg, mReco), np.int32)
    rc = lib().thx_InsertI2D(P(hF), P(hT), P(hO), P(hc), None, P(dat.view(np.float32)), P(ctf),
                             None, P(w), P(off), P(ncl), P(np.ascontiguousarray(rot)), P(trans),
                             None, None, P(px.iColPad), P(px.iRowPad), 0.0, 0, nK, pf, px.n,
                             mReco, N, vdim, nImg)
    assert rc == 0, lib().thx_last_error()
    assert np.max(np.abs(hF.view(np.complex64) - F)) <= 1e-5 * np.abs(F).max()
    assert np.array_equal(hc, cnt.astype(np.int32))


def test_local_2d_through_interface_forwards(orc):
    """MODE_2D through the per-image local surface (ExpectLocalV2D ->
    ExpectLocalRTD with 4-double rotation rows -> ExpectLocalPreI2D ->
    ExpectLocalM), against the restatement's 2D phase per image."""
    s = _stack(orc, nImg=3, nK=2, seed=9)
    N, pf, vdim, px = s["N"], s["pf"], s["vdim"], s["px"]
    L = lib()
    npxl, mR, mT, gpu, cpy = px.n, 20, 6, 0, 2
    iCol, iRow = px.iCol.copy(), px.iRow.copy()
    dCol, dRow = vp(), vp()
    assert L.thx_ExpectPreidx(gpu, ctypes.byref(dCol), ctypes.byref(dRow), P(iCol), P(iRow), npxl) == 0
    mgr = vp()
    assert L.thx_tex_create(0, vdim, gpu, ctypes.byref(mgr)) == 0
    dat = np.ascontiguousarray(s["dat"]).view(np.float32)
    ctf, sig = np.ascontiguousarray(s["ctf"]), np.ascontiguousarray(s["sig"])
    dD, dC, dO, dS = vp(), vp(), vp(), vp()
    assert L.thx_ExpectLocalIn(gpu, ctypes.byref(dD), ctypes.byref(dC), ctypes.byref(dO),
                               ctypes.byref(dS), npxl, cpy, 1) == 0
    mcp = vp()
    assert L.thx_calpoint_create(0, 1, gpu, mR, mT, 1, npxl, ctypes.byref(mcp)) == 0
    rng = np.random.default_rng(3)
    wC, wR, wT, wD = (np.zeros(n, np.float32) for n in (1, mR, mT, 1))
    for img in range(3):
        k = int(s["k"][img])
        cl = np.ascontiguousarray(s["cl"][k]).view(np.float32)
        assert L.thx_ExpectLocalV2D(gpu, mgr, P(cl), (vdim // 2 + 1) * vdim) == 0, L.thx_last_error()
        slot = img % cpy
        assert L.thx_ExpectLocalP(gpu, dD, dC, dO, dS, P(dat), P(ctf), None, P(sig), slot, img,
                                  npxl, 0) == 0
        th = s["th"][img] + rng.standard_normal(mR) * 0.05
        rot4 = np.zeros((mR, 4))
        rot4[:, 0], rot4[:, 1] = np.cos(th), np.sin(th)
        trans = s["t"][img][None, :] + rng.standard_normal((mT, 2)) * 0.5
        pR = rng.uniform(0.5, 1.5, mR)
        pR /= pR.sum()
        pT = np.full(mT, 1.0 / mT)
        oldD, dpara = np.ones(1), np.ones(1)
        rot4c, transc = np.ascontiguousarray(rot4), np.ascontiguousarray(trans)
        assert L.thx_ExpectLocalRTD(gpu, mcp, P(pR), P(pT), P(oldD), P(transc), P(rot4c),
                                    P(dpara)) == 0
        assert L.thx_ExpectLocalPreI2D(gpu, slot, mgr, mcp, None, None, dCol, dRow, 0.0, 0.1, 0.0,
                                       0.0, pf, N, vdim, npxl, 1) == 0, L.thx_last_error()
        oldC = 0.8
        assert L.thx_ExpectLocalM(gpu, slot, mcp, dD, dC, dS, P(wC), P(wR), P(wT), P(wD), oldC,
                                  npxl) == 0, L.thx_last_error()
        ref = np.empty((mR, mT), np.float32)
        for r in range(mR):
            pri = orc.project2d(s["cl"][k], vdim, pf, _rot(th[r]), px)
            for t in range(mT):
                pt = (orc.translate(px, *trans[t], N) * pri).astype(np.complex64)
                ref[r, t] = orc.logdatavs(s["dat"][img], pt, s["ctf"][img], s["sig"][img])
        e = np.exp((ref - ref.max()).astype(np.float64))
        rR = (e * pT[None, :]).sum(1) * oldC
        rT = (e * pR[:, None]).sum(0) * oldC
        rC = (e * pR[:, None] * pT[None, :]).sum()
        for got, want in ((wR, rR), (wT, rT)):
            m = want >= 1e-4 * want.max()
            assert np.max(np.abs(got - want)[m] / want[m]) < 2e-3
        assert abs(wC[0] - rC) <= 2e-3 * rC
    assert L.thx_calpoint_destroy(mcp) == 0
    assert L.thx_ExpectLocalFin(gpu, ctypes.byref(dD), ctypes.byref(dC), ctypes.byref(dO), None,
                                ctypes.byref(dS), 0) == 0
    assert L.thx_tex_destroy(mgr) == 0
    assert L.thx_ExpectFreeIdx(gpu, ctypes.byref(dCol), ctypes.byref(dRow)) == 0


def test_c1_shape_global_scan(orc):
    """Config C1's global scan (script/demo_2D.json: box 64, 8 classes, 2D
    global sampling mS 100 -> nR 100, transS 10 -> nT 151, global-search ring
    rU 7 -> nPxl 69) through thx_ExpectGlobal2D on 16 images against the
    restatement: orc.project2d / orc.translate per sample, the likelihood of
    every (image, class, rotation, translation) in float64 (the FP32 sum of
    orc.logdatavs over 69 pixels agrees with it to ~1e-7 relative; 1.9 M
    ctypes calls would take minutes), and orc.weights_global(kIdx, nK) for the
    running baseline and marginals over the 8 classes."""
    N, pf, nK, rU, nImg = 64, 2, 8, 7, 16
    s = _stack(orc, N=N, pf=pf, rU=rU, nImg=nImg, nK=nK, seed=31)
    vdim = s["vdim"]
    px = orc.pixel_set(N, pf, rU, 0)
    assert px.n == 69                       # SURVEY 8's C1 global-search count
    mS, nR, nT = ops.global_sample_sizes(100, mode=0)
    assert (nR, nT) == (100, 151)
    rng = np.random.default_rng(32)
    # the images on the rL 0 ring (the stack's own set is rL 1)
    k_true = rng.integers(0, nK, nImg)
    th_true = rng.uniform(0, 2 * np.pi, nImg)
    t_true = rng.standard_normal((nImg, 2)) * 2
    dat = np.stack([orc.project2d(s["cl"][k_true[l]], vdim, pf, _rot(th_true[l]), px) *
                    orc.translate(px, *t_true[l], N) for l in range(nImg)])
    dat = (dat + 0.5 * (rng.standard_normal(dat.shape) + 1j * rng.standard_normal(dat.shape))
           ).astype(np.complex64)
    ctf = rng.uniform(0.3, 1.0, (nImg, px.n)).astype(np.float32)
    sig = -rng.uniform(0.5, 2.0, (nImg, px.n)).astype(np.float32)
    rot = _rot(rng.uniform(0, 2 * np.pi, nR))
    trans = rng.standard_normal((nT, 2)) * 10.0
    pR = np.full(nR, 1.0 / nR)
    pT = rng.uniform(0.5, 1.5, nT)
    pT /= pT.sum()
    tra = np.stack([orc.translate(px, *trans[t], N) for t in range(nT)]).astype(np.complex128)
    state = None
    for k in range(nK):
        pri = np.stack([orc.project2d(s["cl"][k], vdim, pf, rot[r], px) for r in range(nR)])
        pt = (pri.astype(np.complex128)[:, None, :] * tra[None, :, :]).astype(np.complex64)
        dvp = np.empty((nImg, nR, nT), np.float32)
        for l in range(nImg):
            e = dat[l].astype(np.complex128) - ctf[l].astype(np.float64) * pt.astype(np.complex128)
            dvp[l] = (sig[l].astype(np.float64) * (e.real ** 2 + e.imag ** 2)).sum(-1)
        state = orc.weights_global(dvp, pR, pT, k, nK, state)
    rC, rR, rT, rb = state
    wC = np.zeros(nImg * nK, np.float32)
    wR = np.zeros(nImg * nK * nR, np.float32)
    wT = np.zeros(nImg * nK * nT, np.float32)
    cl = np.ascontiguousarray(s["cl"]).view(np.float32)
    datf = np.ascontiguousarray(dat).view(np.float32)
    rc = lib().thx_ExpectGlobal2D(P(cl), P(datf), P(ctf), P(sig), P(np.ascontiguousarray(trans)),
                                  P(wC), P(wR), P(wT), P(pR), P(pT), P(np.ascontiguousarray(rot)),
                                  P(px.iCol), P(px.iRow), nK, nR, nT, pf, 1, N, vdim, px.n, nImg)
    assert rc == 0, lib().thx_last_error()
    for got, want in ((wC, rC), (wR, rR), (wT, rT)):
        got, want = got.reshape(nImg, -1), want.reshape(nImg, -1)
        m = want >= 1e-4 * want.max(axis=1, keepdims=True)
        assert np.max(np.abs(got - want)[m] / want[m]) < 2e-3
    # the classes the scan puts the weight on are the images' true classes
    assert np.mean(wC.reshape(nImg, nK).argmax(1) == k_true) >= 0.75


def test_c1_shape_phase_and_insert(orc):
    """Config C1 (script/demo_2D.json): box 64, 8 classes, the full-resolution
    ring rU 30 (nPxl 1367): the 2D phase per image against the restatement and
    the 8-class insert with per-sample classes."""
    N, pf, nK = 64, 2, 8
    s = _stack(orc, N=N, pf=pf, rU=30, nImg=3, nK=nK, seed=21)
    vdim, px = s["vdim"], s["px"]
    # SURVEY 8's C1 count 1367 is the rL 0 ring; the stack's rL 1 drops the origin
    assert px.n == 1366
    nImg, mR, mT = 3, 16, 5
    rng = s["rng"]
    th = s["th"][:, None] + rng.standard_normal((nImg, mR)) * 0.05
    rot = _rot(th)
    trans = s["t"][:, None, :] + rng.standard_normal((nImg, mT, 2)) * 0.5
    pC = np.full(nImg, 0.9)
    pR = np.full((nImg, mR), 1.0 / mR)
    pT = np.full((nImg, mT), 1.0 / mT)
    cls = s["k"].astype(np.int32)
    _, _, _, _, d = ops.local_phase2d(T_(s["cl"]), T_(rot), T_(trans), T_(pC), T_(pR), T_(pT),
                                      T_(s["dat"]), T_(s["ctf"]), T_(s["sig"]), s["gpx"],
                                      cls=T_(cls), want_dvp=True)
    d = d.cpu().numpy()
    for l in range(nImg):
        ref = np.empty((mR, mT), np.float32)
        for r in range(mR):
            pri = orc.project2d(s["cl"][cls[l]], vdim, pf, rot[l, r], px)
            for t in range(mT):
                pt = (orc.translate(px, *trans[l, t], N) * pri).astype(np.complex64)
                ref[r, t] = orc.logdatavs(s["dat"][l], pt, s["ctf"][l], s["sig"][l])
        assert np.max(np.abs(d[l] - ref)) <= 1e-5 * np.abs(ref).max()
    mReco = 20
    irot = _rot(rng.uniform(0, 2 * np.pi, (nImg, mReco)))
    itr = rng.standard_normal((nImg, mReco, 2))
    off = rng.standard_normal((nImg, 2)) * 0.2
    w = np.full(nImg, 1.0 / mReco, np.float32)
    nc = rng.integers(0, nK, (nImg, mReco)).astype(np.int32)
    F, Tm, O, cnt = orc.insert2d_batch(vdim, pf, s["dat"], s["ctf"], irot, itr, off, w, nc, px, N,
                                       nK=nK)
    hm = ops.HalfMap2D(vdim, nK, DEV)
    ops.insert2d(hm, T_(s["dat"]), T_(s["ctf"]), T_(irot), T_(itr), T_(off), T_(w), s["gpx"],
                 nc=T_(nc))
    assert np.max(np.abs(hm.F.cpu().numpy().reshape(-1) - F)) <= 1e-5 * np.abs(F).max()
    assert np.max(np.abs(hm.T.cpu().numpy().reshape(-1) - Tm)) <= 1e-5 * np.abs(Tm).max()
    assert np.array_equal(hm.counter.cpu().numpy(), cnt.astype(np.int32))


def test_insert_i2d_ctf_search_and_devices(orc, monkeypatch):
    """thx_InsertI2D with cSearch (Interface.h:239-265's argument list): every
    sample inserts with its own CTF, CTFAttr at defocus factor nD (CTF.cpp at
    (dU d, dV d)), per-sample classes, read-modify-write of the caller's
    buffers -- against the restatement inserting sample by sample with
    orc.ctf; once on the current device and once dealt over THX_DEVICES
    "0,0" (two workers, the peer-copy reduction)."""
    N, pf, nK = 32, 2, 3
    vdim = N * pf
    px = orc.pixel_set(N, pf, N // 2 - 2, 0)
    rng = np.random.default_rng(17)
    nImg, mReco = 5, 4
    dat = (rng.standard_normal((nImg, px.n)) + 1j * rng.standard_normal((nImg, px.n))).astype(np.complex64)
    rot = _rot(rng.uniform(0, 2 * np.pi, (nImg, mReco)))
    trans = rng.standard_normal((nImg, mReco, 2))
    off = rng.standard_normal((nImg, 2)) * 0.2
    w = rng.uniform(0.1, 0.3, nImg).astype(np.float32)
    nc = rng.integers(0, nK, (nImg, mReco)).astype(np.int32)
    nD = rng.uniform(0.97, 1.03, (nImg, mReco))
    pixel = 1.32
    # CTFAttr: voltage, defocusU, defocusV, defocusTheta, Cs, amplitudeContrast, phaseShift
    ca = np.stack([np.full(nImg, 300e3), rng.uniform(1.5e4, 3e4, nImg), rng.uniform(1.5e4, 3e4, nImg),
                   rng.uniform(0, np.pi, nImg), np.full(nImg, 2.7e7), np.full(nImg, 0.1),
                   np.zeros(nImg)], 1).astype(np.float32)
    size = (vdim // 2 + 1) * vdim
    rF = np.zeros(nK * size, np.complex64)
    rT = np.zeros(nK * size, np.float32)
    rO = np.zeros(2 * nK)
    rc = np.zeros(nK, np.int64)
    for l in range(nImg):
        for m in range(mReco):
            a = ca[l]
            c = orc.ctf(px, (pixel, a[0], a[1] * nD[l, m], a[2] * nD[l, m], a[3], a[4], a[5], a[6]), N)
            F, Tm, O, cnt = orc.insert2d_batch(vdim, pf, dat[l:l + 1], c[None], rot[l:l + 1, m:m + 1],
                                               trans[l:l + 1, m:m + 1], off[l:l + 1], w[l:l + 1],
                                               nc[l:l + 1, m:m + 1].copy(), px, N, nK=nK)
            rF += F.reshape(-1)
            rT += Tm.reshape(-1)
            rO += O.reshape(-1)
            rc += np.asarray(cnt).reshape(-1)
    for devs in ("current", "0,0"):
        monkeypatch.setenv("THX_DEVICES", devs)
        hF = np.zeros(2 * nK * size, np.float32)
        hT = np.zeros(nK * size, np.float32)
        hO = np.zeros(2 * nK)
        hc = np.zeros(nK, np.int32)
        rc_ = lib().thx_InsertI2D(P(hF), P(hT), P(hO), P(hc), None, P(dat.view(np.float32)), None,
                                  None, P(w), P(off), P(nc), P(np.ascontiguousarray(rot)),
                                  P(trans), P(nD), P(ca), P(px.iColPad), P(px.iRowPad), pixel, 1,
                                  nK, pf, px.n, mReco, N, vdim, nImg)
        assert rc_ == 0, lib().thx_last_error()
        assert np.max(np.abs(hF.view(np.complex64) - rF)) <= 1e-5 * np.abs(rF).max()
        assert np.max(np.abs(hT - rT)) <= 1e-5 * np.abs(rT).max()
        assert np.allclose(hO, rO, rtol=1e-12, atol=1e-12)
        assert np.array_equal(hc, rc.astype(np.int32))
