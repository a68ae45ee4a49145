"""The MODE_2D expectation driver (thx_expectation2d) and its von Mises
particle statistics.

The deterministic statistics are checked against the restatement
(oracle/particle.py: inferVMS's k1, 1/pdfVMS priors, src/Particle.cpp:
1013-1016, 2317-2329); the perturbation by its distribution (the angle
increments of sampleVMS have E cos = I1(kappa)/I0(kappa),
DirectionalStat.cpp:264-318) and by the priors of the cloud it returns; the
end-to-end driver at config C1's shape (box 64, 8 classes; script/demo_2D.json)
by the properties the reference's urandom-seeded loop guarantees: images made
from a known class at a known angle and shift come back in that class, at that
angle and shift, and a fixed seed reproduces the run bit for bit."""
import numpy as np
import pytest
import torch
from scipy.special import i0, i1

from oracle import particle as op
from thunder_amd import expectation as ex
from thunder_amd import ops, synth
from thunder_amd._lib import check, lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def T(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


def rows(th):
    return np.stack([np.cos(th), np.sin(th), 0 * th, 0 * th], -1)


def test_calvari2d_and_balance_match_restatement():
    rng = np.random.default_rng(5)
    nImg, mR, mT = 24, 125, 9
    # from wide (kappa < 5: the I0 branch) to tight clouds (the Gaussian branch)
    spread = np.geomspace(0.02, 2.5, nImg)
    th = rng.uniform(0, 2 * np.pi, nImg)[:, None] + rng.standard_normal((nImg, mR)) * spread[:, None]
    R = rows(th)
    tr = rng.standard_normal((nImg, mT, 2)) * 3
    k = torch.empty(nImg, 3, dtype=torch.float64, device=DEV)
    sd = torch.empty(nImg, 2, dtype=torch.float64, device=DEV)
    dR, dT = T(R), T(tr)
    check(lib().thx_pf_calvari2d(nImg, mR, ops._ptr(dR), mT, ops._ptr(dT), 0.0, 0.0,
                                 ops._ptr(k), ops._ptr(sd), None), "thx_pf_calvari2d")
    pR = torch.empty(nImg, mR, dtype=torch.float64, device=DEV)
    check(lib().thx_pf_balance_rot2d(nImg, mR, ops._ptr(dR), ops._ptr(pR), None),
          "thx_pf_balance_rot2d")
    k, sd, pR = k.cpu().numpy(), sd.cpu().numpy(), pR.cpu().numpy()
    kappas = []
    for l in range(nImg):
        k1 = op.cal_vari_rot2d(R[l])
        assert abs(k[l, 0] - k1) <= 1e-12 * max(k1, 1e-3) and k[l, 1] == k[l, 0] == k[l, 2]
        assert np.allclose(sd[l], op.cal_vari_trans(tr[l]), rtol=1e-12)
        want = op.balance_rot2d(R[l])
        assert np.max(np.abs(pR[l] - want) / want) < 1e-9, l
        kappas.append(op.vms_kappa(k1))
    assert min(kappas) < 5 < max(kappas)            # both pdfVMS branches ran


def test_calvari2d_floor():
    R = rows(np.full((2, 16), 0.3))                  # a point cloud: k1 = 0
    tr = np.zeros((2, 4, 2))
    k = torch.empty(2, 3, dtype=torch.float64, device=DEV)
    sd = torch.empty(2, 2, dtype=torch.float64, device=DEV)
    dR, dT = T(R), T(tr)        # held: a temporary's memory would be reused at once
    check(lib().thx_pf_calvari2d(2, 16, ops._ptr(dR), 4, ops._ptr(dT), 0.02, 0.5,
                                 ops._ptr(k), ops._ptr(sd), None), "thx_pf_calvari2d")
    assert np.allclose(k.cpu().numpy(), 0.02) and np.allclose(sd.cpu().numpy(), 0.5)


@pytest.mark.parametrize("k1, pf", [(0.05, 0.5), (0.004, 1.0), (0.8, 2.0)])
def test_perturb2d_distribution_and_priors(k1, pf):
    """Perturb a cloud at angle 0: the increments follow von Mises with kappa =
    vms_kappa(min(1, k1 pf)) (uniform when that is below 0.1), rows stay unit,
    and the returned priors are 1/pdfVMS of the perturbed cloud."""
    nImg, mR, mT = 2048, 32, 9
    R = rows(np.zeros((nImg, mR)))
    tr = np.zeros((nImg, mT, 2))
    dR, dT = T(R), T(tr)
    pR = torch.empty(nImg, mR, dtype=torch.float64, device=DEV)
    pT = torch.empty(nImg, mT, dtype=torch.float64, device=DEV)
    k = T(np.full((nImg, 3), k1))
    sd = T(np.full((nImg, 2), 1.5))
    check(lib().thx_pf_perturb2d(nImg, mR, mT, ops._ptr(dR), ops._ptr(dT), ops._ptr(pR),
                                 ops._ptr(pT), ops._ptr(k), ops._ptr(sd), pf, 10.0, 1e9, 17, 3,
                                 None), "thx_pf_perturb2d")
    Rn, pRn, tn = dR.cpu().numpy(), pR.cpu().numpy(), dT.cpu().numpy()
    assert np.allclose(np.hypot(Rn[..., 0], Rn[..., 1]), 1.0, atol=1e-12)
    assert np.all(Rn[..., 2:] == 0.0)
    kappa = op.vms_kappa(min(1.0, k1 * pf))
    c, s = Rn[..., 0].ravel(), Rn[..., 1].ravel()
    want = i1(kappa) / i0(kappa) if kappa >= 0.1 else 0.0
    assert abs(c.mean() - want) < 0.01 and abs(s.mean()) < 0.01, (c.mean(), want)
    for l in range(0, nImg, 256):
        ref = op.balance_rot2d(Rn[l])
        assert np.max(np.abs(pRn[l] - ref) / ref) < 1e-9
    # translations: N(0, sd pf) steps
    assert abs(tn.std() - 1.5 * pf) < 0.05 * 1.5 * pf
    # reproducible per (seed, stream)
    dR2, dT2 = T(R), T(tr)
    check(lib().thx_pf_perturb2d(nImg, mR, mT, ops._ptr(dR2), ops._ptr(dT2), ops._ptr(pR),
                                 ops._ptr(pT), ops._ptr(k), ops._ptr(sd), pf, 10.0, 1e9, 17, 3,
                                 None), "thx_pf_perturb2d")
    assert torch.equal(dR2, dR) and torch.equal(dT2, dT)


def test_sample_set2d():
    rot, tr, pR, pT = ops.global_sample_set2d(4096, 151, 10.0, 5, DEV)
    r = rot.cpu().numpy()
    assert np.allclose(np.hypot(r[:, 0], r[:, 1]), 1.0, atol=1e-14) and np.all(r[:, 2:] == 0)
    th = np.arctan2(r[:, 1], r[:, 0])
    h, _ = np.histogram(th, bins=8, range=(-np.pi, np.pi))
    assert h.min() > 0.85 * 512 and h.max() < 1.15 * 512
    assert torch.allclose(pR, torch.full_like(pR, 1 / 4096)) and abs(float(pT.sum()) - 1) < 1e-12


# ---------------------------------------------------------------- C1 driver
N1, PF1, K1 = 64, 2, 8


def _classes(nK, seed):
    """nK half-complex 2D class projectees [nK, vdim, vdim/2+1] (blob images
    in the padded box, as the 2D Projector holds them)."""
    vdim = N1 * PF1
    rng = np.random.default_rng(seed)
    out = np.empty((nK, vdim, vdim // 2 + 1), np.complex64)
    yy, xx = np.mgrid[:vdim, :vdim] - vdim // 2
    for k in range(nK):
        img = np.zeros((vdim, vdim))
        for _ in range(6):
            cx, cy = rng.uniform(-N1 / 3, N1 / 3, 2)
            w = rng.uniform(2, 5)
            img += rng.uniform(0.5, 1.5) * np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * w * w))
        out[k] = np.fft.rfft2(np.fft.ifftshift(img)) / vdim
    return T(out)


@pytest.fixture(scope="module")
def c1():
    """C1's shape: box 64, 8 classes, 2D global sampling mS 100 -> nR 100, nT
    151; the scan ring rU 16 for a usable signal; images of known classes at
    grid poses, SNR 10."""
    cl = _classes(K1, 81)
    px = ops.PixelSet(N1, PF1, 16, 1, device=DEV)
    mS, nR, nT = ops.global_sample_sizes(100, mode=0)
    gset = [t.cpu().numpy() for t in ops.global_sample_set2d(nR, nT, 10.0, 83, DEV)]
    n = 192
    rng = np.random.default_rng(82)
    cls = rng.integers(0, K1, n)
    # grid poses of the global set (the class is decided by the scan's class
    # marginal, so off-grid images at nR 100 may land in a neighbour class);
    # translations among the 40 samples nearest the centre
    q, t = gset[0], gset[1]
    th = np.arctan2(q[:, 1], q[:, 0])[rng.integers(0, len(q), n)]
    near = np.argsort(np.linalg.norm(t, axis=1))[:40]
    tt = t[near[rng.integers(0, len(near), n)]]
    ctf = ops.ctf(T(synth.ctf_attrs(n, seed=84)), px)
    P = torch.empty(n, px.n, dtype=torch.complex64, device=DEV)
    for l in range(n):
        P[l] = ops.project2d(cl[cls[l]].contiguous(), T(np.array([[np.cos(th[l]), np.sin(th[l])]])),
                             px)[0]
    sigl = ctf * P * ops.trans_table(T(tt), px)
    dat, sig = synth.noisy_images(sigl, px.iSig, N1 // 2 + 1, snr=10.0, seed=85)
    return dict(cl=cl, px=px, gset=gset, dat=dat, ctf=ctf, sig=sig, cls=cls, th=th, tt=tt)


def _ang_err_deg(rot, th):
    """angle of the cloud's resultant vs the true angle, degrees."""
    r = rot.cpu().numpy()
    a = np.arctan2(r[:, :, 1].sum(1), r[:, :, 0].sum(1))
    d = np.angle(np.exp(1j * (a - th)))
    return np.degrees(np.abs(d))


@pytest.mark.parametrize("converge", [False, True])
def test_c1_driver_recovers_class_angle_shift(c1, converge):
    e = ex.Expectation(c1["cl"], c1["px"], c1["gset"], n_phase=10, seed=9, converge=converge,
                       mode="2d")
    rot, trans, pR, pT, score, cls, nph = e.run(c1["dat"], c1["ctf"], c1["sig"])
    cls = cls.cpu().numpy()
    acc = np.mean(cls == c1["cls"])
    assert acc >= 0.9, acc
    ok = cls == c1["cls"]
    err = _ang_err_deg(rot, c1["th"])[ok]
    assert np.median(err) < 2.0, np.median(err)
    tm = trans.mean(1).cpu().numpy()[ok]
    assert np.median(np.linalg.norm(tm - c1["tt"][ok], axis=1)) < 0.5
    r = rot.cpu().numpy()
    assert np.allclose(np.hypot(r[..., 0], r[..., 1]), 1.0, atol=1e-9) and np.all(r[..., 2:] == 0)
    assert torch.isfinite(score).all() and torch.isfinite(pR).all() and torch.isfinite(pT).all()
    nph = nph.cpu().numpy()
    if converge:
        assert nph.min() >= 11 and nph.max() <= 99, (nph.min(), nph.max())
    else:
        assert (nph == 10).all()


def test_c1_driver_reproducible_and_local_continuation(c1):
    e = ex.Expectation(c1["cl"], c1["px"], c1["gset"], n_phase=4, seed=21, mode="2d")
    a = e.run(c1["dat"], c1["ctf"], c1["sig"])
    b = e.run(c1["dat"], c1["ctf"], c1["sig"])
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    # a local search continues from that state (its class kept)
    loc = ex.Expectation(c1["cl"], c1["px"], None, n_phase=3, seed=22, search="local", mode="2d")
    state = tuple(t.clone() for t in a[:4]) + (a[5].clone(),)
    rot, trans, pR, pT, score, cls, nph = loc.run(c1["dat"], c1["ctf"], c1["sig"], state=state)
    assert torch.equal(cls, a[5])
    ok = cls.cpu().numpy() == c1["cls"]
    assert np.median(_ang_err_deg(rot, c1["th"])[ok]) < 2.0


# ------------------------------------------------------- 2D CTF search
def _ctf_table(orc, px, attrs, dD, N):
    out = []
    for l, a in enumerate(attrs):
        rf, rd, r1, r2 = orc.defocus_pre(px, a, N)
        out.append(orc.ctf_search(rd, rf, dD[l], r1, r2, a[7], a[6]))
    return np.stack(out).astype(np.float32)


@pytest.mark.parametrize("nR,nT,nD", [(10, 9, 3), (20, 5, 9), (7, 3, 1)])
def test_local_phase2d_d_matches_restatement(orc, nR, nT, nD):
    """The 2D (r, t, d) phase (thx_local_phase2d_d) per image against
    orc.local_phase2d_d on the same CTF table: dvp 1e-5, marginals 1e-3."""
    N, pf, nK, nImg = 32, 2, 2, 4
    vdim = N * pf
    px = orc.pixel_set(N, pf, 12, 1)
    gpx = ops.PixelSet(N, pf, 12, 1, device=DEV)
    cl = _classes2(nK, N, pf, 40 + nD)
    rng = np.random.default_rng(nR + nD)
    cls = rng.integers(0, nK, nImg).astype(np.int32)
    th = rng.uniform(0, 2 * np.pi, (nImg, 1)) + rng.standard_normal((nImg, nR)) * 0.1
    rot = np.stack([np.cos(th), np.sin(th)], -1)
    trans = rng.standard_normal((nImg, nT, 2))
    attrs = synth.ctf_attrs(nImg, seed=nR)
    dD = 1 + rng.standard_normal((nImg, nD)) * 0.02
    ctfD = _ctf_table(orc, px, attrs, dD, N)
    dat = (rng.standard_normal((nImg, px.n)) + 1j * rng.standard_normal((nImg, px.n))).astype(np.complex64)
    sig = -rng.uniform(0.5, 2, (nImg, px.n)).astype(np.float32)
    pC = rng.uniform(0.5, 1, nImg)
    pR, pT, pD = (rng.uniform(0.1, 1, (nImg, n)) for n in (nR, nT, nD))
    outs = [torch.empty(nImg, n, dtype=torch.float32, device=DEV) for n in (1, nR, nT, nD, 1)]
    dvp = torch.empty(nImg, nR, nT, nD, dtype=torch.float32, device=DEV)
    args = [T(x) for x in (cl, cls, rot, trans, pC, pR, pT, pD, dat, ctfD, sig)]
    p = ops._ptr
    check(lib().thx_local_phase2d_d(p(args[0]), vdim, pf, p(args[1]), p(args[2]), nR, p(args[3]),
                                    nT, nD, p(args[4]), p(args[5]), p(args[6]), p(args[7]),
                                    p(args[8]), p(args[9]), p(args[10]), p(gpx.d_iCol),
                                    p(gpx.d_iRow), px.n, N, nImg, *[p(o) for o in outs], p(dvp),
                                    None, 0, None), "thx_local_phase2d_d")
    wC, wR, wT, wD, base = [o.cpu().numpy() for o in outs]
    d = dvp.cpu().numpy()
    for l in range(nImg):
        rc, rr, rt, rdd, rb, rdv = orc.local_phase2d_d(cl[cls[l]], vdim, pf, rot[l], trans[l], pC[l],
                                                       pR[l], pT[l], pD[l], dat[l], ctfD[l], sig[l],
                                                       px, N)
        assert np.max(np.abs(d[l] - rdv) / np.abs(rdv)) < 1e-5
        assert abs(base[l, 0] - rb) <= 1e-5 * abs(rb)
        for a, b in ((wR[l], rr), (wT[l], rt), (wD[l], rdd)):
            m = b >= 1e-4 * b.max()
            assert np.all(np.abs(a - b)[m] <= 1e-3 * b[m])
        assert abs(wC[l, 0] - rc) <= 1e-3 * rc


def _classes2(nK, N, pf, seed):
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


def test_ctf_search_2d_through_interface_forwards(orc):
    """ExpectLocalPreI2D with cSearch (devdefO / devfreQ, Interface.h:89-105):
    the calpoint's CTF per defocus sample and the 2D (r, t, d) phase through
    ExpectLocalM, against orc.local_phase2d_d on orc.ctf_search's table."""
    import ctypes
    vp = ctypes.c_void_p
    Pn = lambda a: a.ctypes.data_as(vp)
    N, pf = 32, 2
    vdim = N * pf
    px = orc.pixel_set(N, pf, 12, 1)
    L = lib()
    npxl, mR, mT, mD, cpy, gpu = px.n, 20, 5, 4, 2, 0
    iCol, iRow = px.iCol.copy(), px.iRow.copy()
    dCol, dRow = vp(), vp()
    assert L.thx_ExpectPreidx(gpu, ctypes.byref(dCol), ctypes.byref(dRow), Pn(iCol), Pn(iRow), npxl) == 0
    attrs = synth.ctf_attrs(3, seed=14)
    attrs[:, 7] = [0.0, 0.2, -0.1]
    pre = [orc.defocus_pre(px, a, N) for a in attrs]
    freq = pre[0][0]
    defO = np.ascontiguousarray(np.stack([q[1] for q in pre]))
    dF = vp()
    assert L.thx_ExpectPrefre(gpu, ctypes.byref(dF), Pn(freq), npxl) == 0
    mgr = vp()
    assert L.thx_tex_create(0, vdim, gpu, ctypes.byref(mgr)) == 0
    cl = _classes2(2, N, pf, 77)
    rng = np.random.default_rng(6)
    dat = (rng.standard_normal((3, npxl)) + 1j * rng.standard_normal((3, npxl))).astype(np.complex64)
    datf = np.ascontiguousarray(dat).view(np.float32)
    sig = -rng.uniform(0.5, 2, (3, npxl)).astype(np.float32)
    dD, dC, dO, dS = vp(), vp(), vp(), vp()
    assert L.thx_ExpectLocalIn(gpu, ctypes.byref(dD), ctypes.byref(dC), ctypes.byref(dO),
                               ctypes.byref(dS), npxl, cpy, 2) == 0
    mcp = vp()
    assert L.thx_calpoint_create(0, 2, gpu, mR, mT, mD, npxl, ctypes.byref(mcp)) == 0, L.thx_last_error()
    wC, wR, wT, wD = (np.zeros(n, np.float32) for n in (1, mR, mT, mD))
    for img in range(3):
        k = img % 2
        clk = np.ascontiguousarray(cl[k]).view(np.float32)
        assert L.thx_ExpectLocalV2D(gpu, mgr, Pn(clk), (vdim // 2 + 1) * vdim) == 0
        slot = img % cpy
        assert L.thx_ExpectLocalP(gpu, dD, dC, dO, dS, Pn(datf), None, Pn(defO), Pn(sig), slot, img,
                                  npxl, 1) == 0, L.thx_last_error()
        th = rng.uniform(0, 2 * np.pi) + rng.standard_normal(mR) * 0.1
        rot4 = np.zeros((mR, 4))
        rot4[:, 0], rot4[:, 1] = np.cos(th), np.sin(th)
        t = np.ascontiguousarray(rng.standard_normal((mT, 2)))
        pR = rng.uniform(0.5, 1.5, mR)
        pT = np.full(mT, 1.0 / mT)
        pD = rng.uniform(0.5, 1.5, mD)
        d = 1 + rng.standard_normal(mD) * 0.02
        assert L.thx_ExpectLocalRTD(gpu, mcp, Pn(pR), Pn(pT), Pn(pD), Pn(t), Pn(rot4), Pn(d)) == 0
        a = attrs[img]
        assert L.thx_ExpectLocalPreI2D(gpu, slot, mgr, mcp, dO, dF, dCol, dRow, float(a[7]),
                                       float(a[6]), float(pre[img][2]), float(pre[img][3]), pf, N,
                                       vdim, npxl, 1) == 0, L.thx_last_error()
        oldC = 0.9
        assert L.thx_ExpectLocalM(gpu, slot, mcp, dD, dC, dS, Pn(wC), Pn(wR), Pn(wT), Pn(wD), oldC,
                                  npxl) == 0, L.thx_last_error()
        ctfD = orc.ctf_search(pre[img][1], freq, d, pre[img][2], pre[img][3], a[7], a[6])
        rC, rR, rT, rDd, rb, rd = orc.local_phase2d_d(cl[k], vdim, pf, rot4[:, :2], t, oldC, pR, pT,
                                                      pD, dat[img], ctfD, sig[img], px, N)
        for got, want in ((wR, rR), (wT, rT), (wD, rDd)):
            m = want >= 1e-4 * want.max()
            assert np.max(np.abs(got - want)[m] / want[m]) < 1e-3
        assert abs(wC[0] - rC) <= 1e-3 * abs(rC)
    assert L.thx_calpoint_destroy(mcp) == 0
    assert L.thx_ExpectLocalFin(gpu, ctypes.byref(dD), ctypes.byref(dC), ctypes.byref(dO),
                                ctypes.byref(dF), ctypes.byref(dS), 1) == 0
    assert L.thx_tex_destroy(mgr) == 0
    assert L.thx_ExpectFreeIdx(gpu, ctypes.byref(dCol), ctypes.byref(dRow)) == 0


def test_c1_ctf_search_refines_defocus(c1):
    """SEARCH_TYPE_CTF in MODE_2D from the global search's particle state:
    images made with a scaled defocus pull their defocus particles toward the
    true factor; the class, angle and priors stay sound."""
    n = c1["dat"].shape[0]
    rng = np.random.default_rng(91)
    attrs = synth.ctf_attrs(n, seed=84)              # the attributes the fixture's CTF used
    dtrue = 1 + rng.uniform(-0.03, 0.03, n)
    a_true = attrs.copy()
    a_true[:, 2:4] *= dtrue[:, None]
    px = c1["px"]
    ctf = ops.ctf(T(a_true), px)
    P = torch.empty(n, px.n, dtype=torch.complex64, device=DEV)
    for l in range(n):
        P[l] = ops.project2d(c1["cl"][c1["cls"][l]].contiguous(),
                             T(np.array([[np.cos(c1["th"][l]), np.sin(c1["th"][l])]])), px)[0]
    sigl = ctf * P * ops.trans_table(T(c1["tt"]), px)
    dat, sig = synth.noisy_images(sigl, px.iSig, N1 // 2 + 1, snr=10.0, seed=92)
    g = ex.Expectation(c1["cl"], px, c1["gset"], n_phase=10, seed=9, mode="2d")
    state = g.run(dat, ops.ctf(T(attrs), px), sig)
    e = ex.Expectation(c1["cl"], px, None, search="ctf", converge=True, seed=5, mLD=9, mode="2d")
    st = tuple(t.clone() for t in state[:4]) + (state[5].clone(),)
    rot, trans, pR, pT, score, cls, nph, d, pD = e.run_ctf(dat, T(attrs), sig, st)
    ok = cls.cpu().numpy() == c1["cls"]
    assert ok.mean() >= 0.9
    dm = d.mean(1).cpu().numpy()
    err0 = np.median(np.abs(1 - dtrue)[ok])
    err = np.median(np.abs(dm - dtrue)[ok])
    assert err < 0.6 * err0, (err, err0)
    assert torch.allclose(pD.sum(1), torch.ones(n, dtype=torch.float64, device=DEV), rtol=1e-9)
    assert torch.isfinite(score).all() and torch.isfinite(d).all()
    assert np.median(_ang_err_deg(rot, c1["th"])[ok]) < 2.0
    nph = nph.cpu().numpy()
    assert nph.min() >= 3 and nph.max() <= 99
