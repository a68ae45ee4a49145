"""Pins the CPU restatement (oracle/) against independent known answers.

The reference has no golden vectors and cannot be built here (DESIGN.md,
"parity unpinned"), so each restated routine is checked against an
independent derivation: float64 closed forms, analytic interpolation cases
(trilinear interpolation is exact on affine fields), the gather/scatter
adjoint identity, and the pixel counts SURVEY.md §8 lists for the
BASELINE.json configs.
"""
import math

import numpy as np
import pytest

from thunder_amd import synth

from stacks import np_dvp, small_stack


def np_pixel_set(N, rU, rL):
    """Independent float64 restatement of src/Optimiser.cpp:8008-8040."""
    out = []
    r = rU + 1
    for j in range(int(-r), int(math.ceil(r))):
        if not j < r:
            continue
        for i in range(0, int(r) + 1):
            if i == 0 and j < 0:
                continue
            u = np.float32(i * i + j * j)
            if np.float32(rL * rL) <= u < np.float32(rU * rU):
                v = int(np.rint(math.hypot(i, j)))
                if rL <= v < rU:
                    out.append((i, j, v))
    return out


# (N, rL, rU, nPxl) from SURVEY.md §8 (global and full-resolution radii)
SURVEY_COUNTS = [(64, 0, 7, 69), (64, 0, 30, 1367), (128, 0, 12, 211), (128, 0, 62, 5941),
                 (256, 1, 24, 870), (256, 1, 126, 24746), (200, 1, 19, 542), (200, 1, 98, 14930),
                 (512, 3, 46, 3242), (512, 3, 254, 100928)]


@pytest.mark.parametrize("N,rL,rU,n", SURVEY_COUNTS)
def test_pixel_set_counts(orc, N, rL, rU, n):
    px = orc.pixel_set(N, 2, rU, rL)
    assert px.n == n


@pytest.mark.parametrize("N,rL,rU", [(32, 0, 10), (64, 1, 24.5), (48, 2, 17)])
def test_pixel_set_matches_independent(orc, N, rL, rU):
    px = orc.pixel_set(N, 2, rU, rL)
    ref = np_pixel_set(N, rU, rL)
    assert px.n == len(ref)
    assert np.array_equal(px.iCol, [a for a, _, _ in ref])
    assert np.array_equal(px.iRow, [b for _, b, _ in ref])
    assert np.array_equal(px.iSig, [c for _, _, c in ref])
    assert np.array_equal(px.iPxl, [(b if b >= 0 else b + N) * (N // 2 + 1) + a for a, b, _ in ref])


def np_ctf(attr, N, iCol, iRow):
    ps, volt, dU, dV, th, Cs, ac, phs = [float(a) for a in attr]
    lam = 12.2643247 / math.sqrt(volt * (1 + volt * 0.978466e-6))
    u = np.hypot(iCol / (ps * N), iRow / (ps * N))
    ang = np.arctan2(iRow, iCol) - th
    df = -(dU + dV + (dU - dV) * np.cos(2 * ang)) / 2
    ki = math.pi * lam * df * u ** 2 + math.pi / 2 * Cs * lam ** 3 * u ** 4 - phs
    return -math.sqrt(1 - ac * ac) * np.sin(ki) + ac * np.cos(ki)


def test_ctf_closed_form(orc):
    px = orc.pixel_set(128, 2, 60, 0)
    for a in synth.ctf_attrs(4, seed=3):
        got = orc.ctf(px, a, 128)
        ref = np_ctf(a, 128, px.iCol.astype(np.float64), px.iRow.astype(np.float64))
        assert np.max(np.abs(got - ref)) < 2e-3   # FP32 phase of |ki| up to ~1e2 rad


def test_translate_closed_form(orc):
    px = orc.pixel_set(64, 2, 30, 0)
    for tx, ty in [(0.0, 0.0), (3.25, -7.5), (-12.0, 9.75)]:
        got = orc.translate(px, tx, ty, 64)
        ref = np.exp(-2j * np.pi * (px.iCol * tx + px.iRow * ty) / 64)
        assert np.max(np.abs(got - ref)) < 1e-5
        src = (np.arange(px.n) + 1j * np.arange(px.n)[::-1]).astype(np.complex64) / px.n
        got2 = orc.translate_src(px, src, tx, ty, 64)
        assert np.max(np.abs(got2 - src * ref)) < 1e-5


def test_rotate3d_matches_quaternion_algebra(orc):
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(0)
    for q in synth.uniform_quaternions(20, rng):
        m = orc.rotate3d(q).reshape(3, 3).T           # column-major -> row-major
        ref = Rotation.from_quat([q[1], q[2], q[3], q[0]]).as_matrix()
        assert np.allclose(m, ref, atol=1e-14)


def affine_volume(vdim, coef):
    """Half-complex volume whose (signed-index) field is affine: trilinear
    interpolation of it is exact, so the projection has a closed form."""
    i = np.arange(vdim // 2 + 1)
    j = np.fft.fftfreq(vdim, 1.0 / vdim)
    k = np.fft.fftfreq(vdim, 1.0 / vdim)
    K, J, I = np.meshgrid(k, j, i, indexing="ij")
    re = coef[0] + coef[1] * I + coef[2] * J + coef[3] * K
    im = coef[4] + coef[5] * I + coef[6] * J + coef[7] * K
    return (re + 1j * im).astype(np.complex64), coef


def affine_at(coef, x, y, z):
    return (coef[0] + coef[1] * x + coef[2] * y + coef[3] * z) + 1j * (
        coef[4] + coef[5] * x + coef[6] * y + coef[7] * z)


def test_project_exact_on_affine_field(orc):
    N, pf = 32, 2
    vdim = N * pf
    vol, coef = affine_volume(vdim, [0.5, 0.01, -0.02, 0.03, -0.1, 0.02, 0.015, -0.01])
    px = orc.pixel_set(N, pf, N // 2 - 1, 0)
    rng = np.random.default_rng(1)
    for q in synth.uniform_quaternions(6, rng):
        m = orc.rotate3d(q)
        got = orc.project3d(vol, vdim, pf, m, px)
        R = m.reshape(3, 3).T
        c = R @ np.stack([px.iCol * pf, px.iRow * pf, np.zeros(px.n)])
        c = c.astype(np.float32).astype(np.float64)
        fold = c[0] < 0
        cc = np.where(fold, -c, c)
        ref = affine_at(coef, *cc)
        ref = np.where(fold, np.conj(ref), ref)
        assert np.max(np.abs(got - ref)) < 1e-5 * np.max(np.abs(ref))


def test_insert_is_adjoint_of_project(orc):
    """Re<insert(v), U> == sum Re(v conj(project(U))) and the T analogue."""
    N, pf = 24, 2
    vdim = N * pf
    rng = np.random.default_rng(2)
    size = (vdim // 2 + 1) * vdim * vdim
    U = (rng.standard_normal(size) + 1j * rng.standard_normal(size)).astype(np.complex64)
    Ur = rng.standard_normal(size).astype(np.float32)
    px = orc.pixel_set(N, pf, N // 2 - 1, 0)
    q = synth.uniform_quaternions(1, rng)[0]
    m = orc.rotate3d(q)
    v = (rng.standard_normal(px.n) + 1j * rng.standard_normal(px.n)).astype(np.complex64)
    ctf = np.ones(px.n, np.float32)
    F = np.zeros(2 * size, np.float32)
    T = np.zeros(size, np.float32)
    orc.insert3d(F, T, vdim, v, ctf, m, 1.0, px)
    Fc = F.view(np.complex64)
    p = orc.project3d(U, vdim, pf, m, px)
    lhs = np.real(np.vdot(U.astype(np.complex128), Fc.astype(np.complex128)))
    rhs = np.sum(np.real(v.astype(np.complex128) * np.conj(p.astype(np.complex128))))
    assert abs(lhs - rhs) < 1e-4 * max(1.0, abs(rhs))
    pr = orc.project3d(Ur.astype(np.complex64), vdim, pf, m, px)
    assert abs(np.dot(T.astype(np.float64), Ur) - np.sum(np.real(pr))) < 1e-4 * px.n


def test_dvp_and_global_weights(orc):
    s = small_stack(orc)
    d = orc.dvp_global(s["vol"], s["vdim"], s["pf"], s["quat"], s["trans"], s["dat"], s["ctf"],
                       s["sig"], s["px"], s["N"], threads=2)
    ref = np_dvp(s, orc)
    assert np.max(np.abs(d - ref) / np.abs(ref)) < 1e-5
    nR, nT = len(s["quat"]), len(s["trans"])
    pR = np.full(nR, 1.0 / nR)
    pT = np.random.default_rng(5).uniform(0.5, 1.5, nT)
    pT /= pT.sum()
    wC, wR, wT, base = orc.weights_global(d, pR, pT)
    e = np.exp(ref - ref.max(axis=(1, 2), keepdims=True))
    assert np.allclose(base, ref.max(axis=(1, 2)), rtol=1e-6)
    assert np.allclose(wR.reshape(-1, nR), (e * pT).sum(2), rtol=1e-4, atol=1e-7)
    assert np.allclose(wT.reshape(-1, nT), (e * pR[:, None]).sum(1), rtol=1e-4, atol=1e-7)
    assert np.allclose(wC, (e * pR[:, None] * pT).sum((1, 2)), rtol=1e-4)


def test_local_phase_matches_global_formulas(orc):
    s = small_stack(orc, nImg=1, nR=9, nT=5)
    nR, nT = 9, 5
    rng = np.random.default_rng(9)
    pR = rng.uniform(0.5, 1, nR); pR /= pR.sum()
    pT = rng.uniform(0.5, 1, nT); pT /= pT.sum()
    pC = 0.7
    wC, wR, wT, base, dvp = orc.local_phase(s["vol"], s["vdim"], s["pf"], s["quat"], s["trans"], pC,
                                             pR, pT, s["dat"][0], s["ctf"][0], s["sig"][0], s["px"],
                                             s["N"])
    ref = np_dvp(s, orc)[0]
    assert np.max(np.abs(dvp - ref) / np.abs(ref)) < 1e-5
    e = np.exp(ref - ref.max())
    assert abs(base - ref.max()) < 1e-5 * abs(ref.max())
    assert np.allclose(wR, pC * (e * pT).sum(1), rtol=1e-4)
    assert np.allclose(wT, pC * (e * pR[:, None]).sum(0), rtol=1e-4)
    assert np.isclose(wC, (e * pR[:, None] * pT).sum(), rtol=1e-4)


def np_resample(w, u, n_out, u0):
    ww = w * u
    ww = ww / ww.sum()
    cdf = np.cumsum(ww)
    cdf = cdf / cdf[-1]
    anc = []
    i = 0
    for j in range(n_out):
        uj = u0 + j / n_out
        while uj > cdf[i]:
            i += 1
        anc.append(i)
    anc = np.array(anc)
    wo = 1.0 / u[anc]
    return anc, wo / wo.sum()


@pytest.mark.parametrize("n_in,n_out", [(125, 125), (2000, 125), (9, 9), (151, 9), (1, 4)])
def test_resample_systematic(orc, n_in, n_out):
    rng = np.random.default_rng(n_in)
    w = rng.uniform(0.1, 1, n_in)
    u = rng.uniform(0, 1, n_in).astype(np.float32).astype(np.float64) ** 4
    u0 = rng.uniform(0, 1.0 / n_out)
    anc, wo, imax = orc.resample(w, u, n_out, u0)
    ra, rw = np_resample(w, u, n_out, u0)
    assert np.array_equal(anc, ra)
    assert np.allclose(wo, rw, rtol=1e-12)
    assert imax == int(np.argmax(u))


def test_fsc_identities(orc):
    vdim = 32
    rng = np.random.default_rng(4)
    shape = (vdim, vdim, vdim // 2 + 1)
    A = (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(np.complex64)
    B = (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(np.complex64)
    n = vdim // 2
    assert np.allclose(orc.fsc(A, A, vdim, n), 1.0, atol=1e-6)
    assert np.allclose(orc.fsc(A, -A, vdim, n), -1.0, atol=1e-6)
    f = orc.fsc(A, B, vdim, n)
    assert np.all(np.abs(f[2:]) < 0.3)
    # independent numpy shell sum
    i = np.arange(vdim // 2 + 1)
    j = np.fft.fftfreq(vdim, 1.0 / vdim)
    K, J, I = np.meshgrid(j, j, i, indexing="ij")
    u = np.rint(np.sqrt(I ** 2 + J ** 2 + K ** 2)).astype(int)
    Ad, Bd = A.astype(np.complex128), B.astype(np.complex128)
    ref = []
    for s in range(n):
        m = u == s
        num = np.sum(np.real(Ad[m] * np.conj(Bd[m])))
        den = np.sqrt(np.sum(np.abs(Ad[m]) ** 2) * np.sum(np.abs(Bd[m]) ** 2))
        ref.append(num / den)
    assert np.allclose(f, ref, atol=1e-6)


def test_insert_batch_recentre_and_direction(orc):
    s = small_stack(orc, nImg=2)
    px = s["px"]
    rng = np.random.default_rng(3)
    q = synth.uniform_quaternions(6, rng).reshape(2, 3, 4)
    t = rng.standard_normal((2, 3, 2))
    off = rng.standard_normal((2, 2))
    w = np.array([1 / 3, 1 / 3], np.float32)
    F, T, O, cnt = orc.insert_batch(s["vdim"], s["pf"], s["dat"], s["ctf"], q, t, off, w, px, s["N"])
    assert cnt == 6
    Oref = np.zeros(3)
    for l in range(2):
        for m in range(3):
            R = orc.rotate3d(q[l, m]).reshape(3, 3).T
            Oref += -(R @ np.array([*(t[l, m] - off[l]), 0.0]))
    assert np.allclose(O, Oref, atol=1e-12)
    assert np.sum(T) > 0 and np.isfinite(F).all()


# ---------------------------------------------------------------- a10 stats
def test_infer_acg_recovers_the_acg_matrix():
    """Tyler's fixed point on n samples of ACG(S) estimates S up to scale
    (trace 4 by construction of the iteration)."""
    from oracle import particle as op
    rng = np.random.default_rng(41)
    S = np.diag([1.0, 0.3, 0.1, 0.05])
    x = rng.standard_normal((20000, 4)) @ np.sqrt(S)
    Q = x / np.linalg.norm(x, axis=1, keepdims=True)
    A = op.infer_acg(Q)
    assert abs(np.trace(A) - 4.0) < 1e-9
    assert np.allclose(A, S * 4 / np.trace(S), atol=0.03)
    k = op.cal_vari_rot(Q)
    assert np.allclose(k, [0.3, 0.1, 0.05], rtol=0.1)


def test_calvari_of_a_degenerate_cloud():
    """All particles equal (a resampled sharp posterior): the reference's loop
    leaves with A = 4 q q^T after the singular inverse turns the criterion to
    NaN, and the de-meaned spreads are 0 (the scan floors then apply)."""
    from oracle import particle as op
    q = np.array([0.5, 0.5, -0.5, 0.5])
    Q = np.tile(q, (125, 1))
    assert np.allclose(op.infer_acg(Q), 4 * np.outer(q, q))
    assert np.allclose(op.cal_vari_rot(Q), 0.0)


def test_balance_and_peak_closed_forms():
    from oracle import particle as op
    rng = np.random.default_rng(42)
    x = rng.standard_normal((4000, 4))
    Q = x / np.linalg.norm(x, axis=1, keepdims=True)
    w = op.balance_rot(Q)                 # near-uniform cloud: A ~ I, pdf ~ 1
    assert np.allclose(w * len(w), 1.0, atol=0.2)
    u = np.arange(1, 17, dtype=np.float64)             # 16 values: u_(16/8) = 14
    assert op.peak_factor_rot(u) == 0.5                # 14/16 clamped to 0.5
    u2 = np.array([100.0] + [1.0] * 15)
    pk = op.peak_factor_rot(u2)
    assert pk == 0.01
    assert np.allclose(op.keep_half_height(u2, pk), [99.0] + [0.0] * 15)
