"""CPU pinning of the 2D restatement (f4; oracle/thunder_oracle.c
orc_project2d / orc_insert2d_batch): bilinear interpolation is exact on
fields affine in (i, j), the Hermitian fold conjugates, and the insert is the
adjoint of the projection (sum_q T[q] g[q] = sum_samples ctf^2 w g(sample))."""
import numpy as np

from thunder_amd import ops


def _affine_img(vdim, a, b, c):
    """img[j][i] = a + b i + c j (j signed, stored wrapped), complex."""
    nc = vdim // 2 + 1
    i = np.arange(nc)[None, :]
    j = np.fft.fftfreq(vdim, 1.0 / vdim)[:, None]
    return (a + b * i + c * j).astype(np.complex64)


def test_project2d_exact_on_affine_fields(orc):
    N, pf = 32, 2
    vdim = N * pf
    px = orc.pixel_set(N, pf, 12, 1)
    img = _affine_img(vdim, 1.5 + 0.5j, 0.25 - 0.1j, -0.75 + 0.3j)
    rng = np.random.default_rng(2)
    for _ in range(5):
        th = rng.uniform(0, 2 * np.pi)
        cs = np.array([np.cos(th), np.sin(th)])
        got = orc.project2d(img, vdim, pf, cs, px)
        x = (cs[0] * px.iCol * pf - cs[1] * px.iRow * pf).astype(np.float32)
        y = (cs[1] * px.iCol * pf + cs[0] * px.iRow * pf).astype(np.float32)
        neg = ~(x >= 0)
        xf, yf = np.where(neg, -x, x), np.where(neg, -y, y)
        val = (1.5 + 0.5j) + (0.25 - 0.1j) * xf + (-0.75 + 0.3j) * yf
        ref = np.where(neg, np.conj(val), val)
        assert np.allclose(got, ref, atol=1e-4 * np.abs(ref).max())


def test_insert2d_is_the_adjoint_of_project2d(orc):
    N, pf = 32, 2
    vdim = N * pf
    px = orc.pixel_set(N, pf, 12, 1)
    rng = np.random.default_rng(3)
    nImg, mReco = 3, 4
    dat = (rng.standard_normal((nImg, px.n)) + 1j * rng.standard_normal((nImg, px.n))).astype(np.complex64)
    ctf = rng.uniform(-1, 1, (nImg, px.n)).astype(np.float32)
    th = rng.uniform(0, 2 * np.pi, (nImg, mReco))
    rot = np.stack([np.cos(th), np.sin(th)], -1)
    trans = np.zeros((nImg, mReco, 2))
    off = np.zeros((nImg, 2))
    w = np.full(nImg, 0.25, np.float32)
    F, T, O, cnt = orc.insert2d_batch(vdim, pf, dat, ctf, rot, trans, off, w, None, px, N)
    assert cnt[0] == nImg * mReco
    g = rng.standard_normal((vdim, vdim // 2 + 1)).astype(np.float32)
    lhs = float(np.sum(T.astype(np.float64) * g.reshape(-1)))
    rhs = 0.0
    for l in range(nImg):
        for m in range(mReco):
            proj = orc.project2d(g.astype(np.complex64), vdim, pf, rot[l, m], px).real
            rhs += float(np.sum(ctf[l].astype(np.float64) ** 2 * w[l] * proj))
    assert abs(lhs - rhs) <= 1e-4 * abs(rhs)


# ---- MODE_2D particle statistics (oracle/particle.py): known answers
def _rows(th):
    return np.stack([np.cos(th), np.sin(th), 0 * th, 0 * th], 1)


def test_infer_vms_symmetric_cloud():
    from oracle import particle as op
    th0, d = 0.7, np.array([-0.3, -0.1, 0.0, 0.1, 0.3])
    mu, k = op.infer_vms(_rows(th0 + d))
    assert np.allclose(mu, [np.cos(th0), np.sin(th0)], atol=1e-14)
    assert abs(k - (1 - np.cos(d).mean())) < 1e-14
    assert abs(op.cal_vari_rot2d(_rows(th0 + d)) - k) < 1e-15


def test_pdf_vms_is_a_density():
    """pdfVMS integrates to 1 over the circle in both of its branches
    (the exact von Mises density below kappa 5; the wrapped Gaussian of
    |x - mu| above, to its approximation error)."""
    from oracle import particle as op
    th = np.linspace(0, 2 * np.pi, 20001)[:-1]
    for k, tol in ((0.9, 1e-10), (0.5, 1e-10), (0.2, 1e-10), (0.05, 2e-2)):
        p = op.pdf_vms(_rows(th), np.array([np.cos(1.0), np.sin(1.0)]), k)
        assert abs(p.mean() * 2 * np.pi - 1) < tol, k


def test_sample_vms_mean_resultant():
    """Best & Fisher's sampler: E cos = I1(kappa) / I0(kappa), E sin = 0."""
    from scipy.special import i0, i1
    from oracle import particle as op
    rng = np.random.default_rng(3)
    for kappa in (0.5, 2.0, 8.0, 40.0):
        x = op.sample_vms(rng, kappa, 20000)
        assert np.allclose(np.hypot(x[:, 0], x[:, 1]), 1.0, atol=1e-12)
        assert abs(x[:, 0].mean() - i1(kappa) / i0(kappa)) < 0.012, kappa
        assert abs(x[:, 1].mean()) < 0.012, kappa
    u = op.sample_vms(rng, 0.05, 20000)          # below 0.1: uniform directions
    assert abs(u[:, 0].mean()) < 0.015 and abs(u[:, 1].mean()) < 0.015


def test_vms_kappa_and_balance_weights():
    from oracle import particle as op
    assert op.vms_kappa(1.0) == 0.0                  # k = 1: uniform (Particle::reset)
    k = 0.1                                           # kappa from k: the inverse of R(kappa) approx
    assert op.vms_kappa(k) > 4.0
    rng = np.random.default_rng(1)
    R = _rows(rng.normal(0.3, 0.4, 64))
    w = op.balance_rot2d(R)
    mu, kk = op.infer_vms(R)
    p = op.pdf_vms(R, mu, kk)
    assert abs(w.sum() - 1) < 1e-12 and np.allclose(w * p, (w * p)[0], rtol=1e-12)


def test_peak_factor_rot2d():
    from oracle import particle as op
    u = np.arange(1, 101, dtype=np.float64)           # largest 100, the 50th largest (index 50) 50
    assert op.peak_factor_rot2d(u) == 0.5
    u = np.concatenate([[1000.0], np.ones(9)])        # index 5 of 10: 1 / 1000
    assert op.peak_factor_rot2d(u) == 1e-3


def test_local_phase2d_d_reduces_to_the_direct_likelihood(orc):
    """orc_local_phase2d_d: dvp[r][t][d] is logDataVSPrior of the 2D
    projection at rotation r, translation t and CTF row d (to 1e-6: numpy's
    complex64 product of translation and projection rounds differently from
    the C loop), and the marginals are the normalisation of
    src/Optimiser.cpp:1383-1402 with the defocus axis (float64 to 1e-5)."""
    N, pf = 32, 2
    vdim = N * pf
    px = orc.pixel_set(N, pf, 10, 1)
    rng = np.random.default_rng(4)
    img = (rng.standard_normal((vdim, vdim // 2 + 1)) + 1j * rng.standard_normal((vdim, vdim // 2 + 1))
           ).astype(np.complex64)
    nR, nT, nD = 5, 4, 3
    th = rng.uniform(0, 2 * np.pi, nR)
    rot = np.stack([np.cos(th), np.sin(th)], 1)
    trans = rng.standard_normal((nT, 2))
    dat = (rng.standard_normal(px.n) + 1j * rng.standard_normal(px.n)).astype(np.complex64)
    ctfD = rng.uniform(-1, 1, (nD, px.n)).astype(np.float32)
    sig = -rng.uniform(0.5, 2, px.n).astype(np.float32)
    pR, pT, pD = rng.uniform(0.1, 1, nR), rng.uniform(0.1, 1, nT), rng.uniform(0.1, 1, nD)
    wC, wR, wT, wD, base, dvp = orc.local_phase2d_d(img, vdim, pf, rot, trans, 0.7, pR, pT, pD, dat,
                                                    ctfD, sig, px, N)
    for r in range(nR):
        pri = orc.project2d(img, vdim, pf, rot[r], px)
        for t in range(nT):
            pt = (orc.translate(px, *trans[t], N) * pri).astype(np.complex64)
            for d in range(nD):
                want = orc.logdatavs(dat, pt, ctfD[d], sig)
                assert abs(dvp[r, t, d] - want) <= 1e-6 * abs(want)
    e = np.exp(dvp.astype(np.float64) - dvp.max())
    assert abs(base - dvp.max()) == 0
    rR = np.einsum("rtd,t,d->r", e, pT, pD) * 0.7
    rT = np.einsum("rtd,r,d->t", e, pR, pD) * 0.7
    rDd = np.einsum("rtd,r,t->d", e, pR, pT) * 0.7
    rC = np.einsum("rtd,r,t,d->", e, pR, pT, pD)
    for got, want in ((wR, rR), (wT, rT), (wD, rDd)):
        assert np.allclose(got, want, rtol=1e-5)
    assert abs(wC - rC) <= 1e-5 * rC
