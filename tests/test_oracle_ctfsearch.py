"""Pins the CTF-search restatement (SEARCH_TYPE_CTF) against independent
known answers: the per-defocus CTF of src/Optimiser.cpp:1252-1271 is the
CTF of src/CTF.cpp at a scaled defocus; the (r, t, d) phase with one defocus
sample reduces to the phase without CTF search; its likelihoods and
marginals follow the float64 formulas; the CTF-search insert at unit
defocus factors is the ordinary insert.
"""
import numpy as np

from oracle import particle
from thunder_amd import synth

from stacks import small_stack


def test_ctf_search_is_ctf_at_scaled_defocus(orc):
    s = small_stack(orc, nImg=1)
    px, N = s["px"], s["N"]
    attrs = synth.ctf_attrs(3, seed=4)
    attrs[:, 7] = [0.0, 0.3, -0.2]        # phase shifts
    for a in attrs:
        freq, dfo, k1, k2 = orc.defocus_pre(px, a, N)
        assert np.allclose(freq, np.hypot(px.iCol, px.iRow) / N / a[0], rtol=1e-6)
        d = np.array([0.97, 1.0, 1.013])
        got = orc.ctf_search(dfo, freq, d, k1, k2, a[7], a[6])
        for iD, dd in enumerate(d):
            b = a.copy()
            b[2:4] = a[2:4] * dd
            # the two wavelength constants differ by 2.2e-7 relative (quirk q5)
            assert np.max(np.abs(got[iD] - orc.ctf(px, b, N))) < 5e-5


def np_dvp_d(s, orc, quat, trans, dat, ctfD, sig):
    px = s["px"]
    rot = np.stack([orc.project3d(s["vol"], s["vdim"], s["pf"], orc.rotate3d(q), px)
                    for q in quat]).astype(np.complex128)
    tra = np.exp(-2j * np.pi * (np.outer(trans[:, 0], px.iCol) +
                                np.outer(trans[:, 1], px.iRow)) / s["N"])
    pri = tra[None, :, None, :] * rot[:, None, None, :]            # [r][t][1][i]
    e = dat.astype(np.complex128) - ctfD.astype(np.float64)[None, None] * pri
    return np.sum(sig.astype(np.float64) * np.abs(e) ** 2, axis=-1)  # [r][t][d]


def test_local_phase_d_formulas(orc):
    s = small_stack(orc, nImg=1, nR=7, nT=4)
    nR, nT, nD = 7, 4, 3
    rng = np.random.default_rng(5)
    a = synth.ctf_attrs(1, seed=2)[0]
    freq, dfo, k1, k2 = orc.defocus_pre(s["px"], a, s["N"])
    ctfD = orc.ctf_search(dfo, freq, np.array([0.98, 1.0, 1.02]), k1, k2, a[7], a[6])
    pR, pT, pD = (rng.uniform(0.5, 1, n) for n in (nR, nT, nD))
    pC = 0.8
    wC, wR, wT, wD, base, dvp = orc.local_phase_d(s["vol"], s["vdim"], s["pf"], s["quat"],
                                                   s["trans"], pC, pR, pT, pD, s["dat"][0], ctfD,
                                                   s["sig"][0], s["px"], s["N"])
    ref = np_dvp_d(s, orc, s["quat"], s["trans"], s["dat"][0], ctfD, s["sig"][0])
    assert np.max(np.abs(dvp - ref) / np.abs(ref)) < 1e-5
    e = np.exp(ref - ref.max())
    assert abs(base - ref.max()) < 1e-5 * abs(ref.max())
    assert np.allclose(wR, pC * np.einsum("rtd,t,d->r", e, pT, pD), rtol=1e-4)
    assert np.allclose(wT, pC * np.einsum("rtd,r,d->t", e, pR, pD), rtol=1e-4)
    assert np.allclose(wD, pC * np.einsum("rtd,r,t->d", e, pR, pT), rtol=1e-4)
    assert np.isclose(wC, np.einsum("rtd,r,t,d->", e, pR, pT, pD), rtol=1e-4)


def test_local_phase_d_one_sample_is_the_plain_phase(orc):
    s = small_stack(orc, nImg=1, nR=6, nT=5)
    rng = np.random.default_rng(8)
    pR, pT = rng.uniform(0.5, 1, 6), rng.uniform(0.5, 1, 5)
    args = (s["vol"], s["vdim"], s["pf"], s["quat"], s["trans"], 0.6, pR, pT)
    wC, wR, wT, base, dvp = orc.local_phase(*args, s["dat"][0], s["ctf"][0], s["sig"][0],
                                             s["px"], s["N"])
    wC2, wR2, wT2, wD2, base2, dvp2 = orc.local_phase_d(*args, np.ones(1), s["dat"][0],
                                                        s["ctf"][:1], s["sig"][0], s["px"], s["N"])
    assert np.array_equal(dvp, dvp2[:, :, 0]) and base == base2
    assert np.array_equal(wR, wR2) and np.array_equal(wT, wT2) and wC == wC2
    assert np.isclose(wD2[0], 0.6 * wC, rtol=1e-6)


def test_insert_batch_d_unit_defocus_is_the_plain_insert(orc):
    s = small_stack(orc, N=16, nImg=3)
    rng = np.random.default_rng(2)
    nImg, mReco = 3, 4
    attrs = synth.ctf_attrs(nImg, seed=9)
    ctf = np.stack([orc.ctf(s["px"], a, s["N"]) for a in attrs])
    quat = synth.uniform_quaternions(nImg * mReco, rng).reshape(nImg, mReco, 4)
    trans = rng.standard_normal((nImg, mReco, 2))
    offS = rng.standard_normal((nImg, 2)) * 0.3
    w = np.full(nImg, 1.0 / mReco, np.float32)
    F, T, O, c = orc.insert_batch(s["vdim"], s["pf"], s["dat"][:nImg], ctf, quat, trans, offS, w,
                                  s["px"], s["N"])
    F2, T2, O2, c2 = orc.insert_batch_d(s["vdim"], s["pf"], s["dat"][:nImg], attrs,
                                        np.ones((nImg, mReco)), quat, trans, offS, w, s["px"],
                                        s["N"])
    assert np.array_equal(F, F2) and np.array_equal(T, T2) and np.array_equal(O, O2) and c == c2
    # a defocus factor changes T by the squared CTF at that defocus
    F3, T3, _, _ = orc.insert_batch_d(s["vdim"], s["pf"], s["dat"][:nImg], attrs,
                                      np.full((nImg, mReco), 1.05), quat, trans, offS, w, s["px"],
                                      s["N"])
    assert not np.allclose(T3, T2)
    assert np.isclose(T3.sum(), sum(
        mReco * w[l] * np.sum(orc.ctf(s["px"], np.r_[a[:2], a[2:4] * 1.05, a[4:]], s["N"]) ** 2)
        for l, a in enumerate(attrs)), rtol=1e-4)


def test_defocus_statistics_closed_forms():
    d = np.array([0.99, 1.0, 1.02, 1.005, 0.985])
    assert np.isclose(particle.cal_vari_defocus(d), np.std(d, ddof=1))
    assert particle.cal_vari_defocus(d[:1]) == 0.0
    w = particle.balance_defocus(d)
    m, sd = d.mean(), np.std(d, ddof=1)
    ref = 1.0 / (np.exp(-0.5 * ((d - m) / sd) ** 2) / (sd * np.sqrt(2 * np.pi)))
    assert np.allclose(w, ref / ref.sum(), rtol=1e-12)
    assert np.allclose(particle.balance_defocus(np.ones(4)), 0.25)
