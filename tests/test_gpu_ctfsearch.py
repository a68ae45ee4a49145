"""GPU parity of the CTF-search path (SEARCH_TYPE_CTF) against the CPU
restatement: the defocus precalculation and kernel_CalCTFL twin, the local
phase over (rotation, translation, defocus) triples in both volume layouts,
and the CTF-search insert.

Tolerances as tests/test_gpu_parity.py: CTF 5e-5 absolute (FP32 rounding of
the reference formula), dvp 1e-5 relative, marginals 1e-3 relative on
entries >= 1e-4 of the image maximum, F / T 1e-5 of max.
"""
import numpy as np
import pytest
import torch

from stacks import small_stack
from thunder_amd import ops, synth

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def T(a, dtype=None):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).to(DEV)


@pytest.fixture(scope="module")
def stack(orc):
    return small_stack(orc, N=32, nImg=6, nR=12, nT=11, seed=7)


def dev_pixels(s):
    return ops.PixelSet(s["N"], s["pf"], s["rU"], s["rL"], device=DEV)


def test_defocus_pre_and_ctf_search(orc, stack):
    s = stack
    px = dev_pixels(s)
    nImg, nD = 4, 5
    attrs = synth.ctf_attrs(nImg, seed=3)
    attrs[:, 7] = [0.0, 0.25, -0.1, 0.5]
    dD = 1 + np.random.default_rng(1).standard_normal((nImg, nD)) * 0.01
    freq, dfo, k1, k2 = ops.defocus_pre(T(attrs), px)
    ctfD = ops.ctf_search(dfo, freq, T(dD), k1, k2, T(attrs)).cpu().numpy()
    freq, dfo, k1, k2 = (x.cpu().numpy() for x in (freq, dfo, k1, k2))
    for l, a in enumerate(attrs):
        rf, rd, r1, r2 = orc.defocus_pre(s["px"], a, s["N"])
        assert np.max(np.abs(freq - rf)) <= 1e-7 * np.max(rf)
        assert np.max(np.abs(dfo[l] - rd)) <= 2e-6 * np.max(np.abs(rd))
        assert k1[l] == np.float32(r1) and abs(k2[l] - r2) <= 1e-6 * abs(r2)
        ref = orc.ctf_search(rd, rf, dD[l], r1, r2, a[7], a[6])
        assert np.max(np.abs(ctfD[l] - ref)) < 5e-5


def phase_inputs(s, orc, nImg, nR, nT, nD, seed, spread=None):
    rng = np.random.default_rng(seed)
    if spread is None:
        quat = synth.uniform_quaternions(nImg * nR, rng).reshape(nImg, nR, 4)
    else:
        quat = synth.clustered_quaternions(nImg, nR, spread, rng)
    trans = rng.standard_normal((nImg, nT, 2)) * 2
    attrs = synth.ctf_attrs(nImg, seed=seed + 1)
    dD = 1 + rng.standard_normal((nImg, nD)) * 0.02
    ctfD = []
    for l, a in enumerate(attrs):
        rf, rd, r1, r2 = orc.defocus_pre(s["px"], a, s["N"])
        ctfD.append(orc.ctf_search(rd, rf, dD[l], r1, r2, a[7], a[6]))
    ctfD = np.stack(ctfD).astype(np.float32)
    pC = rng.uniform(0.5, 1, nImg)
    pR = rng.uniform(0.1, 1, (nImg, nR))
    pT = rng.uniform(0.1, 1, (nImg, nT))
    pD = rng.uniform(0.1, 1, (nImg, nD))
    return quat, trans, ctfD, pC, pR, pT, pD


@pytest.mark.parametrize("nR,nT,nD,layout", [(10, 9, 3, 0), (10, 9, 3, 1), (20, 5, 9, 0),
                                             (130, 3, 1, 0), (12, 4, 7, 1), (20, 5, 9, 1),
                                             (130, 3, 1, 1)])
def test_local_phase_d(orc, stack, nR, nT, nD, layout):
    s = stack
    px = dev_pixels(s)
    nImg = 4
    quat, trans, ctfD, pC, pR, pT, pD = phase_inputs(s, orc, nImg, nR, nT, nD, seed=nR + nD)
    vol = T(s["vol"])
    cells = ops.volume_cells(vol) if layout == 1 else None
    wC, wR, wT, wD, base, d = ops.local_phase_d(vol, T(quat), T(trans), T(pC), T(pR), T(pT), T(pD),
                                                T(s["dat"][:nImg]), T(ctfD), T(s["sig"][:nImg]),
                                                px, want_dvp=True, cells=cells)
    wC, wR, wT, wD, base, d = [x.cpu().numpy() for x in (wC, wR, wT, wD, base, d)]
    for l in range(nImg):
        rc, rr, rt, rdd, rb, rdv = orc.local_phase_d(s["vol"], s["vdim"], s["pf"], quat[l],
                                                     trans[l], pC[l], pR[l], pT[l], pD[l],
                                                     s["dat"][l], ctfD[l], s["sig"][l], s["px"],
                                                     s["N"])
        assert np.max(np.abs(d[l] - rdv) / np.abs(rdv)) < 1e-5
        assert abs(base[l] - rb) <= 1e-5 * abs(rb)
        for a, b in ((wR[l], rr), (wT[l], rt), (wD[l], rdd)):
            m = b >= 1e-4 * b.max()
            assert np.all(np.abs(a - b)[m] <= 1e-3 * b[m])
        assert abs(wC[l] - rc) <= 1e-3 * rc


def test_local_phase_d_one_sample_matches_plain_phase(orc, stack):
    """nD = 1 through the CTF-search kernel (bias on the MFMA) agrees with
    the phase without CTF search (bias on the VALU)."""
    s = stack
    px = dev_pixels(s)
    nImg, nR, nT = 5, 40, 9
    quat, trans, _, pC, pR, pT, _ = phase_inputs(s, orc, nImg, nR, nT, 1, seed=4, spread=3.0)
    args = (T(s["vol"]), T(quat), T(trans), T(pC), T(pR), T(pT))
    r1 = ops.local_phase(*args, T(s["dat"][:nImg]), T(s["ctf"][:nImg]), T(s["sig"][:nImg]), px,
                         want_dvp=True)
    r2 = ops.local_phase_d(*args, T(np.ones((nImg, 1))), T(s["dat"][:nImg]),
                           T(s["ctf"][:nImg, None, :]), T(s["sig"][:nImg]), px, want_dvp=True)
    d1, d2 = r1[4].cpu().numpy(), r2[5].cpu().numpy()[..., 0]
    assert np.max(np.abs(d1 - d2) / np.abs(d1)) < 1e-5
    for a, b in ((r1[1], r2[1]), (r1[2], r2[2])):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        m = a >= 1e-4 * a.max(axis=1, keepdims=True)
        assert np.all(np.abs(a - b)[m] <= 1e-3 * a[m])
    assert torch.allclose(r2[3][:, 0], r1[0] * T(pC, torch.float32), rtol=1e-4)


@pytest.mark.parametrize("mD", [1, 9, 40])
def test_pf_defocus_ops(mD):
    from oracle import particle
    nImg = 64
    d = torch.zeros(nImg, mD, dtype=torch.float64, device=DEV)
    pD = torch.zeros_like(d)
    sd = torch.zeros(nImg, dtype=torch.float64, device=DEV)
    ops.pf_defocus("init", d, pD, arg=0.01, seed=3)
    dn, pn = d.cpu().numpy(), pD.cpu().numpy()
    assert np.all(np.abs(dn - 1) < 0.08)
    if mD == 40:
        assert abs(np.std(dn - 1) - 0.01) < 0.001
    for l in range(nImg):
        assert np.allclose(pn[l], particle.balance_defocus(dn[l]), rtol=1e-12, atol=0)
    ops.pf_defocus("vari", d, sd=sd)
    sn = sd.cpu().numpy()
    for l in range(nImg):
        assert np.isclose(sn[l], particle.cal_vari_defocus(dn[l]), rtol=1e-12, atol=0)
    d0 = dn.copy()
    ops.pf_defocus("perturb", d, pD, sd, arg=0.5, seed=3, stream_id=1)
    dn, pn = d.cpu().numpy(), pD.cpu().numpy()
    if mD > 1:
        step = (dn - d0) / (sn[:, None] * 0.5)
        assert abs(np.std(step) - 1) < 0.2 and abs(np.mean(step)) < 0.2
    else:
        assert np.array_equal(dn, d0)       # s = 0 for a single sample
    for l in range(nImg):
        assert np.allclose(pn[l], particle.balance_defocus(dn[l]), rtol=1e-12, atol=0)


def test_ctf_search_driver_refines_defocus():
    """SEARCH_TYPE_CTF from a particle state near the true pose: the defocus
    particles move toward each image's true defocus factor, the pose stays
    refined, the priors are normalised and the stopping rule runs."""
    from thunder_amd import expectation as ex
    N, rU, n = 64, 16, 128
    vol = synth.projectee(synth.blob_volume(N, seed=31, device=DEV), 2)
    px = ops.PixelSet(N, 2, rU, 1, device=DEV)
    rng = np.random.default_rng(32)
    qtrue = synth.uniform_quaternions(n, rng)
    ttrue = rng.standard_normal((n, 2))
    attrs = synth.ctf_attrs(n, seed=33)
    dtrue = 1 + rng.uniform(-0.03, 0.03, n)
    a_true = attrs.copy()
    a_true[:, 2:4] *= dtrue[:, None]
    ctf = ops.ctf(T(a_true), px)
    sigl = ctf * ops.project3d(vol, ops.rotmat(T(qtrue)), px) * ops.trans_table(T(ttrue), px)
    dat, sig = synth.noisy_images(sigl, px.iSig, N // 2 + 1, snr=5.0, seed=34)
    mR, mT = 125, 9
    e0 = rng.standard_normal((n, mR, 4)) * np.radians(1.0) / 2
    e0[..., 0] = 1.0
    e0 /= np.linalg.norm(e0, axis=-1, keepdims=True)
    w0, x0, y0, z0 = [qtrue[:, None, k] for k in range(4)]
    w1, x1, y1, z1 = [e0[..., k] for k in range(4)]
    quat = np.stack([w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1, w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
                     w0 * y1 - x0 * z1 + y0 * w1 + z0 * x1, w0 * z1 + x0 * y1 - y0 * x1 + z0 * w1], -1)
    trans = ttrue[:, None, :] + rng.uniform(-0.5, 0.5, (n, mT, 2))
    state = (T(quat), T(trans), T(np.full((n, mR), 1.0 / mR)), T(np.full((n, mT), 1.0 / mT)))
    e = ex.Expectation(vol, px, None, search="ctf", converge=True, seed=5, mLD=9)
    q, t, pR, pT, score, cls, nph, d, pD = e.run_ctf(dat, T(attrs), sig, state)
    dm = d.mean(1).cpu().numpy()
    err0 = np.median(np.abs(1 - dtrue))
    err = np.median(np.abs(dm - dtrue))
    assert err < 0.6 * err0, (err, err0)
    assert torch.allclose(pD.sum(1), torch.ones(n, dtype=torch.float64, device=DEV), rtol=1e-9)
    assert torch.allclose(pR.sum(1), torch.ones(n, dtype=torch.float64, device=DEV), rtol=1e-9)
    assert torch.isfinite(score).all() and torch.isfinite(d).all()
    nph = nph.cpu().numpy()
    assert nph.min() >= 4 and nph.max() <= 99
    qm = ex.cloud_mode(q).cpu().numpy()
    ang = np.degrees(2 * np.arccos(np.clip(np.abs(np.sum(qm * qtrue, 1)), 0, 1)))
    assert np.median(ang) < 2.0


@pytest.mark.parametrize("spread,mReco,dup", [(0.0, 6, False), (2.0, 100, True), (8.0, 150, True)])
def test_insert_ctf_search(orc, stack, spread, mReco, dup):
    """Every sample at its own defocus factor; dup: copies of 12 ancestors
    (one rotation group holds members of different defocus)."""
    s = stack
    px = dev_pixels(s)
    nImg = 4
    rng = np.random.default_rng(22)
    if spread > 0:
        quat = synth.clustered_quaternions(nImg, mReco, spread, rng)
    else:
        quat = synth.uniform_quaternions(nImg * mReco, rng).reshape(nImg, mReco, 4)
    if dup:
        anc = rng.integers(0, 12, (nImg, mReco))
        quat = np.ascontiguousarray(np.take_along_axis(quat, anc[..., None], axis=1))
    trans = rng.standard_normal((nImg, mReco, 2)) * 3
    off = rng.standard_normal((nImg, 2))
    w = np.full(nImg, 1.0 / mReco, np.float32)
    attrs = synth.ctf_attrs(nImg, seed=12)
    nD = 1 + rng.standard_normal((nImg, mReco)) * 0.02
    hm = ops.HalfMap(s["vdim"], DEV)
    ops.insert3d_ctf(hm, T(s["dat"][:nImg]), T(attrs), T(nD), T(quat), T(trans), T(off), T(w), px)
    F, Tm, O, cnt = orc.insert_batch_d(s["vdim"], s["pf"], s["dat"][:nImg], attrs, nD, quat, trans,
                                       off, w, s["px"], s["N"])
    gF = hm.F.cpu().numpy().reshape(-1)
    gT = hm.T.cpu().numpy().reshape(-1)
    assert np.max(np.abs(gF - F)) <= 1e-5 * np.max(np.abs(F))
    assert np.max(np.abs(gT - Tm)) <= 1e-5 * np.max(np.abs(Tm))
    assert np.allclose(hm.O.cpu().numpy(), O, rtol=1e-12, atol=1e-12)
    assert int(hm.counter.item()) == cnt == nImg * mReco


def test_global_sample_set_on_device():
    """a3: Particle::reset's global set from the C-ABI producer."""
    nR, nT, transS = 4000, 151, 10.0
    q, t, pR, pT = [x.cpu().numpy() for x in ops.global_sample_set(nR, nT, transS, 7, DEV)]
    assert np.allclose(np.linalg.norm(q, axis=1), 1, atol=1e-14)
    assert np.allclose(q.T @ q / nR, np.eye(4) / 4, atol=0.02)        # uniform on S^3
    assert abs(t.mean()) < 1.5 and abs(t.std() - transS) < 1.5
    assert np.allclose(pR, 1.0 / nR)
    m, s = t.mean(0), t.std(0, ddof=1)
    ref = 1.0 / (np.exp(-0.5 * (((t - m) / s) ** 2).sum(1)) / (2 * np.pi * s[0] * s[1]))
    assert np.allclose(pT, ref / ref.sum(), rtol=1e-12, atol=0)
    q2 = ops.global_sample_set(nR, nT, transS, 7, DEV)[0].cpu().numpy()
    assert np.array_equal(q, q2)
