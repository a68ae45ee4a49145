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
                                             (130, 3, 1, 0), (12, 4, 7, 1)])
def test_local_phase_d(orc, stack, nR, nT, nD, layout):
    s = stack
    px = dev_pixels(s)
    nImg = 4
    quat, trans, ctfD, pC, pR, pT, pD = phase_inputs(s, orc, nImg, nR, nT, nD, seed=nR + nD)
    vol = T(s["vol"])
    cells = ops.volume_cells(vol) if layout else None
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
