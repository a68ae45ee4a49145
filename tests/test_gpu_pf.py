"""GPU parity of the expectation driver's own resampling kernel (k_pf_resample
through thx_pf_resample): Particle::resample (src/Particle.cpp:1291-1478) with
and without the support shuffle (src/Particle.cpp:1298, 2202-2300)."""
import numpy as np
import pytest
import torch

from thunder_amd import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def T(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


def _inputs(rng, nImg, nIn, shared_w=False):
    w = rng.uniform(0.1, 1, nIn if shared_w else (nImg, nIn))
    u = (rng.uniform(0.01, 1, (nImg, nIn)) ** 4).astype(np.float32)
    return w, u


@pytest.mark.parametrize("nIn,nOut,shared", [(125, 125, False), (2000, 125, True), (151, 9, True),
                                             (9, 9, False), (1, 4, False)])
def test_unshuffled_matches_oracle(orc, nIn, nOut, shared):
    rng = np.random.default_rng(nIn)
    nImg = 6
    w, u = _inputs(rng, nImg, nIn, shared)
    anc, wo, imax, perm, u0 = (x.cpu().numpy() for x in ops.pf_resample(T(w), T(u), nOut, seed=3,
                                                                         shuffle=False))
    for l in range(nImg):
        wl = w if shared else w[l]
        assert np.array_equal(perm[l], np.arange(nIn))
        assert 0.0 < u0[l] < 1.0 / nOut
        ra, rw, ri = orc.resample(wl, u[l].astype(np.float64), nOut, u0[l])
        assert np.array_equal(anc[l], ra)
        assert np.allclose(wo[l], rw, rtol=1e-12, atol=0)
        assert imax[l] == ri


@pytest.mark.parametrize("nIn", [1, 151, 1500, 2048, 2049, 5000])
def test_shuffled_is_a_permutation_and_matches_oracle(orc, nIn):
    """Shuffled support: perm is a permutation; ancestors, iMax and priors are
    the oracle's resampling of the permuted support mapped back through perm."""
    rng = np.random.default_rng(100 + nIn)
    nImg, nOut = 5, 125
    w, u = _inputs(rng, nImg, nIn)
    anc, wo, imax, perm, u0 = (x.cpu().numpy() for x in ops.pf_resample(T(w), T(u), nOut, seed=9,
                                                                         stream_id=7))
    for l in range(nImg):
        p = perm[l]
        assert np.array_equal(np.sort(p), np.arange(nIn)), "not a permutation"
        ra, rw, ri = orc.resample(w[l][p], u[l][p].astype(np.float64), nOut, u0[l])
        assert np.array_equal(anc[l], p[ra])
        assert np.allclose(wo[l], rw, rtol=1e-12, atol=0)
        assert imax[l] == p[ri]
    if nIn > 8:
        # different images draw different permutations
        assert not np.array_equal(perm[0], perm[1])


def test_shuffle_is_uniform():
    """Position of every element after the shuffle is uniform (chi-square over
    4096 images at nIn = 8, 64 cells: 5-sigma bound on the statistic)."""
    nImg, nIn = 4096, 8
    w = np.ones(nIn)
    u = np.ones((nImg, nIn), np.float32)
    *_, perm, _ = ops.pf_resample(T(w), T(u), 4, seed=21)
    perm = perm.cpu().numpy()
    counts = np.zeros((nIn, nIn))
    for pos in range(nIn):
        counts[pos] = np.bincount(perm[:, pos], minlength=nIn)
    exp = nImg / nIn
    chi2 = ((counts - exp) ** 2 / exp).sum()
    dof = (nIn - 1) ** 2
    assert chi2 < dof + 5 * np.sqrt(2 * dof), chi2


def _philox_4x32_10(seed, a, b, c, d):
    """Philox-4x32-10 as thunder_amd/csrc/common.h's Philox::next() draws it:
    counter (a, b, c, d), key = the 64-bit seed's halves; numpy uint64
    arithmetic on arrays of counters."""
    M0, M1, W0, W1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), 0x9E3779B9, 0xBB67AE85
    m32 = np.uint64(0xFFFFFFFF)
    x = [np.asarray(v, np.uint64) & m32 for v in (a, b, c, d)]
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0, p1 = M0 * x[0], M1 * x[2]
        x = [((p1 >> np.uint64(32)) ^ x[1] ^ np.uint64(k0)) & m32, p1 & m32,
             ((p0 >> np.uint64(32)) ^ x[3] ^ np.uint64(k1)) & m32, p0 & m32]
        k0, k1 = (k0 + W0) & 0xFFFFFFFF, (k1 + W1) & 0xFFFFFFFF
    return x


@pytest.mark.parametrize("nIn", [8, 100, 256, 300, 2000])
def test_shuffle_is_the_sort_of_its_philox_keys(nIn):
    """The support permutation is the ascending order of the 64-bit keys
    (32 random bits << 32 | entry): entry i's bits are component i / 64 % 4
    of draw i / 256 of the Philox stream (image, stream id, 0x5f1e0000 | i %
    64) -- whichever sort the kernel runs for this size (the LDS network below
    64 entries, the wave's registers up to 256, k_pf_shuffle_perm above)."""
    nImg, seed, sid = 3, 1234567, 77
    rng = np.random.default_rng(nIn)
    w = rng.uniform(0.5, 1.0, nIn)
    u = rng.uniform(0.1, 1.0, (nImg, nIn)).astype(np.float32)
    *_, perm, _ = ops.pf_resample(T(w), T(u), 4, seed=seed, stream_id=sid)
    perm = perm.cpu().numpy()
    i = np.arange(nIn)
    for l in range(nImg):
        x = _philox_4x32_10(seed, np.full(nIn, l), np.full(nIn, sid), 0x5F1E0000 | (i % 64), i // 256)
        bits = np.choose((i // 64) % 4, x)
        keys = (bits.astype(np.uint64) << np.uint64(32)) | i.astype(np.uint64)
        assert np.array_equal(perm[l], np.argsort(keys, kind="stable")), (nIn, l)


def test_seed_and_stream_determine_the_draw():
    rng = np.random.default_rng(1)
    w, u = _inputs(rng, 4, 300)
    a = [x.cpu().numpy() for x in ops.pf_resample(T(w), T(u), 50, seed=5, stream_id=1)]
    b = [x.cpu().numpy() for x in ops.pf_resample(T(w), T(u), 50, seed=5, stream_id=1)]
    c = [x.cpu().numpy() for x in ops.pf_resample(T(w), T(u), 50, seed=5, stream_id=2)]
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert not np.array_equal(a[3], c[3])
