"""Point-group symmetry on the GPU against the restatement
(oracle/symmetry.py): SYMMETRIZE_FT of F and T, Reconstructor::prepareTF,
Particle::symmetrise; C4 and D2 half-maps through insert -> prepareTF ->
reconstruct; the expectation driver with a symmetric sample set and
symmetrised particle clouds recovers the generating poses modulo the group.

Tolerances: symmetrised / prepared volumes 1e-5 of max (FP32 sums of up to
60 trilinear gathers vs float64); reconstructed maps 1e-4 of max (as the C1
test); particle counterparts 1e-12."""
import numpy as np
import pytest
import torch

from oracle import reconstruct as orc_rc
from oracle import symmetry as osym
from thunder_amd import expectation as ex
from thunder_amd import ops, synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def T_(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


def _volumes(vdim, seed):
    """F: the transform of a real volume; T: positive, |.| of one -- both
    Hermitian on the x = 0 plane, where the symmetry elements' FP32-angle
    rotations of a grid point land on either side of the fold."""
    rng = np.random.default_rng(seed)
    F = np.fft.rfftn(rng.standard_normal((vdim, vdim, vdim))).astype(np.complex64)
    quad = orc_rc._ft_quad(vdim).astype(np.float64)
    A = np.abs(np.fft.rfftn(rng.standard_normal((vdim, vdim, vdim))))
    T = ((50.0 / (1.0 + np.sqrt(quad))) * (0.8 + 0.4 * A / A.max())).astype(np.float32)
    return F, T


def _decided(vdim, R, r):
    """Voxels whose every rotated copy is clearly inside or outside the radius:
    at |R v|^2 = r^2 (grid points on the sphere, rotated by near-exact quarter
    turns) the reference's own test is decided by FP64 rounding."""
    i = np.arange(vdim // 2 + 1, dtype=np.float64)
    j = np.fft.fftfreq(vdim, 1.0 / vdim)
    K, J, I = np.meshgrid(j, j, i, indexing="ij")
    ok = np.ones(K.shape, bool)
    for M in R:
        q = ((M[0, 0] * I + M[0, 1] * J + M[0, 2] * K) ** 2 + (M[1, 0] * I + M[1, 1] * J + M[1, 2] * K) ** 2
             + (M[2, 0] * I + M[2, 1] * J + M[2, 2] * K) ** 2)
        ok &= np.abs(q - r * r) > 1e-6 * r * r
    return ok


@pytest.mark.parametrize("sym", ["C4", "D2", "T", "I1"])
def test_symmetrize_ft_matches_restatement(sym):
    vdim = 32
    F, Tm = _volumes(vdim, 3)
    R, _ = ops.symmetry(sym)
    r = 13.0
    ok = _decided(vdim, R, r)
    for V in (F, Tm):
        got = ops.symmetrize_ft(T_(V), R, r).cpu().numpy()
        ref = osym.symmetrize_ft(V, R, r)
        assert np.max(np.abs(got - ref)[ok]) <= 1e-5 * np.max(np.abs(ref)), sym


@pytest.mark.parametrize("sym", ["C1", "C4", "D2"])
def test_prepare_tf_matches_restatement(sym):
    N, pf = 16, 2
    vdim = N * pf
    F, Tm = _volumes(vdim, 5)
    R, _ = ops.symmetry(sym)
    hm = ops.HalfMap(vdim, DEV)
    hm.F.copy_(T_(F))
    hm.T.copy_(T_(Tm))
    ops.prepare_tf(hm, R, N // 2 - 2, pf)
    rF, rT = osym.prepare_tf(F, Tm, R, N // 2 - 2, pf)
    ok = _decided(vdim, R, (N // 2 - 2) * pf + 1)
    assert np.max(np.abs(hm.F.cpu().numpy() - rF)[ok]) <= 1e-5 * np.max(np.abs(rF))
    assert np.max(np.abs(hm.T.cpu().numpy() - rT)[ok]) <= 1e-5 * np.max(np.abs(rT))
    if sym == "C1":     # normalisation only: T[0] = 1
        assert abs(float(hm.T.view(-1)[0]) - 1.0) < 1e-6


@pytest.mark.parametrize("sym", ["C4", "D3", "O"])
def test_pf_symmetrise_matches_restatement(sym):
    _, Q = ops.symmetry(sym)
    rng = np.random.default_rng(9)
    nImg, mR = 5, 125
    cloud = synth.clustered_quaternions(nImg, mR, 40.0, rng)
    anchors = synth.uniform_quaternions(nImg, rng)
    # anchorMode 0: (1, 0, 0, 0); 1: given anchors
    for mode in (0, 1):
        got = ops.pf_symmetrise(T_(cloud.copy()), Q, mode, T_(anchors) if mode else None).cpu().numpy()
        for l in range(nImg):
            ref = osym.symmetrise(cloud[l], Q, anchors[l] if mode else (1, 0, 0, 0))
            assert np.allclose(got[l], ref, rtol=0, atol=1e-12)
    # anchorMode 2: a particle drawn from each cloud -- the result is the
    # restatement's for one of the cloud's own particles
    got = ops.pf_symmetrise(T_(cloud.copy()), Q, 2, None, seed=7, stream_id=11).cpu().numpy()
    for l in range(nImg):
        assert any(np.allclose(got[l], osym.symmetrise(cloud[l], Q, cloud[l][j]), rtol=0, atol=1e-12)
                   for j in range(mR))


@pytest.mark.parametrize("sym", ["C4", "D2"])
def test_symmetric_halfmap_insert_prepare_reconstruct(orc, sym):
    """A C4 / D2 map: images at random poses inserted (GPU binned insert vs
    the C restatement), prepareTF (normalise + symmetrise F and T), the
    reconstruction solve -- the map matches the restatement chain to 1e-4 of
    max and is itself symmetric."""
    N, pf = 32, 2
    vdim = N * pf
    R, _ = ops.symmetry(sym)
    vol = synth.projectee(synth.blob_volume(N, n_blobs=5, seed=8, sym_R=R), pf).numpy()
    pxh = orc.pixel_set(N, pf, N // 2 - 2, 0)
    px = ops.PixelSet(N, pf, N // 2 - 2, 0, device=DEV)
    rng = np.random.default_rng(31)
    nImg, mReco = 200, 4
    qt = synth.uniform_quaternions(nImg, rng)
    dat = np.stack([orc.project3d(vol, vdim, pf, orc.rotate3d(q), pxh) for q in qt]).astype(np.complex64)
    ctf = np.ones((nImg, pxh.n), np.float32)
    quat = synth.clustered_quaternions(nImg, mReco, 1.0, rng)
    quat[:, 0] = qt
    trans = rng.standard_normal((nImg, mReco, 2)) * 0.3
    off = np.zeros((nImg, 2))
    w = np.full(nImg, 1.0 / mReco, np.float32)
    hm = ops.HalfMap(vdim, DEV)
    ops.insert3d(hm, T_(dat), T_(ctf), T_(quat), T_(trans), T_(off), T_(w), px)
    F, Tm, O, cnt = orc.insert_batch(vdim, pf, dat, ctf, quat, trans, off, w, pxh, N)
    F = F.reshape(vdim, vdim, vdim // 2 + 1)
    Tm = Tm.reshape(vdim, vdim, vdim // 2 + 1)
    maxR = N // 2 - 2
    ops.prepare_tf(hm, R, maxR, pf)
    rF, rT = osym.prepare_tf(F, Tm, R, maxR, pf)
    ok = _decided(vdim, R, maxR * pf + 1)
    assert np.max(np.abs(hm.F.cpu().numpy() - rF)[ok]) <= 1e-5 * np.max(np.abs(rF))
    assert np.max(np.abs(hm.T.cpu().numpy() - rT)[ok]) <= 1e-5 * np.max(np.abs(rT))
    # the solve on the restatement's own prepared F / T where the device's
    # differs at the rounding-decided sphere voxels
    hm.F.copy_(T_(rF.astype(np.complex64)))
    hm.T.copy_(T_(rT.astype(np.float32)))
    got, _, it, _ = ops.reconstruct(hm, N, pf, max_radius=maxR)
    ref, rit, _ = orc_rc.reconstruct(rF.astype(np.complex64), rT.astype(np.float32), N, pf,
                                     max_radius=maxR)
    got = got.cpu().numpy()
    assert it == rit
    assert np.max(np.abs(got - ref)) <= 1e-4 * np.max(np.abs(ref))
    # the map is symmetric: V(R x) = V(x) on the grid for these 90 / 180 degree groups
    c = np.fft.fftfreq(N, 1.0 / N).astype(int)
    Z, Y, X = np.meshgrid(c, c, c, indexing="ij")
    for M in np.rint(R).astype(int):
        x = M[0, 0] * X + M[0, 1] * Y + M[0, 2] * Z
        y = M[1, 0] * X + M[1, 1] * Y + M[1, 2] * Z
        z = M[2, 0] * X + M[2, 1] * Y + M[2, 2] * Z
        rot = got[z % N, y % N, x % N]
        # F / T symmetric inside the sphere; the shell the radius test
        # decides by rounding and the FP32-angle rotations leave ~2e-3
        assert np.max(np.abs(rot - got)) <= 5e-3 * np.max(np.abs(got))


def _angle_mod_group(q, qt, Q):
    """Angle (deg) between q and the nearest symmetry copy s qt of the true pose."""
    best = abs(float(q @ qt))
    for s in Q:
        best = max(best, abs(float(q @ osym.quat_mul(s, qt))))
    return np.degrees(2 * np.arccos(min(1.0, best)))


def test_expectation_with_symmetry_recovers_poses():
    """Global search at box 64 on a C4 map with the group's sample set
    (nR = mS / 4, symmetrised towards the identity) and the driver's
    symmetrised particle clouds: the poses come back modulo C4, and every
    global sample is the copy of itself nearest the identity."""
    N, pf, sym = 64, 2, "C4"
    R, Q = ops.symmetry(sym)
    vol = synth.projectee(synth.blob_volume(N, n_blobs=10, seed=4, sym_R=R, device=DEV), pf)
    # rU 12: the global search's resolution (at rU 20 the 1500-rotation grid
    # is too coarse for both the C4 and the C1 search)
    px = ops.PixelSet(N, pf, 12, 1, device=DEV)
    mS, nR, nT = ops.global_sample_sizes(1500, n_sym_elem=len(Q))
    assert (mS, nR) == (6000, 1500)
    gq, gt, gpR, gpT = ops.global_sample_set(nR, nT, 10.0, 5, DEV, sym=sym)
    gqn = gq.cpu().numpy()
    for q in gqn[:200]:
        assert np.allclose(q, osym.counterpart(q, Q), atol=1e-12)
    rng = np.random.default_rng(6)
    nImg = 96
    qt = synth.uniform_quaternions(nImg, rng)
    tt = rng.standard_normal((nImg, 2)) * 2
    ctf = ops.ctf(T_(synth.ctf_attrs(nImg, seed=7)), px)
    sig = ctf * ops.project3d(vol, ops.rotmat(T_(qt)), px) * ops.trans_table(T_(tt), px)
    dat, sigRcp = synth.noisy_images(sig, px.iSig, N // 2 + 1, snr=20.0, seed=8)
    gset = tuple(x.cpu().numpy() for x in (gq, gt, gpR, gpT))
    e = ex.Expectation(vol, px, gset, n_phase=10, seed=3, sym=sym)
    quat, trans, pR, pT, score = e.run(dat.to(DEV), ctf, sigRcp.to(DEV))[:5]
    mode = ex.cloud_mode(quat).cpu().numpy()
    err = np.array([_angle_mod_group(mode[l], qt[l], Q) for l in range(nImg)])
    assert torch.isfinite(quat).all()
    # the C1 search of the same images over all of SO(3) (4x the rotations)
    g1 = tuple(x.cpu().numpy() for x in ops.global_sample_set(4 * nR, nT, 10.0, 5, DEV))
    q1 = ex.Expectation(vol, px, g1, n_phase=10, seed=3).run(dat.to(DEV), ctf, sigRcp.to(DEV))[0]
    m1 = ex.cloud_mode(q1).cpu().numpy()
    err1 = np.array([_angle_mod_group(m1[l], qt[l], Q) for l in range(nImg)])
    assert np.median(err) < 3.0, (np.median(err), np.median(err1))
    assert np.mean(err > 15) <= np.mean(err1 > 15) + 0.06, (np.mean(err > 15), np.mean(err1 > 15))
