"""f2 on the GPU: a synthetic particle stack written as an MRC2014 stack plus
a .thu table, read back (thunder_amd.io), preprocessed on the device
(thx_img_stats / thx_img_finish / thx_remask / thx_img_gather /
thx_ctf_image: Optimiser::initImg, reMaskImg, allocPreCal, GCTFinit) against
the numpy restatement (oracle/preprocess.py), then through thx_expectation
(the round trip: the poses the stack was made at come back)."""
import numpy as np
import pytest
import torch

from oracle import preprocess as opp
from thunder_amd import expectation as ex
from thunder_amd import ingest, io, ops, synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
N, PF, NIMG, PIX, MASK_A = 64, 2, 96, 1.32, 34.0


def T(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


@pytest.fixture(scope="module")
def written(tmp_path_factory):
    """Real-space images centred as on disk: the inverse FFT of ctf x shifted
    projection at grid poses of a global sample set, plus white noise."""
    d = tmp_path_factory.mktemp("stack")
    vol = synth.projectee(synth.blob_volume(N, seed=31, device=DEV), PF)
    full = ops.PixelSet(N, PF, N // 2 - 1, 0, device=DEV)
    gset = synth.global_sample_set(1500, seed=32)
    q, t, _, _ = gset
    rng = np.random.default_rng(33)
    ir = rng.integers(0, len(q), NIMG)
    near = np.argsort(np.linalg.norm(t, axis=1))[:20]
    it = near[rng.integers(0, len(near), NIMG)]
    attr = synth.ctf_attrs(NIMG, seed=34, pixel_size=PIX)
    ctf = ops.ctf(T(attr), full)
    P = ops.project3d(vol, ops.rotmat(T(q[ir])), full) * ops.trans_table(T(t[it]), full) * ctf
    grid = torch.zeros(NIMG, N * (N // 2 + 1), dtype=torch.complex64, device=DEV)
    grid[:, torch.as_tensor(full.iPxl.astype(np.int64), device=DEV)] = P
    # the pixel set is the half plane without i == 0, j < 0: fill those by symmetry
    g = grid.reshape(NIMG, N, N // 2 + 1)
    g[:, N // 2 + 1:, 0] = torch.conj(g[:, 1:N // 2, 0].flip(1))
    rl = torch.fft.irfft2(g, s=(N, N)).cpu().numpy()
    scale = float(rl.std())
    rl /= scale
    rl += rng.standard_normal(rl.shape) * 0.05
    centred = np.roll(rl, (N // 2, N // 2), axis=(1, 2)).astype(np.float32)
    io.write_mrc(d / "stack.mrcs", centred, pixel_size=PIX)
    ca = attr[:, 1:8].astype(np.float64)
    table = io.thu_table(NIMG, [f"{k + 1:06d}@stack.mrcs" for k in range(NIMG)], ca)
    io.write_thu(d / "particles.thu", table)
    return dict(dir=str(d), vol=vol, gset=gset, qtrue=q[ir], centred=centred, attr=attr,
                scale=scale)


def test_preprocess_matches_restatement(written):
    w = written
    table = io.read_thu(w["dir"] + "/particles.thu")
    imgs = io.load_images(table, w["dir"])
    assert np.array_equal(imgs, w["centred"])
    r = MASK_A / PIX
    norm, st = ingest.image_stats(T(imgs), True, r)
    ref = [opp.stats_and_normalise(opp.load(x), r) for x in imgs]
    rn = np.stack([x[0] for x in ref])
    rs = np.stack([x[1] for x in ref])
    assert np.max(np.abs(norm.cpu().numpy() - rn)) <= 1e-5 * np.abs(rn).max()
    assert np.allclose(st.cpu().numpy(), rs, rtol=1e-5, atol=1e-6)
    std_n = float(st[:, 2].double().mean())
    ft, oft = ingest.finish(norm.clone(), r, std_n)
    for l in range(0, NIMG, 17):
        rf, rof = opp.finish(rn[l], r, std_n)
        assert np.max(np.abs(ft[l].cpu().numpy() - rf)) <= 2e-5 * np.abs(rf).max()
        assert np.max(np.abs(oft[l].cpu().numpy() - rof)) <= 2e-5 * np.abs(rof).max()
    # reMaskImg on device vs the restatement
    before = ft.cpu().numpy()
    ingest.remask(ft, r)
    for l in range(0, NIMG, 23):
        rr = opp.remask(before[l].astype(np.complex128), N, r)
        assert np.max(np.abs(ft[l].cpu().numpy() - rr)) <= 2e-5 * np.abs(rr).max()
    # allocPreCal's gather and GCTFinit's CTF images
    px = ops.PixelSet(N, PF, N // 4, 1, device=DEV)
    dat = ingest.gather(ft, px.iPxl).cpu().numpy()
    assert np.array_equal(dat, ft.cpu().numpy().reshape(NIMG, -1)[:, px.iPxl])
    ci = ingest.ctf_images(T(w["attr"]), N).cpu().numpy().reshape(NIMG, -1)
    assert np.allclose(ci[:, px.iPxl], ops.ctf(T(w["attr"]), px).cpu().numpy(), rtol=0, atol=1e-6)


def test_stack_round_trip_through_expectation(written):
    """MRC + .thu -> Stack (device preprocessing) -> pixel batch ->
    thx_expectation: the grid poses the stack was made at come back."""
    w = written
    table = io.read_thu(w["dir"] + "/particles.thu")
    stack = ingest.Stack.from_thu(table, w["dir"], PIX, MASK_A, DEV)
    assert 0.9 < stack.std_n < 1.1
    px = ops.PixelSet(N, PF, 12, 1, device=DEV)
    # white noise of sd 0.05 scale per pixel: sd 0.05 scale N per Fourier coefficient
    sig_rcp = -0.5 / (N * N * (0.05 * w["scale"]) ** 2)
    dat, ctf, sig = stack.pixel_batch(px, sig_rcp=np.full(px.n, sig_rcp, np.float32))
    # back to the projectee's scale: the stack was divided by its sd (scale),
    # each image by its background sd (stats[:, 1]) and all by stdN (the
    # intensity-scale correction that would do this is outside the path)
    f = (w["scale"] * stack.stats[:, 1] * stack.std_n).to(torch.complex64)
    dat = (dat * f[:, None]).contiguous()
    e = ex.Expectation(w["vol"], px, w["gset"], n_phase=4, seed=5)
    quat = e.run(dat, ctf, sig)[0]
    c = (ex.cloud_mode(quat) * T(w["qtrue"])).sum(-1).abs().clamp(max=1)
    err = torch.rad2deg(2 * torch.acos(c))
    assert float(err.median()) < 3.0, float(err.median())
