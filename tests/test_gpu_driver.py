"""The expectation driver's modes (thx_expectation, ABI 3): K-class
classification (config C4's multi-reference projector path), local search from
a caller's particle state (config C5's mode), the per-image vari-decrease
stopping rule and the inferACG perturbation mean.

Parity of the scan across classes is pinned against the restatement
(orc.weights_global with kIdx / nK, the running baseline of
src/Optimiser.cpp:834-894); the end-to-end particle filter is pinned by the
properties the reference's loop guarantees (its GSL generator is urandom
seeded): images made at grid poses of a known class at high SNR come back in
that class and pose."""
import numpy as np
import pytest
import torch

from thunder_amd import expectation as ex
from thunder_amd import ops, synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def T(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


def angle_deg(qa, qb):
    c = (qa * qb).sum(-1).abs().clamp(max=1)
    return torch.rad2deg(2 * torch.acos(c))


def grid_images(vols, px, gset, n_img, seed, cls=None, snr=20.0):
    """Images of class cls[l] at grid poses of gset (high SNR)."""
    q, t, _, _ = gset
    rng = np.random.default_rng(seed)
    ir = rng.integers(0, len(q), n_img)
    near = np.argsort(np.linalg.norm(t, axis=1))[:40]
    it = near[rng.integers(0, len(near), n_img)]
    qtrue, ttrue = T(q[ir]), T(t[it])
    ctf = ops.ctf(T(synth.ctf_attrs(n_img, seed=seed + 1)), px)
    if cls is None:
        cls = np.zeros(n_img, np.int64)
    P = torch.empty(n_img, px.n, dtype=torch.complex64, device=DEV)
    for k in range(vols.shape[0]):
        m = np.nonzero(cls == k)[0]
        if len(m):
            mi = T(m)
            P[mi] = ops.project3d(vols[k].contiguous(), ops.rotmat(qtrue[mi].contiguous()), px)
    sigl = ctf * P * ops.trans_table(ttrue, px)
    dat, sig = synth.noisy_images(sigl, px.iSig, px.idim // 2 + 1, snr=snr, seed=seed + 2)
    return dat, ctf, sig, qtrue, ttrue


# ------------------------------------------------------------ C4: K classes
N4, K4, RU4, NR4 = 200, 4, 19, 1500


@pytest.fixture(scope="module")
def c4():
    vols = torch.stack([synth.projectee(synth.blob_volume(N4, seed=50 + k, device=DEV), 2)
                        for k in range(K4)]).contiguous()
    px = ops.PixelSet(N4, 2, RU4, 1, device=DEV)
    assert px.n == 542
    gset = synth.global_sample_set(NR4, seed=6)
    return dict(vols=vols, px=px, gset=gset)


def test_c4_class_scan_matches_oracle(orc, c4):
    """kIdx = 0..3 scans merged into one running baseline vs the restatement."""
    px, gset = c4["px"], c4["gset"]
    q, t, pR, pT = gset
    cls = np.arange(12) % K4
    dat, ctf, sig, *_ = grid_images(c4["vols"], px, gset, 12, seed=60, cls=cls, snr=0.2)
    traP = ops.trans_table(T(t), px)
    state, ref = None, None
    pxh = orc.pixel_set(N4, 2, RU4, 1)
    for k in range(K4):
        rotP = ops.project3d(c4["vols"][k].contiguous(), ops.rotmat(T(q)), px)
        state = ops.global_scan(rotP, traP, dat, ctf, sig, T(pR), T(pT), kIdx=k, nK=K4, state=state)
        d = orc.dvp_global(c4["vols"][k].cpu().numpy(), 2 * N4, 2, q, t, dat.cpu().numpy(),
                           ctf.cpu().numpy(), sig.cpu().numpy(), pxh, N4, threads=16)
        ref = orc.weights_global(d, pR, pT, kIdx=k, nK=K4, state=ref)
    wC, wR, wT, base = (x.cpu().numpy() for x in state)
    rC, rR, rT, rb = ref
    assert np.allclose(base, rb, rtol=1e-5, atol=0)
    for got, want in ((wC.reshape(12, -1), rC.reshape(12, -1)), (wR.reshape(12, -1), rR.reshape(12, -1)),
                      (wT.reshape(12, -1), rT.reshape(12, -1))):
        m = want >= 1e-4 * want.max(axis=-1, keepdims=True)
        assert (np.abs(got - want)[m] / want[m]).max() < 1e-3


@pytest.mark.parametrize("converge", [False, True])
def test_c4_classification_recovers_class_and_pose(c4, converge):
    px, gset = c4["px"], c4["gset"]
    n = 256
    cls_true = np.random.default_rng(61).integers(0, K4, n)
    dat, ctf, sig, qtrue, ttrue = grid_images(c4["vols"], px, gset, n, seed=62, cls=cls_true)
    e = ex.Expectation(c4["vols"], px, gset, n_phase=10, seed=9, converge=converge)
    quat, trans, pR, pT, score, cls, nph = e.run(dat, ctf, sig)
    cls = cls.cpu().numpy()
    assert np.mean(cls == cls_true) >= 0.95, np.mean(cls == cls_true)
    err = angle_deg(ex.cloud_mode(quat), qtrue)
    ok = torch.as_tensor(cls == cls_true, device=DEV)
    assert float(err[ok].median()) < 2.0
    assert torch.isfinite(quat).all() and torch.isfinite(score).all()
    nph = nph.cpu().numpy()
    if converge:
        # global search: first check at phase 10 always continues, so >= 11
        assert nph.min() >= 11 and nph.max() <= 99, (nph.min(), nph.max())
    else:
        assert (nph == 10).all()


# --------------------------------------------------- local search / C5 mode
N5, RU5 = 128, 30


@pytest.fixture(scope="module")
def local_stack():
    vol = synth.projectee(synth.blob_volume(N5, seed=71, device=DEV), 2)
    px = ops.PixelSet(N5, 2, RU5, 1, device=DEV)
    gset = synth.global_sample_set(1500, seed=72)
    n = 256
    rng = np.random.default_rng(73)
    qtrue = T(synth.uniform_quaternions(n, rng))
    ttrue = T(rng.standard_normal((n, 2)) * 2.0)
    ctf = ops.ctf(T(synth.ctf_attrs(n, seed=74)), px)
    sigl = ctf * ops.project3d(vol, ops.rotmat(qtrue), px) * ops.trans_table(ttrue, px)
    dat, sig = synth.noisy_images(sigl, px.iSig, N5 // 2 + 1, snr=5.0, seed=75)
    return dict(vol=vol, px=px, gset=gset, dat=dat, ctf=ctf, sig=sig, qtrue=qtrue, ttrue=ttrue)


def _start_state(s, spread_deg, mR=125, mT=9, seed=76):
    """A particle state around (but not at) the true pose: clouds of spread
    ~spread_deg about a pose offset by ~spread_deg, translations +- 1 px."""
    n = s["dat"].shape[0]
    rng = np.random.default_rng(seed)
    q0 = s["qtrue"].cpu().numpy()
    off = synth.clustered_quaternions(n, 1, spread_deg, rng)[:, 0]
    # compose: pose = q0 * small rotation
    d = rng.standard_normal((n, 4)) * np.radians(spread_deg) / 2
    d[:, 0] = 1.0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    del off
    w0, x0, y0, z0 = q0.T
    w1, x1, y1, z1 = d.T
    qc = np.stack([w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1, w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
                   w0 * y1 - x0 * z1 + y0 * w1 + z0 * x1, w0 * z1 + x0 * y1 - y0 * x1 + z0 * w1], 1)
    e = rng.standard_normal((n, mR, 4)) * np.radians(spread_deg) / 2
    e[..., 0] = 1.0
    e /= np.linalg.norm(e, axis=-1, keepdims=True)
    w0, x0, y0, z0 = [qc[:, None, k] for k in range(4)]
    w1, x1, y1, z1 = [e[..., k] for k in range(4)]
    quat = np.stack([w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1, w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
                     w0 * y1 - x0 * z1 + y0 * w1 + z0 * x1, w0 * z1 + x0 * y1 - y0 * x1 + z0 * w1], -1)
    trans = s["ttrue"].cpu().numpy()[:, None, :] + rng.uniform(-1, 1, (n, mT, 2))
    return (T(quat), T(trans), T(np.full((n, mR), 1.0 / mR)), T(np.full((n, mT), 1.0 / mT)))


@pytest.mark.parametrize("mean", ["acg", "top"])
def test_local_search_refines_from_a_particle_state(local_stack, mean):
    s = local_stack
    state = _start_state(s, 4.0)
    start_err = angle_deg(ex.cloud_mode(state[0]), s["qtrue"])
    e = ex.Expectation(s["vol"], s["px"], None, search="local", converge=True, perturb_mean=mean,
                       seed=4)
    quat, trans, pR, pT, score, cls, nph = e.run(s["dat"], s["ctf"], s["sig"], state=state)
    err = angle_deg(ex.cloud_mode(quat), s["qtrue"])
    assert float(err.median()) < 0.5 * float(start_err.median()), (err.median(), start_err.median())
    assert float(err.median()) < 1.5
    terr = (trans.mean(1) - s["ttrue"]).norm(dim=-1)
    assert float(terr.median()) < 0.5
    nph = nph.cpu().numpy()
    # local search: phases 0..; the first check (phase 3) always continues
    assert nph.min() >= 4 and nph.max() <= 99
    assert torch.allclose(pR.sum(-1), torch.ones_like(pR[:, 0]), rtol=1e-9)
    assert torch.isfinite(score).all()


def test_local_search_fixed_phases_is_reproducible(local_stack):
    s = local_stack
    outs = []
    for _ in range(2):
        state = _start_state(s, 3.0)
        e = ex.Expectation(s["vol"], s["px"], None, search="local", n_phase=3, seed=8)
        outs.append([x.clone() for x in e.run(s["dat"], s["ctf"], s["sig"], state=state)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert (outs[0][6] == 2).all()      # phases 0, 1, 2


@pytest.mark.parametrize("converge", [False, True])
def test_view_order_leaves_every_image_unchanged(local_stack, monkeypatch, converge):
    """thx_view_order (csrc/order.hip) only changes which workgroup takes
    which image in the 3D phases: with the order (default) and without
    (THX_VIEW_ORDER=0) the driver returns bit-identical particles, priors,
    scores, classes and phase counts -- global search, fixed phases and the
    stopping rule."""
    s = local_stack
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("THX_VIEW_ORDER", flag)
        e = ex.Expectation(s["vol"], s["px"], s["gset"], n_phase=4, seed=12, converge=converge)
        outs.append([x.clone() for x in e.run(s["dat"], s["ctf"], s["sig"])])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_ypair_ball_leaves_every_image_unchanged(local_stack, monkeypatch):
    """The driver's compact y-pair ball (slices interleaved, no wrap) reads
    the same taps with the same weights as the whole copy: with the ball
    (default) and without (THX_YPAIR_BALL=0) the driver returns bit-identical
    particles, priors, scores and classes.  The stack is the bench's SNR
    (0.05), whose wide clouds the device route sends to the y-pair kernel in
    every phase -- asserted, so the ball is really read."""
    from bench import make_stack
    s = local_stack
    _, dat, ctf, sig, *_ = make_stack(N5, 2, RU5, 1, 256, DEV, seed=77, vol=s["vol"])
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("THX_YPAIR_BALL", flag)
        e = ex.Expectation(s["vol"], s["px"], s["gset"], n_phase=4, seed=13)
        routes = e.track_routes(4)
        outs.append([x.clone() for x in e.run(dat, ctf, sig)])
        assert routes.cpu().tolist() == [2] * 4, (flag, routes.cpu().tolist())
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_global_converge_matches_fixed_quality(local_stack):
    """The stopping rule ends every image between phase 11 and 99 and keeps
    the grid-pose recovery of the fixed 10-phase run."""
    s = local_stack
    gset = s["gset"]
    dat, ctf, sig, qtrue, ttrue = grid_images(s["vol"][None], s["px"], gset, 128, seed=80)
    res = {}
    for conv in (False, True):
        e = ex.Expectation(s["vol"], s["px"], gset, n_phase=10, seed=3, converge=conv)
        quat, trans, pR, pT, score, cls, nph = e.run(dat, ctf, sig)
        res[conv] = (angle_deg(ex.cloud_mode(quat), qtrue), nph.cpu().numpy())
    assert float(res[True][0].median()) < 2.0 and float(res[False][0].median()) < 2.0
    assert res[True][1].min() >= 11 and res[True][1].max() <= 99


def test_concurrent_sub_batches_on_three_streams(local_stack):
    """Three sub-batches of a global search enqueued from three host threads on
    three HIP streams at once give bit-identical particles, priors, scores and
    phase counts to the same sub-batches run one after the other on one
    stream.  Every call gets its own scratch (ops.workspace is per stream):
    the per-device buffer the driver used to share let concurrent calls
    overwrite each other's patch records and active lists."""
    import threading
    s = local_stack
    gset = s["gset"]
    dat, ctf, sig, _, _ = grid_images(s["vol"][None], s["px"], gset, 3 * 96, seed=81, snr=1.0)
    e = ex.Expectation(s["vol"], s["px"], gset, n_phase=10, seed=5)
    parts = [slice(96 * k, 96 * (k + 1)) for k in range(3)]
    args = [(dat[p].contiguous(), ctf[p].contiguous(), sig[p].contiguous()) for p in parts]
    torch.cuda.synchronize()
    serial = [[x.clone() for x in e.run(*a)] for a in args]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(DEV) for _ in range(3)]
    got, errs = [None] * 3, []
    go = threading.Barrier(3)

    def worker(k):
        try:
            go.wait()
            with torch.cuda.stream(streams[k]):
                got[k] = e.run(*args[k])
        except Exception as exc:      # noqa: BLE001 -- reported below
            errs.append(exc)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    torch.cuda.synchronize()
    assert not errs, errs
    for k in range(3):
        for a, b in zip(serial[k], got[k]):
            assert torch.equal(a, b), k
    ops.release_workspaces()


def test_local_search_with_cell_projectee(local_stack):
    """thx_expect_cfg.volCells: the phases gather 64-B cells; the same state,
    seed and phases give the same refinement quality and, phase by phase, the
    same likelihood baselines up to the gathers' rounding."""
    s = local_stack
    cells = ops.volume_cells(s["vol"])
    res = {}
    for name, c in (("halfcomplex", None), ("cells", cells)):
        state = _start_state(s, 3.0)
        e = ex.Expectation(s["vol"], s["px"], None, search="local", n_phase=1, seed=8, cells=c)
        quat, trans, pR, pT, score, cls, nph = e.run(s["dat"], s["ctf"], s["sig"], state=state)
        res[name] = (score.clone(), quat.clone())
        state = _start_state(s, 3.0)
        e3 = ex.Expectation(s["vol"], s["px"], None, search="local", n_phase=4, seed=8, cells=c)
        q3 = e3.run(s["dat"], s["ctf"], s["sig"], state=state)[0]
        res[name + "_err"] = angle_deg(ex.cloud_mode(q3), s["qtrue"])
    # one phase from the same state and seed: the same samples, baselines to FP32 rounding
    a, b = res["halfcomplex"][0], res["cells"][0]
    assert torch.allclose(a, b, rtol=1e-5, atol=0)
    for name in ("halfcomplex", "cells"):
        assert float(res[name + "_err"].median()) < 1.5
