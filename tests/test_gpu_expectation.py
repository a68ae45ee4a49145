"""The expectation driver end to end (a11, Optimiser::expectationG,
src/Optimiser.cpp:1684-3403 -> thx_expectation): global scan + particle-
filter phases on device.  Parity unpinned against the reference (its particle
filter draws from an urandom-seeded GSL generator), so the checks are the
properties the reference's loop guarantees.  The images are made exactly at
poses of the global sample set (rotation grid x translation grid) at high
SNR, so the scan's posterior mode must be that grid pose, and the particle
filter must keep its cloud on it; plus a well-formed particle state and
reproducibility for a fixed seed.

(At poses off the grid, a 1500-2000 rotation grid is coarse against a
15-7 A scan resolution: tools/diag_expect.py shows the scan mode in a wrong
basin for about half of the images, as the grid density dictates.)"""
import numpy as np
import pytest
import torch

from thunder_amd import expectation as ex
from thunder_amd import ops, synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
N, PF, RU, NIMG, NR = 64, 2, 12, 64, 1500


def angle_deg(qa, qb):
    c = (qa * qb).sum(-1).abs().clamp(max=1)
    return torch.rad2deg(2 * torch.acos(c))


@pytest.fixture(scope="module")
def grid_stack():
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=DEV), PF)
    px = ops.PixelSet(N, PF, RU, 1, device=DEV)
    gset = synth.global_sample_set(NR, seed=2)
    q, t, pR, pT = gset
    rng = np.random.default_rng(31)
    ir = rng.integers(0, len(q), NIMG)
    near = np.argsort(np.linalg.norm(t, axis=1))[:40]     # translations within the prior's bulk
    it = near[rng.integers(0, len(near), NIMG)]
    qtrue = torch.as_tensor(q[ir], device=DEV)
    ttrue = torch.as_tensor(t[it], device=DEV)
    attrs = torch.as_tensor(synth.ctf_attrs(NIMG, seed=32), device=DEV)
    ctf = ops.ctf(attrs, px)
    sigl = ctf * ops.project3d(vol, ops.rotmat(qtrue), px) * ops.trans_table(ttrue, px)
    dat, sig = synth.noisy_images(sigl, px.iSig, N // 2 + 1, snr=20.0, seed=33)
    return dict(vol=vol, px=px, gset=gset, dat=dat, ctf=ctf, sig=sig, ir=ir, it=it,
                qtrue=qtrue, ttrue=ttrue)


def test_scan_mode_is_the_generating_grid_pose(grid_stack):
    s = grid_stack
    q, t, pR, pT = s["gset"]
    rotP = ops.project3d(s["vol"], ops.rotmat(torch.as_tensor(q, device=DEV)), s["px"])
    traP = ops.trans_table(torch.as_tensor(t, device=DEV), s["px"])
    wC, wR, wT, base = ops.global_scan(rotP, traP, s["dat"], s["ctf"], s["sig"],
                                       torch.as_tensor(pR, device=DEV),
                                       torch.as_tensor(pT, device=DEV))
    r = wR.reshape(NIMG, -1).argmax(-1).cpu().numpy()
    tt = wT.reshape(NIMG, -1).argmax(-1).cpu().numpy()
    assert np.mean(r == s["ir"]) >= 0.95, (r, s["ir"])
    assert np.mean(tt == s["it"]) >= 0.95, (tt, s["it"])


# shuffle: the support is shuffled before every resampling, as
# Particle::resample does (src/Particle.cpp:1298, 2202-2300); ordered: the
# support is resampled in its stored order
@pytest.fixture(scope="module", params=[True, False], ids=["shuffle", "ordered"])
def driver(grid_stack, request):
    s = grid_stack
    e = ex.Expectation(s["vol"], s["px"], s["gset"], n_phase=10, seed=5, shuffle=request.param)
    out = [x.clone() for x in e.run(s["dat"], s["ctf"], s["sig"])]
    again = e.run(s["dat"], s["ctf"], s["sig"])
    return dict(out=out, again=again, shuffle=request.param)


def test_shuffle_changes_the_draw(grid_stack):
    """Same seed, shuffle on / off: the resampled supports differ (the shuffle
    is applied), both are valid particle clouds (checked above)."""
    s = grid_stack
    outs = [ex.Expectation(s["vol"], s["px"], s["gset"], n_phase=2, seed=5, shuffle=f)
            .run(s["dat"], s["ctf"], s["sig"])[0].clone() for f in (True, False)]
    assert not torch.equal(outs[0], outs[1])


def test_particle_filter_stays_on_the_pose(grid_stack, driver):
    quat, trans, pR, pT, score = driver["out"][:5]
    err = angle_deg(ex.cloud_mode(quat), grid_stack["qtrue"])
    assert float(err.median()) < 2.0 and float((err > 10).double().mean()) <= 0.05, err
    terr = (trans - grid_stack["ttrue"][:, None, :]).norm(dim=-1).median(dim=1).values
    assert float(terr.median()) < 0.5, terr


def test_particle_state_is_well_formed(driver):
    quat, trans, pR, pT, score = driver["out"][:5]
    assert torch.isfinite(quat).all() and torch.isfinite(trans).all()
    assert torch.allclose(quat.norm(dim=-1), torch.ones_like(quat[..., 0]), atol=1e-9)
    for w in (pR, pT):
        assert (w >= 0).all()
        assert torch.allclose(w.sum(-1), torch.ones_like(w[:, 0]), rtol=1e-9)
    assert torch.isfinite(score).all()


def test_fixed_seed_is_reproducible(driver):
    for a, b in zip(driver["out"], driver["again"]):
        assert torch.equal(a, b)
