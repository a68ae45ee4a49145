"""GPU parity at the BASELINE.json metric configuration (box 256, pf 2,
nR 2000, nT 151, rU 24 -> nPxl 870; full-resolution phase rU 126 ->
nPxl 24 746): the four global-scan algorithms agree with each other on a
64-image batch, and with the CPU restatement on an image / rotation subset
the oracle evaluates in seconds."""
import numpy as np
import pytest
import torch

from thunder_amd import ops, synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def c3():
    from bench import make_stack
    N, pf = 256, 2
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=DEV), pf)
    px, dat, ctf, sig, qtrue, ttrue = make_stack(N, pf, 24, 1, 64, DEV, seed=9, vol=vol)
    return dict(N=N, pf=pf, vol=vol, px=px, dat=dat, ctf=ctf, sig=sig)


def test_scan_algorithms_agree_at_metric_config(c3):
    q, t, pR, pT = synth.global_sample_set(2000, seed=2)
    px = c3["px"]
    rotP = ops.project3d(c3["vol"], ops.rotmat(torch.as_tensor(q, device=DEV)), px)
    traP = ops.trans_table(torch.as_tensor(t, device=DEV), px)
    pRd, pTd = torch.as_tensor(pR, device=DEV), torch.as_tensor(pT, device=DEV)
    res = {a: [x.cpu().numpy() for x in ops.global_scan(rotP, traP, c3["dat"], c3["ctf"], c3["sig"],
                                                         pRd, pTd, algo=a)] for a in (0, 1, 2, 4)}
    ref = res[0]
    for a in (1, 2, 4):
        wC, wR, wT, base = res[a]
        assert np.allclose(base, ref[3], rtol=1e-5, atol=0)
        for x, y in ((wR, ref[1]), (wT, ref[2]), (wC, ref[0])):
            m = y >= 1e-4 * y.max(axis=-1, keepdims=True)
            rel = np.abs(x - y)[m] / y[m]
            assert rel.max() < 2e-3, (a, rel.max())


def test_dvp_matches_oracle_subset(orc, c3):
    q, t, pR, pT = synth.global_sample_set(2000, seed=2)
    sub = np.arange(0, 2000, 125)          # 16 rotations
    px = c3["px"]
    rotP = ops.project3d(c3["vol"], ops.rotmat(torch.as_tensor(q[sub], device=DEV)), px)
    traP = ops.trans_table(torch.as_tensor(t, device=DEV), px)
    n = 4
    d = ops.dvp(rotP, traP, c3["dat"][:n].contiguous(), c3["ctf"][:n].contiguous(),
                c3["sig"][:n].contiguous()).cpu().numpy()
    pxh = orc.pixel_set(c3["N"], c3["pf"], 24, 1)
    ref = orc.dvp_global(c3["vol"].cpu().numpy(), 2 * c3["N"], c3["pf"], q[sub], t,
                         c3["dat"][:n].cpu().numpy(), c3["ctf"][:n].cpu().numpy(),
                         c3["sig"][:n].cpu().numpy(), pxh, c3["N"], threads=8)
    assert np.max(np.abs(d - ref) / np.abs(ref)) < 1e-5


@pytest.mark.parametrize("layout", ["halfcomplex", "cells", "ypair", "routed"])
@pytest.mark.parametrize("spread", [1.5, 3.0, 0.0])
def test_full_resolution_phase_matches_oracle(orc, c3, layout, spread):
    """The north-star shape (box 256, nPxl 24 746, 125 x 9) on 1.5 and 3
    degree clouds and uniformly random rotations (spread 0), in every layout
    the bench's roofline_local prices and on the device route with a y-pair
    copy; dvp 1e-5 relative to the oracle."""
    from bench import make_stack
    N, pf = c3["N"], c3["pf"]
    px, dat, ctf, sig, *_ = make_stack(N, pf, 126, 1, 3, DEV, seed=13, vol=c3["vol"])
    assert px.n == 24746
    nImg, mR, mT = 3, 125, 9
    rng = np.random.default_rng(4)
    quat = (synth.clustered_quaternions(nImg, mR, spread, rng) if spread > 0
            else synth.uniform_quaternions(nImg * mR, rng).reshape(nImg, mR, 4))
    trans = rng.standard_normal((nImg, mT, 2))
    ones = np.ones(nImg)
    pR = np.full((nImg, mR), 1 / mR)
    pT = np.full((nImg, mT), 1 / mT)
    T = lambda a: torch.as_tensor(a, device=DEV)
    cl = ops.volume_cells(c3["vol"]) if layout == "cells" else None
    yp = ops.volume_ypair(c3["vol"]) if layout in ("ypair", "routed") else None
    out = ops.local_phase(c3["vol"], T(quat), T(trans), T(ones), T(pR), T(pT), dat, ctf, sig, px,
                          want_dvp=True, cells=cl, ypair=yp, routed=layout == "routed")
    d = out[4].cpu().numpy()
    if layout == "routed":
        assert out[5] in (0, 2), out[5]
        if spread == 0.0:
            assert out[5] == 2          # uniform rotations: no box fits
    pxh = orc.pixel_set(N, pf, 126, 1)
    vnp = c3["vol"].cpu().numpy()
    for l in range(nImg):
        *_, rd = orc.local_phase(vnp, 2 * N, pf, quat[l], trans[l], 1.0, pR[l], pT[l],
                                 dat[l].cpu().numpy(), ctf[l].cpu().numpy(), sig[l].cpu().numpy(),
                                 pxh, N)
        assert np.max(np.abs(d[l] - rd) / np.abs(rd)) < 1e-5


@pytest.mark.parametrize("algo,nT", [(2, 151), (4, 151), (4, 120), (4, 90), (4, 50), (4, 20)])
def test_split_scan_every_tile_row_matches_direct(c3, algo, nT):
    """A whole 64-image tile (both 32-row halves of every MFMA operand, all 16
    accumulator rows per lane) of the split scans' dumped dvp against the
    direct formulation (thx_dvp) at 1e-5, and a repeated call bit-identical.
    A schedule of the bf16x6 main loop once corrupted rows 16-31 of each half
    nondeterministically ("bf16x6 scan"): this is the guard, for
    every instantiation of the kernel's translation fragments (nT 20 / 50 /
    90 / 120 / 151: NF 1-5, padded to 32 .. 160 columns)."""
    q, t, pR, pT = synth.global_sample_set(2000, seed=2)
    t, pT = t[:nT], pT[:nT] / pT[:nT].sum()
    px = c3["px"]
    assert c3["dat"].shape[0] == 64
    rotP = ops.project3d(c3["vol"], ops.rotmat(torch.as_tensor(q, device=DEV)), px)
    traP = ops.trans_table(torch.as_tensor(t, device=DEV), px)
    pRd, pTd = torch.as_tensor(pR, device=DEV), torch.as_tensor(pT, device=DEV)
    ref = ops.dvp(rotP, traP, c3["dat"], c3["ctf"], c3["sig"]).cpu().numpy().astype(np.float64)
    runs = [ops.global_scan(rotP, traP, c3["dat"], c3["ctf"], c3["sig"], pRd, pTd, algo=algo,
                            want_dvp=True)[4].cpu().numpy() for _ in range(2)]
    rel = (np.abs(runs[0] - ref) / np.abs(ref)).reshape(64, -1).max(1)
    assert rel.max() < 1e-5, np.nonzero(rel >= 1e-5)[0]
    assert np.array_equal(runs[0], runs[1])
