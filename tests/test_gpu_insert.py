"""K-class insert (InsertFT with nC, gpu/interface/Interface.h:267-292: each
class's reconstructor inserts image l's first nC[l] samples,
src/Optimiser.cpp:6852-6950) against the restatement, and the RCCL half-map
reduction behind the C-ABI (thx_halfmap_allreduce, the ncclAllReduce of
gpu/src/cuthunder.cu:5903-5993)."""
import ctypes

import numpy as np
import pytest
import torch

from stacks import small_stack
from thunder_amd import ops, synth
from thunder_amd._lib import lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def T(a):
    return torch.as_tensor(np.ascontiguousarray(a), device=DEV)


@pytest.fixture(scope="module")
def stack(orc):
    return small_stack(orc, N=32, nImg=6, nR=4, nT=3, seed=8)


def _samples(nImg, mReco, seed):
    rng = np.random.default_rng(seed)
    quat = synth.clustered_quaternions(nImg, mReco, 3.0, rng)
    trans = rng.standard_normal((nImg, mReco, 2)) * 2
    off = rng.standard_normal((nImg, 2))
    w = np.full(nImg, 1.0 / mReco, np.float32)
    return quat, trans, off, w


def _oracle_truncated(orc, s, quat, trans, off, w, nC):
    """Sum over images of the restatement's insert of image l's first nC[l] samples."""
    size = (s["vdim"] // 2 + 1) * s["vdim"] ** 2
    F = np.zeros(2 * size, np.float32)
    Tm = np.zeros(size, np.float32)
    O = np.zeros(3)
    cnt = 0
    for l, n in enumerate(nC):
        if n == 0:
            continue
        f, t, o, c = orc.insert_batch(s["vdim"], s["pf"], s["dat"][l:l + 1], s["ctf"][l:l + 1],
                                      quat[l:l + 1, :n], trans[l:l + 1, :n], off[l:l + 1], w[l:l + 1],
                                      s["px"], s["N"])
        F += f.view(np.float32)
        Tm += t
        O += o
        cnt += c
    return F.view(np.complex64), Tm, O, cnt


@pytest.mark.parametrize("method", ["direct", "tiled", "binned"])
def test_insert_with_per_image_counts(orc, stack, method):
    s = stack
    nImg, mReco = 6, 140                   # two 128-sample tiles per image
    nC = np.array([0, 5, 140, 129, 1, 77], np.int32)
    quat, trans, off, w = _samples(nImg, mReco, 31)
    px = ops.PixelSet(s["N"], s["pf"], s["rU"], s["rL"], device=DEV)
    hm = ops.HalfMap(s["vdim"], DEV)
    ops.insert3d(hm, T(s["dat"]), T(s["ctf"]), T(quat), T(trans), T(off), T(w), px, method=method,
                 nC=T(nC))
    F, Tm, O, cnt = _oracle_truncated(orc, s, quat, trans, off, w, nC)
    gF = hm.F.cpu().numpy().reshape(-1)
    gT = hm.T.cpu().numpy().reshape(-1)
    assert np.max(np.abs(gF - F)) <= 1e-5 * np.max(np.abs(F))
    assert np.max(np.abs(gT - Tm)) <= 1e-5 * np.max(np.abs(Tm))
    assert np.allclose(hm.O.cpu().numpy(), O, rtol=1e-12, atol=1e-12)
    assert int(hm.counter.item()) == cnt == int(nC.sum())


def test_host_insert_ftc_matches_oracle(orc, stack):
    """thx_InsertFTC: the Interface.h K-class InsertFT shape (host pointers,
    padded pixel set, read-modify-write of the caller's F/T/O/counter)."""
    s = stack
    nImg, mReco = 6, 12
    nC = np.array([3, 0, 12, 7, 1, 12], np.int32)
    quat, trans, off, w = _samples(nImg, mReco, 32)
    size = (s["vdim"] // 2 + 1) * s["vdim"] ** 2
    F = np.zeros(2 * size, np.float32)
    Tm = np.zeros(size, np.float32)
    O = np.zeros(3)
    cnt = np.zeros(1, np.int32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    dat = np.ascontiguousarray(s["dat"]).view(np.float32)
    ctf = np.ascontiguousarray(s["ctf"])
    iq, it = np.ascontiguousarray(quat), np.ascontiguousarray(trans)
    iColP = (s["px"].iCol * s["pf"]).astype(np.int32)
    iRowP = (s["px"].iRow * s["pf"]).astype(np.int32)
    st = lib().thx_InsertFTC(P(F), P(Tm), P(O), P(cnt), P(dat), P(ctf), P(off), P(w), P(iq), P(it),
                             P(nC), P(iColP), P(iRowP), s["pf"], s["px"].n, mReco, s["N"], s["vdim"],
                             nImg)
    assert st == 0, lib().thx_last_error()
    rF, rT, rO, rc = _oracle_truncated(orc, s, quat, trans, off, w, nC)
    assert np.max(np.abs(F - rF.view(np.float32))) <= 1e-5 * np.max(np.abs(rF.view(np.float32)))
    assert np.max(np.abs(Tm - rT)) <= 1e-5 * np.max(np.abs(rT))
    assert np.allclose(O, rO, rtol=1e-12, atol=1e-12) and int(cnt[0]) == rc


def test_rccl_halfmap_allreduce_single_rank():
    """A one-rank hemisphere communicator: the in-place sum leaves F / T / O /
    counter bit-identical (the multi-rank case is RCCL's own; bench.py runs it
    across the hemisphere's GPUs at N > 1)."""
    uid = ops.RcclComm.unique_id()
    assert len(uid) == 128
    comm = ops.RcclComm(1, uid, 0)
    hm = ops.HalfMap(64, DEV)
    g = torch.Generator(device=DEV).manual_seed(3)
    hm.F.copy_(torch.complex(torch.randn(hm.F.shape, generator=g, device=DEV),
                             torch.randn(hm.F.shape, generator=g, device=DEV)))
    hm.T.copy_(torch.rand(hm.T.shape, generator=g, device=DEV))
    hm.O.copy_(torch.tensor([1.5, -2.0, 3.25], dtype=torch.float64))
    hm.counter.fill_(17)
    ref = [x.clone() for x in (hm.F, hm.T, hm.O, hm.counter)]
    comm.allreduce(hm)
    torch.cuda.synchronize()
    for a, b in zip((hm.F, hm.T, hm.O, hm.counter), ref):
        assert torch.equal(a, b)
    comm.close()


def test_rccl_halfmap_sendrecv_self():
    """thx_halfmap_sendrecv (the leads' B -> A hand-over) as a self send /
    receive in one group on a one-rank communicator: the map arrives
    bit-identical; a receive-only and a send-only call to self pair up the
    same way inside the group."""
    comm = ops.RcclComm(1, ops.RcclComm.unique_id(), 0)
    g = torch.Generator(device=DEV).manual_seed(5)
    src = torch.randn(3 * 1000 + 7, generator=g, device=DEV)
    dst = torch.full_like(src, -1.0)
    comm.sendrecv(send=src, peer_send=0, recv=dst, peer_recv=0, n_recv=src.numel())
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    comm.close()


def test_rccl_round_end_single_rank_group():
    """ops.RcclComm.from_group on a one-rank torch.distributed (gloo) group
    and hemisphere.RoundEnd's RCCL transport at world 1: the unique id goes
    through the group's broadcast, the hemisphere reduction is the identity."""
    import socket

    import torch.distributed as dist

    from thunder_amd import hemisphere
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        comm = ops.RcclComm.from_group(dist.group.WORLD, DEV)
        assert comm.nranks == 1 and comm.rank == 0
        hm = ops.HalfMap(32, DEV)
        hm.F.copy_(torch.complex(torch.randn(hm.F.shape, device=DEV), torch.randn(hm.F.shape, device=DEV)))
        hm.T.copy_(torch.rand(hm.T.shape, device=DEV))
        hm.counter.fill_(3)
        ref = [x.clone() for x in (hm.F, hm.T, hm.counter)]
        comm.allreduce(hm)
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip((hm.F, hm.T, hm.counter), ref))
        comm.close()
        re = hemisphere.RoundEnd(1, 0, "rccl", DEV)
        assert re.is_lead and re.hemi_comm.nranks == 1
        re.reduce(hm)
        torch.cuda.synchronize()
        assert all(torch.equal(a, b) for a, b in zip((hm.F, hm.T, hm.counter), ref))
        re.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("rmax_div,mReco,nImg", [(2, 7, 3), (1, 1, 1)])
def test_binned_insert_outside_tile_grid_and_single_sample(orc, stack, rmax_div, mReco, nImg):
    """thx_insert3d_binned with an rMax below the pixel set's radius: the
    entries past the tile grid go straight to HBM by direct atomics and the
    result still matches the restatement; mReco = 1, one image."""
    from thunder_amd.ops import _ptr, _stream, workspace
    s = stack
    quat, trans, off, w = _samples(nImg, mReco, 41)
    px = ops.PixelSet(s["N"], s["pf"], s["rU"], s["rL"], device=DEV)
    hm = ops.HalfMap(s["vdim"], DEV)
    rMax = max(1, int(np.ceil(s["rU"])) // rmax_div)
    L = lib()
    ws = workspace(L.thx_insert3d_binned_workspace(nImg, mReco, len(px.order), s["pf"], rMax), DEV)
    d, c = T(s["dat"][:nImg]), T(s["ctf"][:nImg])
    q, t, o, ww = T(quat), T(trans), T(off), T(w)
    assert L.thx_insert3d_binned(_ptr(hm.F), _ptr(hm.T), _ptr(hm.O), _ptr(hm.counter), hm.vdim,
                                 s["pf"], _ptr(d), _ptr(c), _ptr(q), _ptr(t), _ptr(o), _ptr(ww), None,
                                 nImg, mReco, _ptr(px.d_iCol), _ptr(px.d_iRow), _ptr(px.d_order),
                                 len(px.order), px.n, px.idim, rMax, _ptr(ws), ws.numel(),
                                 _stream(DEV)) == 0, L.thx_last_error()
    F, Tm, O, cnt = orc.insert_batch(s["vdim"], s["pf"], s["dat"][:nImg], s["ctf"][:nImg], quat,
                                     trans, off, w, s["px"], s["N"])
    gF = hm.F.cpu().numpy().reshape(-1)
    gT = hm.T.cpu().numpy().reshape(-1)
    assert np.max(np.abs(gF - F)) <= 1e-5 * np.max(np.abs(F))
    assert np.max(np.abs(gT - Tm)) <= 1e-5 * np.max(np.abs(Tm))
    assert int(hm.counter.item()) == cnt == nImg * mReco


def _host_insert_ftc(s, quat, trans, off, w, nC, mReco):
    size = (s["vdim"] // 2 + 1) * s["vdim"] ** 2
    F = np.zeros(2 * size, np.float32)
    Tm = np.zeros(size, np.float32)
    O = np.zeros(3)
    cnt = np.zeros(1, np.int32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    dat = np.ascontiguousarray(s["dat"]).view(np.float32)
    ctf = np.ascontiguousarray(s["ctf"])
    iq, it = np.ascontiguousarray(quat), np.ascontiguousarray(trans)
    iColP = (s["px"].iCol * s["pf"]).astype(np.int32)
    iRowP = (s["px"].iRow * s["pf"]).astype(np.int32)
    st = lib().thx_InsertFTC(P(F), P(Tm), P(O), P(cnt), P(dat), P(ctf), P(off), P(w), P(iq), P(it),
                             P(nC), P(iColP), P(iRowP), s["pf"], s["px"].n, mReco, s["N"], s["vdim"],
                             len(nC))
    assert st == 0, lib().thx_last_error()
    return F, Tm, O, cnt


def test_host_adapters_split_images_over_devices(orc, stack, monkeypatch):
    """The batch adapters deal contiguous image blocks over the devices of
    THX_DEVICES, one host thread each, and sum the insert's partial half-maps
    onto the first device (cuthunder's round-robin over every GPU,
    gpu/src/cuthunder.cu:2002-2198, 5570-5826).  On a one-GPU box the list
    "0,0,0" runs that whole path -- three workers, the peer-copy reduction --
    on one device: the insert matches the restatement and the scan's weights
    are bit-identical to the one-device call."""
    s = stack
    nImg, mReco = 6, 12
    nC = np.array([3, 0, 12, 7, 1, 12], np.int32)
    quat, trans, off, w = _samples(nImg, mReco, 33)
    rF, rT, rO, rc = _oracle_truncated(orc, s, quat, trans, off, w, nC)
    L = lib()
    for devs in ("current", "0,0,0", "local"):
        monkeypatch.setenv("THX_DEVICES", devs)
        monkeypatch.setenv("LOCAL_RANK", "0")
        buf = (ctypes.c_int * 8)()
        n = ctypes.c_int()
        assert L.thx_adapter_devices(buf, 8, ctypes.byref(n)) == 0
        assert list(buf[:n.value]) == ([0, 0, 0] if devs == "0,0,0" else [0])
        F, Tm, O, cnt = _host_insert_ftc(s, quat, trans, off, w, nC, mReco)
        assert np.max(np.abs(F - rF.view(np.float32))) <= 1e-5 * np.max(np.abs(rF.view(np.float32)))
        assert np.max(np.abs(Tm - rT)) <= 1e-5 * np.max(np.abs(rT))
        assert np.allclose(O, rO, rtol=1e-12, atol=1e-12) and int(cnt[0]) == rc
    # ExpectGlobal3D: per-image work, so the split is exact
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    nR, nT = len(s["quat"]), len(s["trans"])
    px = ops.PixelSet(s["N"], s["pf"], s["rU"], s["rL"], device=DEV)
    rotP = ops.project3d(T(s["vol"]), ops.rotmat(T(s["quat"])), px).cpu().numpy()
    traP = ops.trans_table(T(s["trans"]), px).cpu().numpy()
    pR, pT = np.full(nR, 1.0 / nR), np.full(nT, 1.0 / nT)
    outs = {}
    for devs in ("current", "0,0,0"):
        monkeypatch.setenv("THX_DEVICES", devs)
        wC, wR, wT = (np.zeros(nImg * k, np.float32) for k in (1, nR, nT))
        base = np.zeros(nImg, np.float32)
        assert L.thx_ExpectGlobal3D(P(rotP.view(np.float32)), P(traP.view(np.float32)),
                                    P(np.ascontiguousarray(s["dat"]).view(np.float32)),
                                    P(np.ascontiguousarray(s["ctf"])),
                                    P(np.ascontiguousarray(s["sig"])), P(wC), P(wR), P(wT), P(pR),
                                    P(pT), P(base), 0, 1, nR, nT, px.n, nImg) == 0, L.thx_last_error()
        outs[devs] = (wC, wR, wT, base)
    for a, b in zip(outs["current"], outs["0,0,0"]):
        assert np.array_equal(a, b)


def test_binned_insert_keeps_small_t_per_voxel(orc, stack):
    """F and T carry separate fixed-point exponents in the binned deposit:
    with data 1e6 x the CTF scale and CTF values spanning four decades, every
    T voxel above 1e-7 of the largest keeps 1e-5 relative accuracy against
    the restatement (a shared exponent set by |F| would round T to 2^-48 of
    max |F| ~ the whole T signal)."""
    s = stack
    nImg, mReco = 6, 9
    quat, trans, off, w = _samples(nImg, mReco, 42)
    rng = np.random.default_rng(43)
    dat = (s["dat"] * 1e6).astype(np.complex64)
    ctf = (10.0 ** rng.uniform(-4, 0, s["ctf"].shape) * np.sign(s["ctf"])).astype(np.float32)
    px = ops.PixelSet(s["N"], s["pf"], s["rU"], s["rL"], device=DEV)
    hm = ops.HalfMap(s["vdim"], DEV)
    ops.insert3d(hm, T(dat), T(ctf), T(quat), T(trans), T(off), T(w), px, method="binned")
    F, Tm, O, cnt = orc.insert_batch(s["vdim"], s["pf"], dat, ctf, quat, trans, off, w, s["px"], s["N"])
    gT = hm.T.cpu().numpy().reshape(-1)
    m = Tm > 1e-7 * Tm.max()
    assert m.sum() > 100
    assert np.max(np.abs(gT - Tm)[m] / Tm[m]) < 1e-5
    gF = hm.F.cpu().numpy().reshape(-1)
    assert np.max(np.abs(gF - F)) <= 1e-5 * np.max(np.abs(F))


def test_adapter_devices_default_policy(monkeypatch):
    """THX_DEVICES unset: every visible GPU for a lone process per node, one
    device (local rank % count) when the launcher reports several processes
    per node (ranks sharing a node must not all fan out and bind
    their hemisphere communicators to device 0)."""
    L = lib()
    nDev = torch.cuda.device_count()
    buf = (ctypes.c_int * 16)()
    n = ctypes.c_int()
    monkeypatch.delenv("THX_DEVICES", raising=False)
    for v in ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS",
              "MV2_COMM_WORLD_LOCAL_SIZE", "SLURM_NTASKS_PER_NODE", "PMI_LOCAL_SIZE",
              "LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
              "MV2_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID", "PMI_LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    assert L.thx_adapter_devices(buf, 16, ctypes.byref(n)) == 0
    assert list(buf[:n.value]) == list(range(nDev))
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    monkeypatch.setenv("LOCAL_RANK", "1")
    assert L.thx_adapter_devices(buf, 16, ctypes.byref(n)) == 0
    assert list(buf[:n.value]) == [1 % nDev]
    monkeypatch.setenv("THX_DEVICES", "all")
    assert L.thx_adapter_devices(buf, 16, ctypes.byref(n)) == 0
    assert list(buf[:n.value]) == list(range(nDev))
