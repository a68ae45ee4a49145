"""CPU-side checks of the C-ABI library: it loads, exports every symbol the
header declares, the host-only entry points agree with the oracle, and
argument validation rejects bad shapes before anything is enqueued."""
import ctypes
import os
import re

import numpy as np
import pytest

from thunder_amd import _lib, build

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                      "thunder_amd.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(thx_\w+)\s*\(", txt)))


@pytest.fixture(scope="module")
def L():
    build.build()
    return _lib.lib()


def test_exports_every_declared_symbol(L):
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib.SIGNATURES, f"{n} missing from the ctypes table"


def test_abi_version(L):
    assert L.thx_abi_version() == 9


def test_pixel_tile_order(L):
    # every pixel once, 16-entry groups padded with -1, each group a compact patch
    from thunder_amd import ops
    for N, rU in ((256, 24), (64, 20), (256, 126)):
        px = ops.PixelSet(N, 2, rU, 1)
        o = px.order
        assert len(o) % 16 == 0 and len(o) < 1.25 * px.n + 16
        assert sorted(o[o >= 0].tolist()) == list(range(px.n))
        ext = []
        for c0 in range(0, len(o), 16):
            s = o[c0:c0 + 16]
            s = s[s >= 0]
            assert len(s) > 0
            ext.append(max(np.ptp(px.iCol[s]), np.ptp(px.iRow[s])))
        ext = np.array(ext)
        assert np.median(ext) <= 3 and np.mean(ext <= 7) > 0.95, (N, rU, np.percentile(ext, 90))
    st = L.thx_pixel_tile_order(None, None, 4, 0, None, None)
    assert st == 1


@pytest.mark.parametrize("N,rL,rU", [(64, 0, 30), (256, 1, 24), (256, 1, 126), (200, 1, 19)])
def test_pixel_set_matches_oracle(L, orc, N, rL, rU):
    cap = (N // 2 + 1) * N
    bufs = [np.zeros(cap, np.int32) for _ in range(4)]
    n = ctypes.c_int()
    st = L.thx_pixel_set(N, 2, rU, rL, cap, *[b.ctypes.data_as(ctypes.c_void_p) for b in bufs],
                         ctypes.byref(n))
    assert st == 0
    px = orc.pixel_set(N, 2, rU, rL)
    assert n.value == px.n
    for a, b in zip(bufs, (px.iCol, px.iRow, px.iSig, px.iPxl)):
        assert np.array_equal(a[:n.value], b)


def test_pixel_set_rejects_radius_past_nyquist(L):
    n = ctypes.c_int()
    st = L.thx_pixel_set(64, 2, 40.0, 0.0, 10, None, None, None, None, ctypes.byref(n))
    assert st == 1
    assert b"rU" in L.thx_last_error()


def test_argument_validation_without_gpu(L):
    # invalid shapes are rejected before any kernel is enqueued
    assert L.thx_global_scan(None, 0, None, 5, None, None, None, 1, 10, None, None, 0, 1,
                             None, None, None, None, 1, None, 0, None) == 1
    assert L.thx_global_scan(None, 4, None, 5, None, None, None, 1, 10, None, None, 2, 1,
                             None, None, None, None, 1, None, 0, None) == 1
    assert L.thx_local_phase(None, 0, 64, 2, None, 0, None, 9, None, None, None, None, None, None,
                             None, None, None, 0, 10, 32, 1, None, None, None, None, None, None,
                             0, None) == 1
    assert L.thx_resample(1, 0, None, None, 4, None, None, None, None, None) == 1
    assert L.thx_fsc(None, None, 31, 8, None, None, 0, None) == 1
    assert L.thx_ExpectProject(None, None, None, None, None, 1, 2, 1, 64, 10) == 1


def test_workspace_queries_are_host_only(L):
    ws0 = L.thx_global_scan_workspace(100, 2000, 151, 870, 0)
    ws1 = L.thx_global_scan_workspace(100, 2000, 151, 870, 1)
    assert ws0 >= 100 * 2000 * 151 * 4
    assert ws1 > 0
    assert L.thx_fsc_workspace(64) >= 3 * 64 * 8
    # dvp + one 64-B neighbourhood record per (image, rotation tile, patch)
    assert L.thx_local_phase_workspace(10, 125, 9, 944) >= 10 * 125 * 9 * 4 + 10 * 59 * 64


def test_round2_entry_points_validate_without_gpu(L):
    """Argument checks of the round-2 entry points run before any device work,
    and empty batches return THX_OK without touching a device."""
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    ok, bad = 0, 1
    # binned insert: rMax * pf reaching the volume edge, mReco above the grouping
    # limit, a missing pixel order; an empty batch is a no-op
    args = lambda vdim, mReco, rMax, order, nImg: (
        None, None, None, None, vdim, 2, None, None, None, None, None, None, None, nImg, mReco,
        None, None, order, 944, 870, 32, rMax, None, 0, None)
    dummy = ctypes.c_void_p(1)
    assert L.thx_insert3d_binned(*args(64, 100, 15, dummy, 4)) == bad
    assert L.thx_insert3d_binned(*args(512, 2000, 24, dummy, 4)) == bad
    assert b"mReco" in L.thx_last_error()
    assert L.thx_insert3d_binned(*args(512, 100, 24, None, 4)) == bad
    assert L.thx_insert3d_binned(*args(512, 100, 24, dummy, 0)) == ok
    # its workspace: entries of at most 2^28 per image batch (24 B each)
    ws_small = L.thx_insert3d_binned_workspace(10, 100, 944, 2, 24)
    ws_big = L.thx_insert3d_binned_workspace(100000, 100, 944, 2, 24)
    assert ws_small >= 10 * 100 * 944 * 24
    assert ws_big <= (1 << 28) * 24 + (64 << 20)
    # 2D: bad sizes, then empty batches
    assert L.thx_project2d(None, 63, 2, None, 4, None, None, 10, None, None) == bad
    assert L.thx_project2d(None, 64, 2, None, 0, None, None, 10, None, None) == ok
    assert L.thx_insert2d(None, None, None, None, 64, 2, None, None, None, None, None, None, None, 0,
                          5, None, None, 10, 32, None) == ok
    assert L.thx_local_phase2d(None, 64, 2, None, None, 4, None, 9, None, None, None, None, None,
                               None, None, None, 10, 32, 0, None, None, None, None, None, None, 0,
                               None) == ok
    # the host 2D insert rejects a sample class outside [0, nk) before allocating
    nImg, mReco, npxl, nk = 2, 3, 4, 2
    F = np.zeros(2 * 33 * 64 * nk, np.float32)
    T = np.zeros(33 * 64 * nk, np.float32)
    O = np.zeros(2 * nk)
    cnt = np.zeros(nk, np.int32)
    dat = np.zeros(2 * nImg * npxl, np.float32)
    ctf = np.ones(nImg * npxl, np.float32)
    w = np.ones(nImg, np.float32)
    off = np.zeros(2 * nImg)
    nc = np.array([0, 1, 2, 0, 1, 0], np.int32)          # 2 >= nk
    rot = np.zeros(2 * nImg * mReco)
    tr = np.zeros(2 * nImg * mReco)
    ic = np.array([2, 4, 6, 8], np.int32)
    ir = np.zeros(4, np.int32)
    assert L.thx_InsertI2D(P(F), P(T), P(O), P(cnt), None, P(dat), P(ctf), None, P(w), P(off),
                           P(nc), P(rot), P(tr), None, None, P(ic), P(ir), 0.0, 0, nk, 2, npxl,
                           mReco, 32, 64, nImg) == bad
    assert b"class index" in L.thx_last_error()
    # ExpectGlobal2D supports the reference's linear interpolation only
    assert L.thx_ExpectGlobal2D(P(F), P(dat), P(ctf), P(ctf), P(tr), P(w), P(w), P(w), P(off),
                                P(off), P(rot), P(ic), P(ir), 1, 3, 3, 2, 0, 32, 64, npxl,
                                nImg) == bad
    # reconstruction and the half-map reduction reject null inputs
    assert L.thx_reconstruct(None, None, 32, 2, 1.9, 15.0, 1, 0, 0, None, 0, 0, None, None, None,
                             None, None, 0, None) == bad
    assert L.thx_halfmap_allreduce(None, None, None, None, None, 10, 1, None) == bad


def test_global_sample_sizes_match_survey():
    """a3 sizes (host function, no GPU): nT = 151 at transS 10, tsf 0.25
    (SURVEY 8a), the 3D clamp 500 -> 1500 (C2), nR = mS / (1 + nSym)."""
    from thunder_amd import ops, synth
    assert ops.global_sample_sizes(2000) == (2000, 2000, 151)
    assert ops.global_sample_sizes(500) == (1500, 1500, 151)
    assert ops.global_sample_sizes(500, n_sym_elem=3) == (6000, 1500, 151)
    assert ops.global_sample_sizes(500, mode=0) == (500, 500, 151)
    assert ops.global_sample_sizes(2000, trans_s=2.0)[2] == 30
    for ts in (3.0, 10.0, 17.5):
        assert ops.global_sample_sizes(2000, trans_s=ts)[2] == synth.n_trans_global(ts, 0.25)


def test_ctf_search_entry_points_validate_without_gpu(L):
    """CTF-search and sample-set entry points check their arguments before any
    device work; empty batches are no-ops."""
    ok, bad = 0, 1
    dummy = ctypes.c_void_p(1)
    # thx_local_phase_d: nD must be positive; an empty batch is a no-op
    args = lambda nD, nImg: (None, dummy, 0, 64, 2, dummy, 10, dummy, 9, nD, dummy, dummy, dummy,
                             dummy, dummy, dummy, dummy, dummy, dummy, None, 0, 200, 32, nImg,
                             dummy, dummy, dummy, dummy, dummy, None, None, 0, None)
    assert L.thx_local_phase_d(*args(0, 4)) == bad
    assert L.thx_local_phase_d(*args(3, 0)) == ok
    assert L.thx_local_phase_d(*args(200, 4)) == bad        # nT * nD > 1024 columns
    # thx_ctf_search / thx_defocus_pre: sizes, then empty batches
    assert L.thx_ctf_search(None, None, None, 0, None, None, None, 4, 10, None, None) == bad
    assert L.thx_ctf_search(None, None, None, 9, None, None, None, 0, 10, None, None) == ok
    assert L.thx_defocus_pre(None, 4, None, None, 10, 0, None, None, None, None, None) == bad
    assert L.thx_defocus_pre(None, 0, None, None, 10, 32, None, None, None, None, None) == ok
    # defocus particles: bad op, empty batch
    assert L.thx_pf_defocus(4, 9, 3, 0.0, 1, 0, dummy, dummy, dummy, None) == bad
    assert L.thx_pf_defocus(0, 9, 0, 0.01, 1, 0, None, None, None, None) == ok
    # the CTF-search driver: no configuration, wrong search type
    assert L.thx_expectation_ctf(None, None, None, None, None, None, None, None, 0, 10, 4,
                                 *([None] * 7), None, 0, None) == bad
    assert b"CTF-search configuration" in L.thx_last_error()
    # the insert with per-sample defocus: attr without nD
    a = (None, None, None, None, 64, 2, None, dummy, None, None, None, None, None, None, 4, 10,
         None, None, dummy, 944, 870, 32, 15, dummy, 1 << 20, None)
    assert L.thx_insert3d_binned_d(*a) == bad
    assert L.thx_InsertFTCS(*([None] * 14), ctypes.c_float(1.32), 2, 10, 5, 32, 64, 1, None) == bad
    # the global sample set producer
    assert L.thx_global_sample_set(0, 151, 10.0, 1, dummy, dummy, dummy, dummy, None) == bad
    assert L.thx_global_sample_set(10, 1, 10.0, 1, dummy, dummy, dummy, dummy, None) == bad


def _policy(L, n, env=None, size=-1, rank=-1, cur=0):
    out = (ctypes.c_int * 16)()
    cnt = ctypes.c_int(0)
    st = L.thx_adapter_device_policy(n, cur, env.encode() if env is not None else None, size, rank,
                                     out, 16, ctypes.byref(cnt))
    assert st == 0
    return list(out[:cnt.value])


def test_adapter_device_policy(L):
    """THX_DEVICES unset: every visible GPU, as cuthunder's getAviDevice --
    including THUNDER's master + two hemisphere ranks (LOCAL_WORLD_SIZE=3) on
    an 8-GPU node; one device per process only when the node runs at least
    one process per GPU."""
    assert _policy(L, 8) == list(range(8))
    for rank in range(3):
        assert _policy(L, 8, size=3, rank=rank) == list(range(8))
    assert _policy(L, 8, size=8, rank=5) == [5]
    assert _policy(L, 8, size=16, rank=13) == [5]
    assert _policy(L, 1, size=3, rank=2) == [0]
    assert _policy(L, 8, env="local", size=3, rank=2) == [2]
    assert _policy(L, 8, env="current", cur=6) == [6]
    assert _policy(L, 8, env="all", size=8, rank=1) == list(range(8))
    assert _policy(L, 8, env="0,3") == [0, 3]
    out = (ctypes.c_int * 4)()
    cnt = ctypes.c_int(0)
    assert L.thx_adapter_device_policy(8, 0, b"9", -1, -1, out, 4, ctypes.byref(cnt)) != 0
    assert L.thx_adapter_device_policy(0, 0, None, -1, -1, out, 4, ctypes.byref(cnt)) != 0


def test_global_scan_dvp_validates_without_gpu(L):
    """thx_global_scan_dvp (ABI 9): only the split algorithms (2, 4) keep a
    per-sample dump; a negative guard and the retired fp16x2 (algo 3) are
    refused before any device work, with or without a dump (NULL dump = guard
    control only)."""
    p = ctypes.c_void_p(16)
    args = lambda algo, guard, dvp: (p, 2000, p, 151, p, p, p, 8, 870, p, p, 0, 1, p, p, p, p, algo,
                                     ctypes.c_float(guard), dvp, p, ctypes.c_size_t(1 << 40), None)
    assert L.thx_global_scan_dvp(*args(1, 4.0, p)) != 0
    assert L.thx_global_scan_dvp(*args(3, 4.0, p)) != 0
    assert L.thx_global_scan_dvp(*args(4, -1.0, p)) != 0
    assert L.thx_global_scan_dvp(*args(3, 4.0, None)) != 0
    assert L.thx_global_scan_dvp(*args(4, -1.0, None)) != 0
    assert L.thx_global_scan(p, 2000, p, 151, p, p, p, 8, 870, p, p, 0, 1, p, p, p, p, 3, p,
                             ctypes.c_size_t(1 << 40), None) != 0
    assert L.thx_global_scan_workspace(8, 2000, 151, 870, 4) > 0
