"""Optimiser::expectation() / Reconstructor::insert() surface over the C-ABI.

Mirrors the reference call surface for this path (include/Optimiser.h:747-749,
include/Reconstructor.h:577-664): an ``Expectation`` holds the device-resident
projectee and the shared global sample set of one round and runs the
expectation of an image batch through ``thx_expectation`` (C++ driver in
csrc/optimiser.hip); ``Reconstructor`` inserts posterior samples into a
device half-map through ``thx_insert3d``.  The half-map reduction across the
ranks of one hemisphere is an RCCL all-reduce (``halfmap_allreduce``).
"""
import ctypes
import math

import numpy as np
import torch

from . import ops, synth
from ._lib import check, lib

INCLUDE_OPTIMISER_H = {
    "MIN_N_PHASE_PER_ITER_GLOBAL": 10,   # include/Optimiser.h:56
    "MIN_N_PHASE_PER_ITER_LOCAL": 3,     # include/Optimiser.h:57
    "MAX_N_PHASE_PER_ITER": 100,         # include/Optimiser.h:58
    "MIN_STD_FACTOR": 1,                 # include/Optimiser.h:73
}
SEARCH = {"global": 0, "local": 1, "ctf": 2}   # SEARCH_TYPE_GLOBAL / _LOCAL / _CTF


class ExpectCfg(ctypes.Structure):
    _fields_ = [("idim", ctypes.c_int), ("pf", ctypes.c_int), ("vdim", ctypes.c_int),
                ("nR", ctypes.c_int), ("nT", ctypes.c_int), ("mLR", ctypes.c_int),
                ("mLT", ctypes.c_int), ("nPhase", ctypes.c_int), ("algo", ctypes.c_int),
                ("perturbFactor", ctypes.c_double), ("kMin", ctypes.c_double),
                ("sMin", ctypes.c_double), ("transS", ctypes.c_double),
                ("transM", ctypes.c_double), ("seed", ctypes.c_ulonglong),
                ("shuffle", ctypes.c_int),
                # ABI 3
                ("nK", ctypes.c_int), ("searchType", ctypes.c_int), ("converge", ctypes.c_int),
                ("minPhase", ctypes.c_int), ("maxPhase", ctypes.c_int),
                ("perturbMean", ctypes.c_int), ("acgIters", ctypes.c_int),
                ("perturbFactorL", ctypes.c_double), ("largeFirst", ctypes.c_int),
                ("phaseEvents", ctypes.c_void_p),
                # ABI 4
                ("volCells", ctypes.c_void_p),
                # ABI 5
                ("nPhaseEvents", ctypes.c_int),
                # ABI 6
                ("phaseRoute", ctypes.c_void_p), ("nPhaseRoute", ctypes.c_int),
                ("symQuat", ctypes.c_void_p), ("nSymElem", ctypes.c_int)]


class CtfSearchCfg(ctypes.Structure):
    _fields_ = [("mLD", ctypes.c_int), ("ctfRefineS", ctypes.c_double),
                ("perturbFactorSCTF", ctypes.c_double), ("attr", ctypes.c_void_p),
                ("d", ctypes.c_void_p), ("pD", ctypes.c_void_p)]


class Expectation:
    """One round of expectation on the current GPU (Optimiser::expectationG).

    vol: half-complex projectee [vdim, vdim, vdim/2+1] complex64 (device), or
         [nK, vdim, vdim, vdim/2+1] for K-class classification.
    gset: (quat [nR,4], trans [nT,2], pR [nR], pT [nT]) numpy float64 (global
          search; None for a local search).
    search: "global" (scan + reseed + phases 1..), "local" (phases 0.. from
            the caller's particle state, passed to run()) or "ctf"
            (SEARCH_TYPE_CTF: a local search that also samples mLD defocus
            factors per image; run() takes the CTF attributes).
    converge: per-image vari-decrease stopping rule between MIN_N_PHASE_PER_ITER
              (10 global / 3 local) and MAX_N_PHASE_PER_ITER (100) phases;
              False: exactly n_phase phases.
    perturb_mean: "acg" = inferACG mean of the cloud (the reference's compiled
                  PARTICLE_ROT_MEAN_USING_STAT_PERTURB), "top" = top particle.
    large_first: OPTIMISER_GLOBAL_PERTURB_LARGE (off in the reference's
                 include/Config.h): the first global phase perturbs by perturbFactorL.
    cells: ops.volume_cells(vol) (K = 1): the phases gather one 64-B cell per
           sample (thx_expect_cfg.volCells); "auto" (default) builds it for
           large boxes at full resolution (ring radius >= 300 voxels), None: off.
    sym: point group ("C4", "D2", ... ; MODE_3D): Particle::symmetrise in the
         particle filter (thx_expect_cfg.symQuat / nSymElem).
    mode: "3d" (MODE_3D) or "2d" (MODE_2D, thx_expectation2d): vol holds
          half-complex class images [vdim, vdim/2+1] or [nK, vdim, vdim/2+1],
          rotations are rows (cos, sin, 0, 0) (gset from
          ops.global_sample_set2d), von Mises particle statistics.
    """

    def __init__(self, vol, px, gset=None, mLR=125, mLT=9, n_phase=10, perturb=0.5,
                 trans_s=10.0, trans_search_factor=0.25, algo=4, seed=7, shuffle=True,
                 search="global", converge=False, perturb_mean="acg", acg_iters=100,
                 perturb_large=2.0, large_first=False, min_phase=None, max_phase=None,
                 mLD=9, ctf_refine_s=0.01, perturb_ctf=0.5, cells="auto", mode="3d", sym=None):
        dev = vol.device
        self.vol, self.px, self.dev = vol, px, dev
        if mode not in ("3d", "2d"):
            raise ValueError("mode: '3d' or '2d'")
        self.two_d = mode == "2d"
        dims = 2 if self.two_d else 3
        nK = vol.shape[0] if vol.dim() == dims + 1 else 1
        vdim = vol.shape[-dims]
        self.search = SEARCH[search]
        if self.search == 0:
            q, t, pR, pT = gset
            self.gQuat = torch.as_tensor(np.ascontiguousarray(q), dtype=torch.float64, device=dev)
            self.gTrans = torch.as_tensor(np.ascontiguousarray(t), dtype=torch.float64, device=dev)
            self.gPR = torch.as_tensor(np.ascontiguousarray(pR), dtype=torch.float64, device=dev)
            self.gPT = torch.as_tensor(np.ascontiguousarray(pT), dtype=torch.float64, device=dev)
            nR, nT = len(q), len(t)
        else:
            self.gQuat = self.gTrans = self.gPR = self.gPT = None
            nR, nT = 0, 0
        # src/Optimiser.cpp:1748-1762: 1 / mS in 2D (nR = mS), mS^(-1/3) in 3D
        scan_min_std_r = (1.0 / nR if self.two_d else nR ** (-1.0 / 3)) if nR else 0.0
        scan_min_std_t = 1.0 / synth.CHI2_QINV_HALF_2DOF / math.sqrt(trans_search_factor * math.pi)
        trans_m = trans_s * (-2.0 * math.log(0.05))           # reCentre, TRANS_Q = 0.05
        # reseed floors with OPTIMISER_SCAN_SET_MIN_STD_WITH_PERTURB (include/Config.h:224,
        # src/Optimiser.cpp:1033-1079); MIN_STD_FACTOR = 1
        # (squared in 3D, :2045-2063; k1 itself in 2D, :2032-2044)
        k_floor = scan_min_std_r / perturb if self.two_d else (scan_min_std_r / perturb) ** 2
        s_floor = scan_min_std_t / perturb
        if min_phase is None:
            min_phase = INCLUDE_OPTIMISER_H["MIN_N_PHASE_PER_ITER_GLOBAL" if self.search == 0
                                            else "MIN_N_PHASE_PER_ITER_LOCAL"]
        if max_phase is None:
            max_phase = INCLUDE_OPTIMISER_H["MAX_N_PHASE_PER_ITER"]
        self.cfg = ExpectCfg(px.idim, px.pf, vdim, nR, nT, mLR, mLT, n_phase, algo, perturb,
                             k_floor, s_floor, trans_s, trans_m, seed, int(bool(shuffle)),
                             nK, self.search, int(bool(converge)), min_phase, max_phase,
                             {"top": 0, "acg": 1}[perturb_mean], acg_iters, perturb_large,
                             int(bool(large_first)), None, None, 0, None, 0, None, 0)
        if self.two_d:
            cells = None
        if isinstance(cells, str):
            if cells != "auto":
                raise ValueError("cells: a thx_volume_cells tensor, None or 'auto'")
            # large boxes at full resolution: the ring's outer radius in projectee
            # voxels past 300 (box 512, rU 254: 508) -> the 8x cell copy
            # (34 GB at box 512), 1.7x faster phases there
            r_vox = px.pf * math.sqrt(2.0 * px.n / math.pi)
            cells = ops.volume_cells(vol) if nK == 1 and r_vox >= 300 else None
        self.cells = cells     # optional thx_volume_cells copy (kept alive here)
        if cells is not None:
            if nK != 1:
                raise ValueError("cells: single-class projectee only")
            ops._req(cells, torch.complex64, tuple(vol.shape) + (8,), "cells")
            self.cfg.volCells = cells.data_ptr()
        # point-group symmetry (MODE_3D): the particle clouds are symmetrised
        # like Particle's (thx_expect_cfg.symQuat); the sample set gset should
        # come from ops.global_sample_set(..., sym=sym)
        self.symQ = None
        if sym is not None and not self.two_d:
            _, q = ops.symmetry(sym)
            if len(q):
                self.symQ = torch.as_tensor(q, device=dev).contiguous()
                self.cfg.symQuat = self.symQ.data_ptr()
                self.cfg.nSymElem = len(q)
        self.mLR, self.mLT, self.nK = mLR, mLT, nK
        self.cs = CtfSearchCfg(mLD, ctf_refine_s, perturb_ctf, None, None, None)

    def track_routes(self, n_phase):
        """Record the device route's kernel choice for the next runs' first
        n_phase phases (thx_expect_cfg.phaseRoute): returns the device int32
        tensor (0 staged, 1 box-less, 2 y-pair, -1 not routed, -2 not run)."""
        self.routes = torch.full((n_phase,), -2, dtype=torch.int32, device=self.dev)
        self.cfg.phaseRoute = self.routes.data_ptr()
        self.cfg.nPhaseRoute = n_phase
        return self.routes

    def workspace_bytes(self, nImg):
        if self.two_d and self.search == 2:
            return lib().thx_expectation2d_ctf_workspace(ctypes.byref(self.cfg), ctypes.byref(self.cs),
                                                         nImg, self.px.n)
        if self.two_d:
            return lib().thx_expectation2d_workspace(ctypes.byref(self.cfg), nImg, self.px.n)
        if self.search == 2:
            return lib().thx_expectation_ctf_workspace(ctypes.byref(self.cfg), ctypes.byref(self.cs),
                                                       nImg, self.px.n, len(self.px.order))
        return lib().thx_expectation_workspace(ctypes.byref(self.cfg), nImg, self.px.n,
                                               len(self.px.order))

    def run_ctf(self, dat, attr, sig, state):
        """SEARCH_TYPE_CTF: attr [nImg, 8] CTF attributes (device float32), state
        (quat, trans, pR, pT[, cls]) updated in place; returns (quat, trans, pR,
        pT, score, cls, nPhase, d [nImg, mLD], pD [nImg, mLD])."""
        if self.search != 2:
            raise ValueError("run_ctf needs search='ctf'")
        nImg, nPxl = dat.shape
        if nPxl != self.px.n:
            raise ValueError("pixel set / image size mismatch")
        ops._req(dat, torch.complex64, (nImg, nPxl), "dat")
        ops._req(sig, torch.float32, (nImg, nPxl), "sigRcp")
        ops._req(attr, torch.float32, (nImg, 8), "attr")
        dev = self.dev
        quat, trans, pR, pT = state[:4]
        for name, t, shp in (("quat", quat, (nImg, self.mLR, 4)), ("trans", trans, (nImg, self.mLT, 2)),
                             ("pR", pR, (nImg, self.mLR)), ("pT", pT, (nImg, self.mLT))):
            ops._req(t, torch.float64, shp, name)
        cls = state[4] if len(state) > 4 else torch.zeros(nImg, dtype=torch.int32, device=dev)
        mLD = self.cs.mLD
        d = torch.empty(nImg, mLD, dtype=torch.float64, device=dev)
        pD = torch.empty(nImg, mLD, dtype=torch.float64, device=dev)
        score = torch.empty(nImg, dtype=torch.float32, device=dev)
        nph = torch.empty(nImg, dtype=torch.int32, device=dev)
        self.cs.attr, self.cs.d, self.cs.pD = attr.data_ptr(), d.data_ptr(), pD.data_ptr()
        ws = ops.workspace(self.workspace_bytes(nImg), dev)
        P = ops._ptr
        if self.two_d:
            check(lib().thx_expectation2d_ctf(ctypes.byref(self.cfg), ctypes.byref(self.cs),
                                              P(self.vol), P(dat), P(sig), P(self.px.d_iCol),
                                              P(self.px.d_iRow), nPxl, nImg, P(quat), P(trans),
                                              P(pR), P(pT), P(score), P(cls), P(nph), P(ws),
                                              ws.numel(), ops._stream(dev)), "thx_expectation2d_ctf")
            return quat, trans, pR, pT, score, cls, nph, d, pD
        check(lib().thx_expectation_ctf(ctypes.byref(self.cfg), ctypes.byref(self.cs), P(self.vol),
                                        P(dat), P(sig), P(self.px.d_iCol), P(self.px.d_iRow),
                                        P(self.px.d_order), len(self.px.order), nPxl, nImg,
                                        P(quat), P(trans), P(pR), P(pT), P(score), P(cls), P(nph),
                                        P(ws), ws.numel(), ops._stream(dev)), "thx_expectation_ctf")
        return quat, trans, pR, pT, score, cls, nph, d, pD

    def run(self, dat, ctf, sig, out=None, state=None):
        """Expectation of one image batch; returns (quat, trans, pR, pT, score,
        cls, nPhase) on device.  state: the starting particle state (quat,
        trans, pR, pT[, cls]) of a local search (updated in place)."""
        nImg, nPxl = dat.shape
        if nPxl != self.px.n:
            raise ValueError("pixel set / image size mismatch")
        for name, t, dt in (("dat", dat, torch.complex64), ("ctf", ctf, torch.float32),
                            ("sigRcp", sig, torch.float32)):
            ops._req(t, dt, (nImg, nPxl), name)
        dev = self.dev
        if self.search == 2:
            raise ValueError("a CTF search runs through run_ctf (it needs the CTF attributes)")
        if self.search == 1:
            if state is None:
                raise ValueError("a local search starts from a particle state")
            quat, trans, pR, pT = state[:4]
            for name, t, shp in (("quat", quat, (nImg, self.mLR, 4)), ("trans", trans, (nImg, self.mLT, 2)),
                                 ("pR", pR, (nImg, self.mLR)), ("pT", pT, (nImg, self.mLT))):
                ops._req(t, torch.float64, shp, name)
            cls = state[4] if len(state) > 4 else torch.zeros(nImg, dtype=torch.int32, device=dev)
            ops._req(cls, torch.int32, (nImg,), "cls")
            out = (quat, trans, pR, pT, torch.empty(nImg, dtype=torch.float32, device=dev), cls,
                   torch.empty(nImg, dtype=torch.int32, device=dev))
        elif out is None:
            out = (torch.empty(nImg, self.mLR, 4, dtype=torch.float64, device=dev),
                   torch.empty(nImg, self.mLT, 2, dtype=torch.float64, device=dev),
                   torch.empty(nImg, self.mLR, dtype=torch.float64, device=dev),
                   torch.empty(nImg, self.mLT, dtype=torch.float64, device=dev),
                   torch.empty(nImg, dtype=torch.float32, device=dev),
                   torch.empty(nImg, dtype=torch.int32, device=dev),
                   torch.empty(nImg, dtype=torch.int32, device=dev))
        quat, trans, pR, pT, score, cls, nph = out
        ws = ops.workspace(self.workspace_bytes(nImg), dev)
        P = ops._ptr
        if self.two_d:
            check(lib().thx_expectation2d(ctypes.byref(self.cfg), P(self.vol), P(self.gQuat),
                                          P(self.gTrans), P(self.gPR), P(self.gPT), P(dat), P(ctf),
                                          P(sig), P(self.px.d_iCol), P(self.px.d_iRow), nPxl, nImg,
                                          P(quat), P(trans), P(pR), P(pT), P(score), P(cls), P(nph),
                                          P(ws), ws.numel(), ops._stream(dev)), "thx_expectation2d")
            return out
        check(lib().thx_expectation(ctypes.byref(self.cfg), P(self.vol), P(self.gQuat),
                                    P(self.gTrans), P(self.gPR), P(self.gPT), P(dat), P(ctf),
                                    P(sig), P(self.px.d_iCol), P(self.px.d_iRow),
                                    P(self.px.d_order), len(self.px.order), nPxl, nImg,
                                    P(quat), P(trans), P(pR), P(pT), P(score), P(cls), P(nph),
                                    P(ws), ws.numel(), ops._stream(dev)), "thx_expectation")
        return out


class PhaseTimer:
    """HIP event pairs the driver records around every phase's k_local_fused
    launch (thx_expect_cfg.phaseEvents): attach to an Expectation, run, read
    the per-phase kernel milliseconds."""

    def __init__(self, expectation, n_pairs):
        self.n = n_pairs
        self.ev = ctypes.c_void_p()
        check(lib().thx_event_pairs_create(n_pairs, ctypes.byref(self.ev)), "thx_event_pairs_create")
        self.e = expectation
        expectation.cfg.phaseEvents = self.ev
        expectation.cfg.nPhaseEvents = n_pairs

    def select(self, first_pair):
        """Record the next run's phases into pairs first_pair, first_pair + 1, ..."""
        if not 0 <= first_pair <= self.n:
            raise ValueError("first_pair outside the timer's event pairs")
        self.e.cfg.phaseEvents = ctypes.c_void_p(self.ev.value + 2 * first_pair *
                                                 ctypes.sizeof(ctypes.c_void_p))
        self.e.cfg.nPhaseEvents = self.n - first_pair

    def ms(self):
        out = (ctypes.c_float * self.n)()
        check(lib().thx_event_pairs_elapsed(self.ev, self.n, out), "thx_event_pairs_elapsed")
        return [v for v in out if v >= 0]

    def close(self):
        self.e.cfg.phaseEvents = None
        self.e.cfg.nPhaseEvents = 0
        lib().thx_event_pairs_destroy(self.ev, self.n)


class Reconstructor:
    """Device half-map of one hemisphere: Reconstructor::insertP / insertI
    (src/Reconstructor.cpp:782-985) over thx_insert3d."""

    def __init__(self, idim, pf, device):
        self.hm = ops.HalfMap(pf * idim, device)
        self.pf = pf

    def insert(self, dat, ctf, quat, trans, offS, w, px, tiled=True):
        return ops.insert3d(self.hm, dat, ctf, quat, trans, offS, w, px, tiled=tiled)


def cloud_mode(quat):
    """Medoid of each image's rotation cloud [nImg, m, 4] (max sum of squared
    cosines to the other particles).  Systematic resampling leaves particles
    in ancestor order, so index 0 is not the top particle; this is the
    estimate of Particle::rank1st without the weights."""
    c = torch.einsum("lik,ljk->lij", quat, quat) ** 2
    return quat[torch.arange(quat.shape[0], device=quat.device), c.sum(-1).argmax(-1)]


def draw_insert_samples(quat, trans, m_reco, seed=11):
    """Particle::rand (src/Particle.cpp:2109-2200): mReco uniform draws from the
    final particle sets of each image -> (quat [nImg,mReco,4], trans [nImg,mReco,2])."""
    nImg, mR, _ = quat.shape
    mT = trans.shape[1]
    g = torch.Generator(device=quat.device).manual_seed(seed)
    ir = torch.randint(0, mR, (nImg, m_reco), generator=g, device=quat.device)
    it = torch.randint(0, mT, (nImg, m_reco), generator=g, device=quat.device)
    q = torch.gather(quat, 1, ir.unsqueeze(-1).expand(-1, -1, 4)).contiguous()
    t = torch.gather(trans, 1, it.unsqueeze(-1).expand(-1, -1, 2)).contiguous()
    return q, t


def hemisphere_shard(n_images, world, rank):
    """Particle indices owned by `rank`: gold-standard hemisphere = rank % 2
    (odd / even split of src/Parallel.cpp:26-53, images alternating between
    hemispheres), then one contiguous block per rank inside its hemisphere
    (Database::split, src/Database.cpp:621-641).  One rank keeps everything."""
    idx = np.arange(n_images)
    if world == 1:
        return idx
    hemi = rank % 2
    members = [r for r in range(world) if r % 2 == hemi]
    idx = idx[hemi::2]
    k = members.index(rank)
    per = (len(idx) + len(members) - 1) // len(members)
    return idx[k * per:(k + 1) * per]


def hemisphere_groups(world):
    """One process group per hemisphere; every rank must call this (collective)."""
    import torch.distributed as dist
    return [dist.new_group([r for r in range(world) if r % 2 == h]) for h in (0, 1)]


def halfmap_allreduce(hm, group=None):
    """RCCL sum of F, T, O, counter over the ranks of one hemisphere
    (the ncclAllReduce of gpu/src/cuthunder.cu:5903-5993, counter as int32)."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return hm
    for t in (hm.F, hm.T, hm.O, hm.counter):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return hm
