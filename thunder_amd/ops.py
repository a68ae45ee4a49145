"""torch-tensor front end of the C-ABI (include/thunder_amd.h).

PyTorch supplies device memory, the current HIP stream and torch.distributed;
all arithmetic runs in the hand-written gfx950 kernels of libthunder_amd.so.
Every function validates shapes / dtypes / devices on the host before a kernel
is enqueued (a mis-shaped launch must never reach the GPU).
"""
import ctypes
import math
import threading

import numpy as np
import torch

from ._lib import check, lib

_ws_cache = {}
_ws_lock = threading.Lock()


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _req(t, dtype, shape, name):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a device (cuda/HIP) tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")
    return t


def workspace(nbytes, device, stream=None):
    """Scratch for one call enqueued on ``stream`` (default: the device's
    current stream).  One buffer per (device, stream): calls on one stream are
    ordered, so they may share it, while calls on different streams (concurrent
    sub-batches, several host threads) never do -- a shared buffer would let
    one call's patch records, active lists and particle scratch overwrite
    another's.  The buffer is allocated with its stream current, so the
    caching allocator reuses its memory only in that stream's order."""
    dev = torch.device(device)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    key = (dev, stream.cuda_stream)
    with _ws_lock:
        buf = _ws_cache.get(key)
        if buf is None or buf.numel() < nbytes:
            with torch.cuda.stream(stream):
                buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=dev)
            _ws_cache[key] = buf
        return buf


def release_workspaces():
    """Drop the cached per-stream scratch buffers (e.g. before destroying streams)."""
    with _ws_lock:
        _ws_cache.clear()


# ------------------------------------------------------------------- a1
class PixelSet:
    """Pixel index set of Optimiser::allocPreCalIdx (src/Optimiser.cpp:7991-8041)."""

    def __init__(self, idim, pf, rU, rL, device=None):
        cap = (idim // 2 + 1) * idim
        bufs = [np.zeros(cap, np.int32) for _ in range(4)]
        n = ctypes.c_int(0)
        check(lib().thx_pixel_set(idim, pf, float(rU), float(rL), cap,
                                  *[b.ctypes.data_as(ctypes.c_void_p) for b in bufs],
                                  ctypes.byref(n)), "thx_pixel_set")
        n = n.value
        self.idim, self.pf, self.rU, self.rL, self.n = idim, pf, rU, rL, n
        self.iCol, self.iRow, self.iSig, self.iPxl = (b[:n].copy() for b in bufs)
        self.order = tile_order(self.iCol, self.iRow)
        self.device = device
        if device is not None:
            self.d_iCol = torch.from_numpy(self.iCol).to(device)
            self.d_iRow = torch.from_numpy(self.iRow).to(device)
            self.d_order = torch.from_numpy(self.order).to(device)


def tile_order(iCol, iRow):
    """thx_pixel_tile_order: local-phase visiting order of a pixel set
    (16-entry patches, -1 = padding)."""
    iCol = np.ascontiguousarray(iCol, np.int32)
    iRow = np.ascontiguousarray(iRow, np.int32)
    n = ctypes.c_int(0)
    vp = ctypes.c_void_p
    check(lib().thx_pixel_tile_order(iCol.ctypes.data_as(vp), iRow.ctypes.data_as(vp), len(iCol),
                                     0, None, ctypes.byref(n)), "thx_pixel_tile_order")
    order = np.zeros(n.value, np.int32)
    check(lib().thx_pixel_tile_order(iCol.ctypes.data_as(vp), iRow.ctypes.data_as(vp), len(iCol),
                                     len(order), order.ctypes.data_as(vp), ctypes.byref(n)),
          "thx_pixel_tile_order")
    return order


# ------------------------------------------------------------------- a2
def ctf(attr, px):
    """attr: [nImg, 8] float32 {pixelSize, voltage, dU, dV, theta, Cs, ampC, phaseShift}."""
    nImg = attr.shape[0]
    _req(attr, torch.float32, (nImg, 8), "attr")
    out = torch.empty(nImg, px.n, dtype=torch.float32, device=attr.device)
    check(lib().thx_ctf(_ptr(attr), nImg, _ptr(px.d_iCol), _ptr(px.d_iRow), px.n, px.idim,
                        _ptr(out), _stream(attr.device)), "thx_ctf")
    return out


def defocus_pre(attr, px):
    """CTF-search precalculation (allocPreCal's cSearch branch): freq [nPxl],
    defocusP [nImg, nPxl], K1, K2 [nImg]."""
    nImg = attr.shape[0]
    _req(attr, torch.float32, (nImg, 8), "attr")
    dev = attr.device
    freq = torch.empty(px.n, dtype=torch.float32, device=dev)
    dfo = torch.empty(nImg, px.n, dtype=torch.float32, device=dev)
    k1 = torch.empty(nImg, dtype=torch.float32, device=dev)
    k2 = torch.empty(nImg, dtype=torch.float32, device=dev)
    check(lib().thx_defocus_pre(_ptr(attr), nImg, _ptr(px.d_iCol), _ptr(px.d_iRow), px.n, px.idim,
                                _ptr(freq), _ptr(dfo), _ptr(k1), _ptr(k2), _stream(dev)),
          "thx_defocus_pre")
    return freq, dfo, k1, k2


def ctf_search(dfo, freq, dD, k1, k2, attr):
    """kernel_CalCTFL: ctfD [nImg, nD, nPxl] for the defocus factors dD [nImg, nD]."""
    nImg, nPxl = dfo.shape
    nD = dD.shape[1]
    _req(dfo, torch.float32, (nImg, nPxl), "defocusP")
    _req(freq, torch.float32, (nPxl,), "freq")
    _req(dD, torch.float64, (nImg, nD), "dD")
    _req(k1, torch.float32, (nImg,), "K1")
    _req(k2, torch.float32, (nImg,), "K2")
    _req(attr, torch.float32, (nImg, 8), "attr")
    out = torch.empty(nImg, nD, nPxl, dtype=torch.float32, device=dfo.device)
    check(lib().thx_ctf_search(_ptr(dfo), _ptr(freq), _ptr(dD), nD, _ptr(k1), _ptr(k2), _ptr(attr),
                               nImg, nPxl, _ptr(out), _stream(dfo.device)), "thx_ctf_search")
    return out


# ------------------------------------------------------------------- a3
def global_sample_sizes(mS, trans_s=10.0, trans_search_factor=0.25, n_sym_elem=0, mode=1):
    """(mS after the 3D clamp, nR, nT) of the global search (host function)."""
    out = [ctypes.c_int() for _ in range(3)]
    check(lib().thx_global_sample_sizes(mode, mS, n_sym_elem, float(trans_s),
                                        float(trans_search_factor),
                                        *[ctypes.byref(o) for o in out]), "thx_global_sample_sizes")
    return tuple(o.value for o in out)


def global_sample_set(nR, nT, trans_s, seed, device, sym=None):
    """Particle::reset's global set on device: (quat [nR,4], trans [nT,2], pR, pT);
    sym (a point-group name, non-C1): the rotations symmetrised towards the
    identity (Particle::reset's symmetrise(), src/Particle.cpp:168), the
    asymmetric unit the scan then covers (nR from global_sample_sizes with
    the group's n_sym_elem)."""
    quat = torch.empty(nR, 4, dtype=torch.float64, device=device)
    trans = torch.empty(nT, 2, dtype=torch.float64, device=device)
    pR = torch.empty(nR, dtype=torch.float64, device=device)
    pT = torch.empty(nT, dtype=torch.float64, device=device)
    check(lib().thx_global_sample_set(nR, nT, float(trans_s), seed, _ptr(quat), _ptr(trans),
                                      _ptr(pR), _ptr(pT), _stream(quat.device)),
          "thx_global_sample_set")
    if sym is not None:
        _, symQ = symmetry(sym)
        if len(symQ):
            pf_symmetrise(quat.view(1, nR, 4), symQ)
    return quat, trans, pR, pT


def global_sample_set2d(nR, nT, trans_s, seed, device):
    """Particle::reset's MODE_2D global set on device: (rot [nR,4] rows
    (cos, sin, 0, 0), trans [nT,2], pR, pT)."""
    rot = torch.empty(nR, 4, dtype=torch.float64, device=device)
    trans = torch.empty(nT, 2, dtype=torch.float64, device=device)
    pR = torch.empty(nR, dtype=torch.float64, device=device)
    pT = torch.empty(nT, dtype=torch.float64, device=device)
    check(lib().thx_global_sample_set2d(nR, nT, float(trans_s), seed, _ptr(rot), _ptr(trans),
                                        _ptr(pR), _ptr(pT), _stream(rot.device)),
          "thx_global_sample_set2d")
    return rot, trans, pR, pT


# ------------------------------------------------------------------- a4
def trans_table(trans, px):
    nT = trans.shape[0]
    _req(trans, torch.float64, (nT, 2), "trans")
    out = torch.empty(nT, px.n, dtype=torch.complex64, device=trans.device)
    check(lib().thx_trans_table(_ptr(trans), nT, _ptr(px.d_iCol), _ptr(px.d_iRow), px.n,
                                px.idim, _ptr(out), _stream(trans.device)), "thx_trans_table")
    return out


# ------------------------------------------------------------------- a5
def rotmat(quat):
    n = quat.shape[0]
    _req(quat, torch.float64, (n, 4), "quat")
    out = torch.empty(n, 9, dtype=torch.float64, device=quat.device)
    check(lib().thx_rotmat(_ptr(quat), n, _ptr(out), _stream(quat.device)), "thx_rotmat")
    return out


# ------------------------------------------------------------------- a6
def _vol_dim(vol):
    if vol.dim() != 3 or vol.shape[0] != vol.shape[1] or vol.shape[2] != vol.shape[0] // 2 + 1:
        raise ValueError(f"vol: expected [vdim, vdim, vdim/2+1] half-complex, got {tuple(vol.shape)}")
    _req(vol, torch.complex64, None, "vol")
    return vol.shape[0]


def project3d(vol, mat, px):
    vdim = _vol_dim(vol)
    if px.rU * px.pf >= vdim // 2 - 1:
        raise ValueError("pixel radius * pf reaches the volume edge")
    nR = mat.shape[0]
    _req(mat, torch.float64, (nR, 9), "mat")
    out = torch.empty(nR, px.n, dtype=torch.complex64, device=vol.device)
    for r0 in range(0, nR, 65535):
        nb = min(65535, nR - r0)
        check(lib().thx_project3d(_ptr(vol), vdim, px.pf, _ptr(mat[r0:r0 + nb]), nb,
                                  _ptr(px.d_iCol), _ptr(px.d_iRow), px.n, _ptr(out[r0:r0 + nb]),
                                  _stream(vol.device)), "thx_project3d")
    return out


# ------------------------------------------------------------------- a7
def _images(dat, ctf_, sig):
    nImg, nPxl = dat.shape
    _req(dat, torch.complex64, (nImg, nPxl), "dat")
    _req(ctf_, torch.float32, (nImg, nPxl), "ctf")
    _req(sig, torch.float32, (nImg, nPxl), "sigRcp")
    return nImg, nPxl


def dvp(rotP, traP, dat, ctf_, sig):
    nImg, nPxl = _images(dat, ctf_, sig)
    nR, nT = rotP.shape[0], traP.shape[0]
    _req(rotP, torch.complex64, (nR, nPxl), "rotP")
    _req(traP, torch.complex64, (nT, nPxl), "traP")
    out = torch.empty(nImg, nR, nT, dtype=torch.float32, device=dat.device)
    for l0 in range(0, nImg, 65535):
        nb = min(65535, nImg - l0)
        check(lib().thx_dvp(_ptr(rotP), nR, _ptr(traP), nT, _ptr(dat[l0:]), _ptr(ctf_[l0:]),
                            _ptr(sig[l0:]), nb, nPxl, _ptr(out[l0:]), _stream(dat.device)), "thx_dvp")
    return out


# ------------------------------------------------------------- a7 + a8
def global_scan(rotP, traP, dat, ctf_, sig, pR, pT, kIdx=0, nK=1, state=None, algo=4, guard=None,
                want_dvp=False):
    """ExpectGlobal3D: returns (wC [nImg,nK], wR [nImg,nK,nR], wT [nImg,nK,nT], baseL [nImg]).
    algo: 0 direct, 1 FP32 MFMA, 2 bf16x3 MFMA, 3 fp16x2, 4 bf16x6 MFMA (default, as the
    expectation driver).  want_dvp (algo 2-4): also return every sample's final dvp
    [nImg, nR, nT] (thx_global_scan_dvp); guard: the cancellation ratio of the
    direct-form recompute (None = the library's default, 0 = off)."""
    nImg, nPxl = _images(dat, ctf_, sig)
    nR, nT = rotP.shape[0], traP.shape[0]
    dev = dat.device
    _req(rotP, torch.complex64, (nR, nPxl), "rotP")
    _req(traP, torch.complex64, (nT, nPxl), "traP")
    _req(pR, torch.float64, (nR,), "pR")
    _req(pT, torch.float64, (nT,), "pT")
    if state is None:
        if kIdx != 0:
            raise ValueError("kIdx > 0 needs the running state of the earlier classes")
        state = (torch.zeros(nImg, nK, dtype=torch.float32, device=dev),
                 torch.zeros(nImg, nK, nR, dtype=torch.float32, device=dev),
                 torch.zeros(nImg, nK, nT, dtype=torch.float32, device=dev),
                 torch.full((nImg,), float("nan"), dtype=torch.float32, device=dev))
    wC, wR, wT, baseL = state
    _req(wC, torch.float32, (nImg, nK), "wC")
    _req(wR, torch.float32, (nImg, nK, nR), "wR")
    _req(wT, torch.float32, (nImg, nK, nT), "wT")
    _req(baseL, torch.float32, (nImg,), "baseL")
    nbytes = lib().thx_global_scan_workspace(nImg, nR, nT, nPxl, algo)
    ws = workspace(nbytes, dev)
    if want_dvp or guard is not None:
        # the dump only when asked for: a guard-only call runs the product
        # kernel's stores (no [nImg, nR, nT] write)
        dvp = torch.empty(nImg, nR, nT, dtype=torch.float32, device=dev) if want_dvp else None
        check(lib().thx_global_scan_dvp(_ptr(rotP), nR, _ptr(traP), nT, _ptr(dat), _ptr(ctf_),
                                        _ptr(sig), nImg, nPxl, _ptr(pR), _ptr(pT), kIdx, nK,
                                        _ptr(wC), _ptr(wR), _ptr(wT), _ptr(baseL), algo,
                                        4.0 if guard is None else float(guard),
                                        _ptr(dvp) if want_dvp else None,
                                        _ptr(ws), ws.numel(), _stream(dev)), "thx_global_scan_dvp")
        return (wC, wR, wT, baseL, dvp) if want_dvp else (wC, wR, wT, baseL)
    check(lib().thx_global_scan(_ptr(rotP), nR, _ptr(traP), nT, _ptr(dat), _ptr(ctf_), _ptr(sig),
                                nImg, nPxl, _ptr(pR), _ptr(pT), kIdx, nK, _ptr(wC), _ptr(wR),
                                _ptr(wT), _ptr(baseL), algo, _ptr(ws), ws.numel(), _stream(dev)),
          "thx_global_scan")
    return wC, wR, wT, baseL


# -------------------------------------------------------- a6 + a7 + a9
def volume_cells(vol):
    """Cell-expanded copy (8 taps per voxel, 64 B) for HBM-bound gathers."""
    vdim = _vol_dim(vol)
    out = torch.empty(vdim, vdim, vdim // 2 + 1, 8, dtype=torch.complex64, device=vol.device)
    check(lib().thx_volume_cells(_ptr(vol), vdim, _ptr(out), _stream(vol.device)), "thx_volume_cells")
    return out


def _layout(vol, cells, ypair=None):
    """(volLayout, volume argument) of thx_local_phase for the given copy:
    0 half-complex, 1 cells, 2 y-pair (pair form)."""
    if cells is not None and ypair is not None:
        raise ValueError("cells and ypair are alternatives")
    if ypair is not None:
        _req(ypair, torch.complex64, _ypair_shape(vol), "ypair")
        return 2, ypair
    if cells is not None:
        _req(cells, torch.complex64, tuple(vol.shape) + (8,), "cells")
        return 1, cells
    return 0, vol


def _ypair_shape(vol):
    """[vdim/2, vdim, vdim/2+1, 2 (z parity), 2 (y, y+1)] of thx_volume_ypair."""
    vdim = vol.shape[0]
    return (vdim // 2, vdim, vol.shape[2], 2, 2)


def volume_ypair(vol):
    """y-pair copy (thx_volume_ypair): yp[zp, y, x, zl] = (v(x, y, z), v(x, y+1, z))
    for z = 2 zp + zl -- the slices z, z+1 of each even z interleaved, so a
    trilinear cell at even z0 is one 64-B piece, else two 32-B pieces."""
    vdim = _vol_dim(vol)
    out = torch.empty(_ypair_shape(vol), dtype=torch.complex64, device=vol.device)
    check(lib().thx_volume_ypair(_ptr(vol), vdim, _ptr(out), _stream(vol.device)),
          "thx_volume_ypair")
    return out


def ypair_ball_radius(px):
    """R of the driver's compact y-pair ball for a pixel set: ceil(pf r_max) + 2."""
    r2 = int(np.max(px.iCol.astype(np.int64) ** 2 + px.iRow.astype(np.int64) ** 2))
    return int(math.ceil(px.pf * math.sqrt(r2))) + 2


def volume_ypair_ball(vol, R):
    """thx_volume_ypair_ball: the compact y-pair ball of radius R the driver
    gathers from ([elements, 2] complex64: (v(x, y, z), v(x, y+1, z)))."""
    vdim = _vol_dim(vol)
    n = lib().thx_ypair_ball_elems(R)
    out = torch.empty(n, 2, dtype=torch.complex64, device=vol.device)
    check(lib().thx_volume_ypair_ball(_ptr(vol), vdim, R, _ptr(out), _stream(vol.device)),
          "thx_volume_ypair_ball")
    return out


def local_phase(vol, quat, trans, pC, pR, pT, dat, ctf_, sig, px, want_dvp=False, cells=None,
                tiled=True, ypair=None, routed=False, ball=None, ball_r=0):
    """cells / ypair: optional thx_volume_cells / thx_volume_ypair copy of vol.
    tiled: visit pixels in px.order (LDS-staged neighbourhoods) instead of set order.
    routed: the device route of thx_local_phase_routed (vol half-complex, ypair
    optional, pxOrder), which then also returns the kernel it picked (0 staged,
    1 box-less, 2 y-pair, -1 not routed) as a sixth value; with ball (the
    volume_ypair_ball of radius ball_r) instead of ypair, the driver's
    thx_local_phase_routed_ball."""
    if ball is not None:
        if not routed or ypair is not None or ball_r <= 0:
            raise ValueError("ball: routed phase with ball_r > 0 and no ypair")
        _req(ball, torch.complex64, (lib().thx_ypair_ball_elems(ball_r), 2), "ball")
    vdim = _vol_dim(vol)
    layout, src = (0, vol) if routed else _layout(vol, cells, ypair)
    if routed and (cells is not None or not tiled):
        raise ValueError("the routed phase takes the half-complex volume and the tile order")
    nImg, nPxl = _images(dat, ctf_, sig)
    if nPxl != px.n:
        raise ValueError("pixel set / image size mismatch")
    nR, nT = quat.shape[1], trans.shape[1]
    dev = dat.device
    _req(quat, torch.float64, (nImg, nR, 4), "quat")
    _req(trans, torch.float64, (nImg, nT, 2), "trans")
    _req(pC, torch.float64, (nImg,), "pC")
    _req(pR, torch.float64, (nImg, nR), "pR")
    _req(pT, torch.float64, (nImg, nT), "pT")
    if routed and ypair is not None:
        _req(ypair, torch.complex64, _ypair_shape(vol), "ypair")
    wC = torch.empty(nImg, dtype=torch.float32, device=dev)
    wR = torch.empty(nImg, nR, dtype=torch.float32, device=dev)
    wT = torch.empty(nImg, nT, dtype=torch.float32, device=dev)
    base = torch.empty(nImg, dtype=torch.float32, device=dev)
    d = torch.empty(nImg, nR, nT, dtype=torch.float32, device=dev) if want_dvp else None
    route = torch.full((1,), -2, dtype=torch.int32, device=dev)
    ws = workspace(lib().thx_local_phase_workspace(min(nImg, 65535), nR, nT,
                                                   len(px.order) if tiled else nPxl), dev)
    for l0 in range(0, nImg, 65535):
        nb = min(65535, nImg - l0)
        if routed and ball is not None:
            check(lib().thx_local_phase_routed_ball(None, _ptr(vol), _ptr(ball), ball_r, vdim, px.pf,
                                                    _ptr(quat[l0:]), nR, _ptr(trans[l0:]), nT,
                                                    _ptr(pC[l0:]), _ptr(pR[l0:]), _ptr(pT[l0:]),
                                                    _ptr(dat[l0:]), _ptr(ctf_[l0:]), _ptr(sig[l0:]),
                                                    _ptr(px.d_iCol), _ptr(px.d_iRow), _ptr(px.d_order),
                                                    len(px.order), nPxl, px.idim, nb, _ptr(wC[l0:]),
                                                    _ptr(wR[l0:]), _ptr(wT[l0:]), _ptr(base[l0:]),
                                                    _ptr(d[l0:]) if d is not None else None, _ptr(route),
                                                    _ptr(ws), ws.numel(), _stream(dev)),
                  "thx_local_phase_routed_ball")
            continue
        if routed:
            check(lib().thx_local_phase_routed(None, _ptr(vol), _ptr(ypair) if ypair is not None else None,
                                               vdim, px.pf, _ptr(quat[l0:]), nR, _ptr(trans[l0:]), nT,
                                               _ptr(pC[l0:]), _ptr(pR[l0:]), _ptr(pT[l0:]),
                                               _ptr(dat[l0:]), _ptr(ctf_[l0:]), _ptr(sig[l0:]),
                                               _ptr(px.d_iCol), _ptr(px.d_iRow), _ptr(px.d_order),
                                               len(px.order), nPxl, px.idim, nb, _ptr(wC[l0:]),
                                               _ptr(wR[l0:]), _ptr(wT[l0:]), _ptr(base[l0:]),
                                               _ptr(d[l0:]) if d is not None else None, _ptr(route),
                                               _ptr(ws), ws.numel(), _stream(dev)),
                  "thx_local_phase_routed")
            continue
        check(lib().thx_local_phase(_ptr(src), layout, vdim, px.pf, _ptr(quat[l0:]), nR,
                                    _ptr(trans[l0:]),
                                    nT, _ptr(pC[l0:]), _ptr(pR[l0:]), _ptr(pT[l0:]), _ptr(dat[l0:]),
                                    _ptr(ctf_[l0:]), _ptr(sig[l0:]), _ptr(px.d_iCol),
                                    _ptr(px.d_iRow), _ptr(px.d_order) if tiled else None,
                                    len(px.order), nPxl, px.idim, nb, _ptr(wC[l0:]),
                                    _ptr(wR[l0:]), _ptr(wT[l0:]), _ptr(base[l0:]),
                                    _ptr(d[l0:]) if d is not None else None, _ptr(ws),
                                    ws.numel(), _stream(dev)), "thx_local_phase")
    if routed:
        return wC, wR, wT, base, d, int(route.item())
    return wC, wR, wT, base, d


def local_phase_d(vol, quat, trans, pC, pR, pT, pD, dat, ctfD, sig, px, want_dvp=False,
                  cells=None, tiled=True):
    """CTF-search phase (thx_local_phase_d): ctfD [nImg, nD, nPxl], pD [nImg, nD];
    returns wC, wR, wT, wD, baseL, dvp [nImg, nR, nT, nD] (or None)."""
    vdim = _vol_dim(vol)
    layout, src = _layout(vol, cells)
    nImg, nPxl = dat.shape
    nR, nT, nD = quat.shape[1], trans.shape[1], pD.shape[1]
    dev = dat.device
    _req(dat, torch.complex64, (nImg, nPxl), "dat")
    _req(ctfD, torch.float32, (nImg, nD, nPxl), "ctfD")
    _req(sig, torch.float32, (nImg, nPxl), "sig")
    if nPxl != px.n:
        raise ValueError("pixel set / image size mismatch")
    _req(quat, torch.float64, (nImg, nR, 4), "quat")
    _req(trans, torch.float64, (nImg, nT, 2), "trans")
    _req(pC, torch.float64, (nImg,), "pC")
    _req(pR, torch.float64, (nImg, nR), "pR")
    _req(pT, torch.float64, (nImg, nT), "pT")
    _req(pD, torch.float64, (nImg, nD), "pD")
    if nImg > 65535:
        raise ValueError("local_phase_d: at most 65535 images per call")
    wC = torch.empty(nImg, dtype=torch.float32, device=dev)
    wR = torch.empty(nImg, nR, dtype=torch.float32, device=dev)
    wT = torch.empty(nImg, nT, dtype=torch.float32, device=dev)
    wD = torch.empty(nImg, nD, dtype=torch.float32, device=dev)
    base = torch.empty(nImg, dtype=torch.float32, device=dev)
    d = torch.empty(nImg, nR, nT, nD, dtype=torch.float32, device=dev) if want_dvp else None
    ws = workspace(lib().thx_local_phase_workspace(nImg, nR, nT * nD,
                                                   len(px.order) if tiled else nPxl), dev)
    check(lib().thx_local_phase_d(None, _ptr(src), layout, vdim, px.pf,
                                  _ptr(quat), nR, _ptr(trans), nT, nD, _ptr(pC), _ptr(pR),
                                  _ptr(pT), _ptr(pD), _ptr(dat), _ptr(ctfD), _ptr(sig),
                                  _ptr(px.d_iCol), _ptr(px.d_iRow),
                                  _ptr(px.d_order) if tiled else None, len(px.order), nPxl,
                                  px.idim, nImg, _ptr(wC), _ptr(wR), _ptr(wT), _ptr(wD),
                                  _ptr(base), _ptr(d), _ptr(ws), ws.numel(), _stream(dev)),
          "thx_local_phase_d")
    return wC, wR, wT, wD, base, d


# ------------------------------------------------------------------ a10
def resample(w, u, n_out, u0):
    nImg, nIn = w.shape
    dev = w.device
    _req(w, torch.float64, (nImg, nIn), "w")
    _req(u, torch.float32, (nImg, nIn), "u")
    _req(u0, torch.float64, (nImg,), "u0")
    anc = torch.empty(nImg, n_out, dtype=torch.int32, device=dev)
    wout = torch.empty(nImg, n_out, dtype=torch.float64, device=dev)
    imax = torch.empty(nImg, dtype=torch.int32, device=dev)
    check(lib().thx_resample(nImg, nIn, _ptr(w), _ptr(u), n_out, _ptr(u0), _ptr(anc), _ptr(wout),
                             _ptr(imax), _stream(dev)), "thx_resample")
    return anc, wout, imax


# ------------------------------------------------------------------ a12
class HalfMap:
    """Device F/T/O/counter accumulators of one Reconstructor (padded box vdim)."""

    def __init__(self, vdim, device):
        self.vdim = vdim
        self.F = torch.zeros(vdim, vdim, vdim // 2 + 1, dtype=torch.complex64, device=device)
        self.T = torch.zeros(vdim, vdim, vdim // 2 + 1, dtype=torch.float32, device=device)
        self.O = torch.zeros(3, dtype=torch.float64, device=device)
        self.counter = torch.zeros(1, dtype=torch.int32, device=device)


def insert_method(hm, mReco, px):
    """The insert variant the front end uses: the binned deposition when its
    limits hold (mReco <= 1024, tile grid <= 16384 tiles), else LDS patches."""
    rMax = int(math.ceil(px.rU))
    R = px.pf * rMax + 2
    nt = ((R + 15) // 16) * ((2 * R + 15) // 16) ** 2
    if mReco <= 1024 and nt <= 16384 and R <= hm.vdim // 2 - 1:
        return "binned"
    return "tiled"


def insert3d(hm, dat, ctf_, quat, trans, offS, w, px, tiled=True, nC=None, method=None):
    """method: "binned" (thx_insert3d_binned), "tiled" (LDS patches,
    thx_insert3d_tiled) or "direct" (one memory-side atomic per tap,
    thx_insert3d); default: binned where its limits hold, else tiled;
    tiled=False selects direct.  nC: optional int32 [nImg], image l inserts
    only its first nC[l] samples (the K-class InsertFT call)."""
    nImg, nPxl = dat.shape
    _req(dat, torch.complex64, (nImg, nPxl), "dat")
    _req(ctf_, torch.float32, (nImg, nPxl), "ctf")
    mReco = quat.shape[1]
    _req(quat, torch.float64, (nImg, mReco, 4), "quat")
    _req(trans, torch.float64, (nImg, mReco, 2), "trans")
    _req(offS, torch.float64, (nImg, 2), "offS")
    _req(w, torch.float32, (nImg,), "w")
    if nC is not None:
        _req(nC, torch.int32, (nImg,), "nC")
    if nPxl != px.n:
        raise ValueError("pixel set / image size mismatch")
    if px.rU * px.pf >= hm.vdim // 2 - 1:
        raise ValueError("pixel radius * pf reaches the volume edge")
    if method is None:
        method = insert_method(hm, mReco, px) if tiled else "direct"
    dev = dat.device
    if method == "binned":
        rMax = int(math.ceil(px.rU))
        ws = workspace(lib().thx_insert3d_binned_workspace(nImg, mReco, len(px.order), px.pf, rMax),
                       dev)
        check(lib().thx_insert3d_binned(
            _ptr(hm.F), _ptr(hm.T), _ptr(hm.O), _ptr(hm.counter), hm.vdim, px.pf, _ptr(dat),
            _ptr(ctf_), _ptr(quat), _ptr(trans), _ptr(offS), _ptr(w),
            _ptr(nC) if nC is not None else None, nImg, mReco, _ptr(px.d_iCol), _ptr(px.d_iRow),
            _ptr(px.d_order), len(px.order), nPxl, px.idim, rMax, _ptr(ws), ws.numel(),
            _stream(dev)), "thx_insert3d_binned")
        return hm
    if method == "tiled":
        ws = workspace(lib().thx_insert3d_workspace(min(nImg, 65535), mReco, len(px.order)), dev)
    elif method != "direct":
        raise ValueError(f"unknown insert method {method!r}")
    for l0 in range(0, nImg, 65535):
        nb = min(65535, nImg - l0)
        nCp = _ptr(nC[l0:]) if nC is not None else None
        if method == "tiled":
            check(lib().thx_insert3d_tiled(
                _ptr(hm.F), _ptr(hm.T), _ptr(hm.O), _ptr(hm.counter), hm.vdim, px.pf,
                _ptr(dat[l0:]), _ptr(ctf_[l0:]), _ptr(quat[l0:]), _ptr(trans[l0:]), _ptr(offS[l0:]),
                _ptr(w[l0:]), nCp, nb, mReco, _ptr(px.d_iCol), _ptr(px.d_iRow), _ptr(px.d_order),
                len(px.order), nPxl, px.idim, _ptr(ws), ws.numel(), _stream(dev)),
                "thx_insert3d_tiled")
            continue
        check(lib().thx_insert3d(_ptr(hm.F), _ptr(hm.T), _ptr(hm.O), _ptr(hm.counter), hm.vdim,
                                 px.pf, _ptr(dat[l0:]), _ptr(ctf_[l0:]), _ptr(quat[l0:]),
                                 _ptr(trans[l0:]), _ptr(offS[l0:]), _ptr(w[l0:]), nCp, nb, mReco,
                                 _ptr(px.d_iCol), _ptr(px.d_iRow), nPxl, px.idim, _stream(dev)),
              "thx_insert3d")
    return hm


def insert3d_ctf(hm, dat, attr, nD, quat, trans, offS, w, px, nC=None):
    """CTF-search insert (thx_insert3d_binned_d): sample (l, m) with the CTF of
    attr[l] at defocus factor nD[l, m]."""
    nImg, nPxl = dat.shape
    mReco = quat.shape[1]
    _req(dat, torch.complex64, (nImg, nPxl), "dat")
    _req(attr, torch.float32, (nImg, 8), "attr")
    _req(nD, torch.float64, (nImg, mReco), "nD")
    _req(quat, torch.float64, (nImg, mReco, 4), "quat")
    _req(trans, torch.float64, (nImg, mReco, 2), "trans")
    _req(offS, torch.float64, (nImg, 2), "offS")
    _req(w, torch.float32, (nImg,), "w")
    if nC is not None:
        _req(nC, torch.int32, (nImg,), "nC")
    if nPxl != px.n:
        raise ValueError("pixel set / image size mismatch")
    if insert_method(hm, mReco, px) != "binned":
        raise ValueError("CTF-search insert needs the binned deposition's limits "
                         "(mReco <= 1024, tile grid <= 16384)")
    dev = dat.device
    rMax = int(math.ceil(px.rU))
    ws = workspace(lib().thx_insert3d_binned_workspace(nImg, mReco, len(px.order), px.pf, rMax), dev)
    check(lib().thx_insert3d_binned_d(
        _ptr(hm.F), _ptr(hm.T), _ptr(hm.O), _ptr(hm.counter), hm.vdim, px.pf, _ptr(dat),
        _ptr(attr), _ptr(nD), _ptr(quat), _ptr(trans), _ptr(offS), _ptr(w), _ptr(nC), nImg, mReco,
        _ptr(px.d_iCol), _ptr(px.d_iRow), _ptr(px.d_order), len(px.order), nPxl, px.idim, rMax,
        _ptr(ws), ws.numel(), _stream(dev)), "thx_insert3d_binned_d")
    return hm


# ------------------------------------------------------------------ a13
class RcclComm:
    """RCCL communicator of one hemisphere for thx_halfmap_allreduce, built
    from a unique id the caller moves between its ranks (MPI_Bcast in THUNDER;
    ``from_group`` uses torch.distributed)."""

    ID_BYTES = 128

    def __init__(self, nranks, uid, rank):
        self.comm = ctypes.c_void_p()
        buf = (ctypes.c_char * self.ID_BYTES).from_buffer_copy(bytes(uid))
        check(lib().thx_rccl_comm_init(nranks, buf, rank, ctypes.byref(self.comm)),
              "thx_rccl_comm_init")
        self.nranks, self.rank = nranks, rank

    @staticmethod
    def unique_id():
        buf = (ctypes.c_char * RcclComm.ID_BYTES)()
        check(lib().thx_rccl_unique_id(buf), "thx_rccl_unique_id")
        return bytes(buf)

    @classmethod
    def from_group(cls, group, device):
        """Collective over ``group``: its first rank draws the id, a broadcast
        hands it to the others (the MPI_Bcast of gpu/src/cuthunder.cu:5309-5322)."""
        import torch.distributed as dist
        ranks = dist.get_process_group_ranks(group)
        me = dist.get_rank()
        t = torch.zeros(cls.ID_BYTES, dtype=torch.uint8, device=device)
        if me == ranks[0]:
            t.copy_(torch.frombuffer(bytearray(cls.unique_id()), dtype=torch.uint8))
        dist.broadcast(t, src=ranks[0], group=group)
        return cls(len(ranks), t.cpu().numpy().tobytes(), ranks.index(me))

    def allreduce(self, hm, nK=1):
        """thx_halfmap_allreduce: in-place sum of F, T, O, counter."""
        dim = hm.T.numel() // nK
        check(lib().thx_halfmap_allreduce(self.comm, _ptr(hm.F), _ptr(hm.T), _ptr(hm.O),
                                          _ptr(hm.counter), dim, nK, _stream(hm.F.device)),
              "thx_halfmap_allreduce")
        return hm

    def sendrecv(self, send=None, peer_send=-1, recv=None, peer_recv=-1, n_recv=0):
        """thx_halfmap_sendrecv: float32 device tensors, ranks of this communicator."""
        ns = send.numel() if send is not None else 0
        nr = n_recv if recv is not None else 0
        if recv is not None and recv.numel() < nr:
            raise ValueError("recv buffer smaller than n_recv")
        dev = (send if send is not None else recv).device
        check(lib().thx_halfmap_sendrecv(self.comm, _ptr(send), ns, peer_send, _ptr(recv), nr,
                                         peer_recv, _stream(dev)), "thx_halfmap_sendrecv")

    def close(self):
        if self.comm:
            check(lib().thx_rccl_comm_destroy(self.comm), "thx_rccl_comm_destroy")
            self.comm = ctypes.c_void_p()


# ------------------------------------------------------------------- f4
def _img2d_dim(vol):
    if vol.dim() not in (2, 3) or vol.shape[-1] != vol.shape[-2] // 2 + 1:
        raise ValueError(f"2D projectee: expected [(nK,) vdim, vdim/2+1], got {tuple(vol.shape)}")
    _req(vol, torch.complex64, None, "vol")
    return vol.shape[-2]


def project2d(vol, rot, px):
    """thx_project2d: vol [vdim, vdim/2+1] complex64, rot [nR, 2] (cos, sin)."""
    vdim = _img2d_dim(vol)
    if px.rU * px.pf >= vdim // 2 - 1:
        raise ValueError("pixel radius * pf reaches the image edge")
    nR = rot.shape[0]
    _req(rot, torch.float64, (nR, 2), "rot")
    out = torch.empty(nR, px.n, dtype=torch.complex64, device=vol.device)
    check(lib().thx_project2d(_ptr(vol), vdim, px.pf, _ptr(rot), nR, _ptr(px.d_iCol),
                              _ptr(px.d_iRow), px.n, _ptr(out), _stream(vol.device)), "thx_project2d")
    return out


def local_phase2d(vol, rot, trans, pC, pR, pT, dat, ctf_, sig, px, cls=None, want_dvp=False):
    """thx_local_phase2d: vol [(nK,) vdim, vdim/2+1]; rot [nImg, mR, 2]; cls int32 [nImg]."""
    vdim = _img2d_dim(vol)
    nImg, nPxl = _images(dat, ctf_, sig)
    nR, nT = rot.shape[1], trans.shape[1]
    dev = dat.device
    _req(rot, torch.float64, (nImg, nR, 2), "rot")
    _req(trans, torch.float64, (nImg, nT, 2), "trans")
    for name, t, shp in (("pC", pC, (nImg,)), ("pR", pR, (nImg, nR)), ("pT", pT, (nImg, nT))):
        _req(t, torch.float64, shp, name)
    if cls is not None:
        _req(cls, torch.int32, (nImg,), "cls")
        if vol.dim() != 3:
            raise ValueError("cls needs [nK, vdim, vdim/2+1] projectees")
    wC = torch.empty(nImg, dtype=torch.float32, device=dev)
    wR = torch.empty(nImg, nR, dtype=torch.float32, device=dev)
    wT = torch.empty(nImg, nT, dtype=torch.float32, device=dev)
    base = torch.empty(nImg, dtype=torch.float32, device=dev)
    d = torch.empty(nImg, nR, nT, dtype=torch.float32, device=dev) if want_dvp else None
    ws = workspace(lib().thx_local_phase2d_workspace(nImg, nR, nT), dev)
    check(lib().thx_local_phase2d(_ptr(vol), vdim, px.pf, _ptr(cls), _ptr(rot), nR, _ptr(trans), nT,
                                  _ptr(pC), _ptr(pR), _ptr(pT), _ptr(dat), _ptr(ctf_), _ptr(sig),
                                  _ptr(px.d_iCol), _ptr(px.d_iRow), nPxl, px.idim, nImg, _ptr(wC),
                                  _ptr(wR), _ptr(wT), _ptr(base), _ptr(d), _ptr(ws), ws.numel(),
                                  _stream(dev)), "thx_local_phase2d")
    return wC, wR, wT, base, d


class HalfMap2D:
    """Device F / T / O / counter of nK 2D class reconstructors (padded box vdim)."""

    def __init__(self, vdim, nK, device):
        self.vdim, self.nK = vdim, nK
        self.F = torch.zeros(nK, vdim, vdim // 2 + 1, dtype=torch.complex64, device=device)
        self.T = torch.zeros(nK, vdim, vdim // 2 + 1, dtype=torch.float32, device=device)
        self.O = torch.zeros(nK, 2, dtype=torch.float64, device=device)
        self.counter = torch.zeros(nK, dtype=torch.int32, device=device)


def insert2d(hm, dat, ctf_, rot, trans, offS, w, px, nc=None):
    """thx_insert2d: rot / trans [nImg, mReco, 2], nc int32 [nImg, mReco] (classes)."""
    nImg, nPxl = dat.shape
    _req(dat, torch.complex64, (nImg, nPxl), "dat")
    _req(ctf_, torch.float32, (nImg, nPxl), "ctf")
    mReco = rot.shape[1]
    _req(rot, torch.float64, (nImg, mReco, 2), "rot")
    _req(trans, torch.float64, (nImg, mReco, 2), "trans")
    _req(offS, torch.float64, (nImg, 2), "offS")
    _req(w, torch.float32, (nImg,), "w")
    if nc is not None:
        _req(nc, torch.int32, (nImg, mReco), "nc")
        if int(nc.min()) < 0 or int(nc.max()) >= hm.nK:
            raise ValueError("class index out of range")
    if px.rU * px.pf >= hm.vdim // 2 - 1:
        raise ValueError("pixel radius * pf reaches the image edge")
    dev = dat.device
    for l0 in range(0, nImg, 65535):
        nb = min(65535, nImg - l0)
        check(lib().thx_insert2d(_ptr(hm.F), _ptr(hm.T), _ptr(hm.O), _ptr(hm.counter), hm.vdim,
                                 px.pf, _ptr(dat[l0:]), _ptr(ctf_[l0:]), _ptr(rot[l0:]),
                                 _ptr(trans[l0:]), _ptr(offS[l0:]), _ptr(w[l0:]),
                                 _ptr(nc[l0:]) if nc is not None else None, nb, mReco,
                                 _ptr(px.d_iCol), _ptr(px.d_iRow), nPxl, px.idim, _stream(dev)),
              "thx_insert2d")
    return hm


# ------------------------------------------------------------------- f1
def prepare_tf2d(hm):
    """thx_prepare_tf2d on a HalfMap2D in place: F_k, T_k /= T_k[0]."""
    check(lib().thx_prepare_tf2d(_ptr(hm.F), _ptr(hm.T), hm.vdim, hm.nK, _stream(hm.F.device)),
          "thx_prepare_tf2d")
    return hm


def reconstruct2d(hm, N, pf=2, a=1.9, alpha=15.0, grid_corr=True, max_radius=0, fsc=None,
                  join_half=False):
    """thx_reconstruct2d: the nK class images of HalfMap2D hm (T modified in
    place); returns (images [nK, N, N] real space, origin at [0, 0],
    iterations per class)."""
    vdim = pf * N
    if hm.vdim != vdim:
        raise ValueError("half-map box != pf N")
    dev = hm.F.device
    nK = hm.nK
    dst = torch.empty(nK, N, N, dtype=torch.float32, device=dev)
    it = (ctypes.c_int * nK)()
    fs = None
    if fsc is not None:
        fs = torch.as_tensor(np.ascontiguousarray(np.atleast_2d(fsc)), dtype=torch.float64,
                             device=dev)
        if fs.shape[0] != nK:
            raise ValueError("fsc: one row per class")
    ws = workspace(lib().thx_reconstruct2d_workspace(N, pf, nK), dev)
    check(lib().thx_reconstruct2d(_ptr(hm.F), _ptr(hm.T), nK, N, pf, float(a), float(alpha),
                                  int(bool(grid_corr)), int(max_radius), _ptr(fs),
                                  fs.shape[1] if fs is not None else 0, int(bool(join_half)),
                                  _ptr(dst), it, _ptr(ws), ws.numel(), _stream(dev)),
          "thx_reconstruct2d")
    return dst, list(it)


# --------------------------------------------------------- point groups
def symmetry(name):
    """thx_symmetry: (R [n, 3, 3] row-major, quat [n, 4]) float64 numpy of the
    non-identity elements of point group `name` ("C4", "D2", "T", "O", "I1"..)."""
    n = ctypes.c_int(0)
    check(lib().thx_symmetry(name.encode(), 0, None, None, ctypes.byref(n)), "thx_symmetry")
    R = np.zeros((max(n.value, 1), 3, 3))
    Q = np.zeros((max(n.value, 1), 4))
    check(lib().thx_symmetry(name.encode(), max(n.value, 1), R.ctypes.data_as(ctypes.c_void_p),
                             Q.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)), "thx_symmetry")
    return R[:n.value], Q[:n.value]


def symmetrize_ft(vol, R, r):
    """thx_symmetrize_ft of a half-complex volume (complex64 F or float32 T)
    with the symmetry matrices R (device or numpy [n, 3, 3]); returns a new tensor."""
    if vol.dim() != 3 or vol.shape[-1] != vol.shape[0] // 2 + 1 or vol.shape[1] != vol.shape[0]:
        raise ValueError("half-complex volume [vdim, vdim, vdim/2+1] expected")
    cplx = vol.dtype == torch.complex64
    if not cplx:
        _req(vol, torch.float32, None, "vol")
    Rd = torch.as_tensor(np.ascontiguousarray(R, np.float64).reshape(-1, 9) if not torch.is_tensor(R)
                         else R.reshape(-1, 9), dtype=torch.float64, device=vol.device).contiguous()
    out = torch.empty_like(vol)
    check(lib().thx_symmetrize_ft(_ptr(vol), _ptr(out), int(cplx), vol.shape[0], _ptr(Rd),
                                  Rd.shape[0], float(r), _stream(vol.device)), "thx_symmetrize_ft")
    return out


def prepare_tf(hm, R, max_radius, pf):
    """thx_prepare_tf on half-map hm in place: F, T /= T[0], then symmetrized
    (Reconstructor::prepareTF); R: [n, 3, 3] (n = 0: normalise only)."""
    dev = hm.F.device
    R = np.asarray(R, np.float64).reshape(-1, 9)
    Rd = torch.as_tensor(np.ascontiguousarray(R), device=dev) if len(R) else None
    ws = workspace(lib().thx_prepare_tf_workspace(hm.vdim), dev)
    check(lib().thx_prepare_tf(_ptr(hm.F), _ptr(hm.T), hm.vdim, _ptr(Rd), len(R), int(max_radius),
                               int(pf), _ptr(ws), ws.numel(), _stream(dev)), "thx_prepare_tf")
    return hm


def pf_symmetrise(quat, symQ, anchor_mode=0, anchor=None, seed=0, stream_id=0):
    """thx_pf_symmetrise of clouds quat [nImg, mR, 4] (device float64) in place."""
    nImg, mR = quat.shape[:2]
    _req(quat, torch.float64, (nImg, mR, 4), "quat")
    Q = torch.as_tensor(np.ascontiguousarray(symQ, np.float64), device=quat.device).reshape(-1, 4)
    if anchor is not None:
        _req(anchor, torch.float64, (nImg, 4), "anchor")
    check(lib().thx_pf_symmetrise(nImg, mR, _ptr(quat), int(anchor_mode), _ptr(anchor), _ptr(Q),
                                  Q.shape[0], int(seed), int(stream_id), _stream(quat.device)),
          "thx_pf_symmetrise")
    return quat


def reconstruct(hm, N, pf=2, a=1.9, alpha=15.0, grid_corr=True, max_radius=0, fsc=None,
                join_half=False, want_ft=True):
    """thx_reconstruct: the reconstruction solve of half-map hm (F, T at box
    pf N; T is modified in place).  Returns (map [N, N, N] real space, origin
    at [0, 0, 0], map_ft [N, N, N/2+1] complex or None, iterations, diffs)."""
    vdim = pf * N
    if hm.vdim != vdim:
        raise ValueError("half-map box != pf N")
    dev = hm.F.device
    dst = torch.empty(N, N, N, dtype=torch.float32, device=dev)
    dft = torch.empty(N, N, N // 2 + 1, dtype=torch.complex64, device=dev) if want_ft else None
    n_it = ctypes.c_int(0)
    diffs = (ctypes.c_float * 32)()
    fs = None
    if fsc is not None:
        fs = torch.as_tensor(np.ascontiguousarray(fsc), dtype=torch.float64, device=dev)
    ws = workspace(lib().thx_reconstruct_workspace(N, pf), dev)
    check(lib().thx_reconstruct(_ptr(hm.F), _ptr(hm.T), N, pf, a, alpha, int(bool(grid_corr)),
                                max_radius, int(fs is not None), _ptr(fs),
                                0 if fs is None else fs.numel(), int(bool(join_half)), _ptr(dst),
                                _ptr(dft), ctypes.byref(n_it), diffs, _ptr(ws), ws.numel(),
                                _stream(dev)), "thx_reconstruct")
    return dst, dft, n_it.value, [diffs[k] for k in range(n_it.value)]


# ------------------------------------------------------------------ a14
def fsc(A, B, n_shell):
    vdim = _vol_dim(A)
    _req(B, torch.complex64, tuple(A.shape), "B")
    out = torch.empty(n_shell, dtype=torch.float64, device=A.device)
    ws = workspace(lib().thx_fsc_workspace(n_shell), A.device)
    check(lib().thx_fsc(_ptr(A), _ptr(B), vdim, n_shell, _ptr(out), _ptr(ws), ws.numel(),
                        _stream(A.device)), "thx_fsc")
    return out


def pf_resample(w, u, n_out, seed, stream_id=0, shuffle=True):
    """thx_pf_resample (the driver's resampling kernel): w [nImg, nIn] float64
    (or [nIn], shared), u [nImg, nIn] float32 -> (ancestors [nImg, n_out],
    priors [nImg, n_out], iMax [nImg], perm [nImg, nIn], u0 [nImg])."""
    nImg, nIn = u.shape
    dev = u.device
    _req(u, torch.float32, (nImg, nIn), "u")
    ldw = 0 if w.dim() == 1 else nIn
    _req(w, torch.float64, (nIn,) if ldw == 0 else (nImg, nIn), "w")
    anc = torch.empty(nImg, n_out, dtype=torch.int32, device=dev)
    wout = torch.empty(nImg, n_out, dtype=torch.float64, device=dev)
    imax = torch.empty(nImg, dtype=torch.int32, device=dev)
    perm = torch.empty(nImg, nIn, dtype=torch.int32, device=dev)
    u0 = torch.empty(nImg, dtype=torch.float64, device=dev)
    ws = workspace(lib().thx_pf_resample_workspace(nImg, nIn), dev)
    check(lib().thx_pf_resample(nImg, nIn, n_out, _ptr(w), ldw, _ptr(u), nIn, seed, stream_id,
                                int(bool(shuffle)), _ptr(anc), _ptr(wout), _ptr(imax), _ptr(perm),
                                _ptr(u0), _ptr(ws), ws.numel(), _stream(dev)), "thx_pf_resample")
    return anc, wout, imax, perm, u0


def pf_calvari(quat, trans, k_floor=0.0, s_floor=0.0):
    """thx_pf_calvari: per-image ACG spreads (k1, k2, k3) and translation
    standard deviations (s0, s1) of particle clouds quat [nImg, mR, 4],
    trans [nImg, mT, 2] (float64, device)."""
    nImg, mR = quat.shape[:2]
    mT = trans.shape[1]
    _req(quat, torch.float64, (nImg, mR, 4), "quat")
    _req(trans, torch.float64, (nImg, mT, 2), "trans")
    k = torch.empty(nImg, 3, dtype=torch.float64, device=quat.device)
    sd = torch.empty(nImg, 2, dtype=torch.float64, device=quat.device)
    check(lib().thx_pf_calvari(nImg, mR, _ptr(quat), mT, _ptr(trans), k_floor, s_floor, _ptr(k),
                               _ptr(sd), _stream(quat.device)), "thx_pf_calvari")
    return k, sd


def pf_balance_rot(quat):
    """thx_pf_balance_rot: normalised 1/pdfACG rotation priors [nImg, mR]."""
    nImg, mR = quat.shape[:2]
    _req(quat, torch.float64, (nImg, mR, 4), "quat")
    pR = torch.empty(nImg, mR, dtype=torch.float64, device=quat.device)
    check(lib().thx_pf_balance_rot(nImg, mR, _ptr(quat), _ptr(pR), _stream(quat.device)),
          "thx_pf_balance_rot")
    return pR


def pf_defocus(op, d, pD=None, sd=None, arg=0.0, seed=1, stream_id=0):
    """thx_pf_defocus: op "init" (d <- 1 + N(0, arg)), "perturb" (d += N(0, sd) arg),
    both rebalancing pD; "vari" (sd <- std of d)."""
    nImg, mD = d.shape
    _req(d, torch.float64, (nImg, mD), "d")
    k = {"init": 0, "perturb": 1, "vari": 2}[op]
    if k != 2:
        _req(pD, torch.float64, (nImg, mD), "pD")
    if k != 0:
        _req(sd, torch.float64, (nImg,), "sd")
    check(lib().thx_pf_defocus(nImg, mD, k, float(arg), seed, stream_id, _ptr(d), _ptr(pD),
                               _ptr(sd), _stream(d.device)), "thx_pf_defocus")


def pf_peak(u, peak=None):
    """thx_pf_peak: keepHalfHeightPeak on marginals u [nImg, n] float32 (in
    place); sets the 3D peak factor first when ``peak`` is None.  Returns
    (u, peak)."""
    nImg, n = u.shape
    _req(u, torch.float32, (nImg, n), "u")
    set_factor = peak is None
    if set_factor:
        peak = torch.empty(nImg, dtype=torch.float64, device=u.device)
    check(lib().thx_pf_peak(nImg, n, _ptr(u), n, _ptr(peak), int(set_factor), _stream(u.device)),
          "thx_pf_peak")
    return u, peak
