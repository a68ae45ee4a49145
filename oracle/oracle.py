"""numpy front-end of the C restatement in oracle/thunder_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
``cpu_baseline`` leg of bench.py, never by the product package ``thunder_amd``.
Parity status: "parity unpinned" (see thunder_oracle.h).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_c_int, _c_float, _c_double = ctypes.c_int, ctypes.c_float, ctypes.c_double


def build():
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    L = ctypes.CDLL(_LIB_PATH)
    L.orc_pixel_set.restype = _c_int
    L.orc_pixel_set.argtypes = [_c_int, _c_int, _c_float, _c_float, _c_int] + [ctypes.c_void_p] * 6
    L.orc_ctf.restype = None
    L.orc_ctf.argtypes = [_f32p] + [_c_float] * 8 + [_c_int, _c_int, _i32p, _i32p, _c_int]
    L.orc_translate.restype = None
    L.orc_translate.argtypes = [_f32p, _c_float, _c_float, _c_int, _c_int, _i32p, _i32p, _c_int]
    L.orc_translate_src.restype = None
    L.orc_translate_src.argtypes = [_f32p, _f32p, _c_float, _c_float, _c_int, _c_int, _i32p, _i32p, _c_int]
    L.orc_rotate3d.restype = None
    L.orc_rotate3d.argtypes = [_f64p, _f64p]
    L.orc_project3d.restype = None
    L.orc_project3d.argtypes = [_f32p, _f32p, _c_int, _c_int, _f64p, _i32p, _i32p, _c_int]
    L.orc_logdatavs.restype = _c_float
    L.orc_logdatavs.argtypes = [_f32p, _f32p, _f32p, _f32p, _c_int]
    L.orc_dvp_global.restype = None
    L.orc_dvp_global.argtypes = [_f32p, _f32p, _c_int, _c_int, _f64p, _c_int, _f64p, _c_int,
                                 _f32p, _f32p, _f32p, _c_int, _i32p, _i32p, _c_int, _c_int, _c_int]
    L.orc_weights_global.restype = None
    L.orc_weights_global.argtypes = [_f32p, _c_int, _c_int, _c_int, _f64p, _f64p, _c_int, _c_int,
                                     _f32p, _f32p, _f32p, _f32p]
    L.orc_local_phase.restype = None
    L.orc_local_phase.argtypes = [_f32p, _c_int, _c_int, _f64p, _c_int, _f64p, _c_int, _c_double,
                                  _f64p, _f64p, _f32p, _f32p, _f32p, _i32p, _i32p, _c_int, _c_int,
                                  _f32p, _f32p, _f32p, _f32p, ctypes.c_void_p]
    L.orc_resample.restype = _c_int
    L.orc_resample.argtypes = [_c_int, _f64p, _f64p, _c_int, _c_double, _i32p, _f64p]
    L.orc_insert3d.restype = None
    L.orc_insert3d.argtypes = [_f32p, _f32p, _c_int, _f32p, _f32p, _f64p, _c_float, _i32p, _i32p, _c_int]
    L.orc_insert_batch.restype = None
    L.orc_insert_batch.argtypes = [_f32p, _f32p, _f64p, _i64p, _c_int, _c_int, _f32p, _f32p,
                                   _f64p, _f64p, _f64p, _f32p, _c_int, _c_int, _i32p, _i32p,
                                   _c_int, _c_int]
    L.orc_project2d.restype = None
    L.orc_project2d.argtypes = [_f32p, _f32p, _c_int, _c_int, _f64p, _i32p, _i32p, _c_int]
    L.orc_insert2d_batch.restype = None
    L.orc_insert2d_batch.argtypes = [_f32p, _f32p, _f64p, _i64p, _c_int, _c_int, _f32p, _f32p,
                                     _f64p, _f64p, _f64p, _f32p, ctypes.c_void_p, _c_int, _c_int,
                                     _i32p, _i32p, _c_int, _c_int]
    L.orc_fsc.restype = None
    L.orc_fsc.argtypes = [_f64p, _c_int, _f32p, _f32p, _c_int]
    L.orc_defocus_pre.restype = None
    L.orc_defocus_pre.argtypes = [_f32p, _i32p, _i32p, _c_int, _c_int, _f32p, _f32p,
                                  ctypes.POINTER(_c_float), ctypes.POINTER(_c_float)]
    L.orc_ctf_search.restype = None
    L.orc_ctf_search.argtypes = [_f32p, _f32p, _f32p, _f64p, _c_int, _c_float, _c_float, _c_float,
                                 _c_float, _c_int]
    L.orc_local_phase_d.restype = None
    L.orc_local_phase_d.argtypes = [_f32p, _c_int, _c_int, _f64p, _c_int, _f64p, _c_int, _c_int,
                                    _c_double, _f64p, _f64p, _f64p, _f32p, _f32p, _f32p, _i32p,
                                    _i32p, _c_int, _c_int, _f32p, _f32p, _f32p, _f32p, _f32p,
                                    ctypes.c_void_p]
    L.orc_local_phase2d_d.restype = None
    L.orc_local_phase2d_d.argtypes = L.orc_local_phase_d.argtypes
    L.orc_insert_batch_d.restype = None
    L.orc_insert_batch_d.argtypes = [_f32p, _f32p, _f64p, _i64p, _c_int, _c_int, _f32p, _f32p,
                                     _f64p, _f64p, _f64p, _f64p, _f32p, _c_int, _c_int, _i32p,
                                     _i32p, _c_int, _c_int]
    _lib = L
    return L


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _cf(a):
    """complex64 array -> contiguous float32 view (re, im interleaved)."""
    a = np.ascontiguousarray(a, dtype=np.complex64)
    return a.view(np.float32)


class PixelSet:
    def __init__(self, iCol, iRow, iSig, iPxl, pf):
        self.iCol, self.iRow, self.iSig, self.iPxl = iCol, iRow, iSig, iPxl
        self.iColPad, self.iRowPad = iCol * pf, iRow * pf
        self.n = len(iCol)


def pixel_set(N, pf, rU, rL):
    cap = (N // 2 + 1) * N
    bufs = [np.zeros(cap, np.int32) for _ in range(6)]
    n = lib().orc_pixel_set(N, pf, rU, rL, cap, *[b.ctypes.data for b in bufs])
    assert n >= 0
    iCol, iRow, iSig, iPxl = (b[:n].copy() for b in bufs[:4])
    return PixelSet(iCol, iRow, iSig, iPxl, pf)


def ctf(px, attr, N):
    """attr = (pixelSize, voltage, dU, dV, theta, Cs, ampContrast, phaseShift)."""
    out = np.zeros(px.n, np.float32)
    lib().orc_ctf(out, *[float(a) for a in attr], N, N, px.iCol, px.iRow, px.n)
    return out


def translate(px, tx, ty, N):
    out = np.zeros(2 * px.n, np.float32)
    lib().orc_translate(out, tx, ty, N, N, px.iCol, px.iRow, px.n)
    return out.view(np.complex64)


def translate_src(px, src, tx, ty, N):
    out = np.zeros(2 * px.n, np.float32)
    lib().orc_translate_src(out, _cf(src), tx, ty, N, N, px.iCol, px.iRow, px.n)
    return out.view(np.complex64)


def rotate3d(quat):
    m = np.zeros(9, np.float64)
    lib().orc_rotate3d(m, _c(quat, np.float64))
    return m  # column-major


def project3d(vol, vdim, pf, mat, px):
    out = np.zeros(2 * px.n, np.float32)
    lib().orc_project3d(out, _cf(vol).reshape(-1), vdim, pf, _c(mat, np.float64),
                        px.iCol, px.iRow, px.n)
    return out.view(np.complex64)


def logdatavs(dat, pri, ctf_, sig):
    return lib().orc_logdatavs(_cf(dat), _cf(pri), _c(ctf_, np.float32), _c(sig, np.float32), len(ctf_))


def dvp_global(vol, vdim, pf, quat, trans, dat, ctf_, sig, px, idim, threads=0):
    nR, nT, nImg = len(quat), len(trans), len(dat)
    out = np.zeros(nImg * nR * nT, np.float32)
    lib().orc_dvp_global(out, _cf(vol).reshape(-1), vdim, pf, _c(quat, np.float64).reshape(-1), nR,
                         _c(trans, np.float64).reshape(-1), nT, _cf(dat).reshape(-1),
                         _c(ctf_, np.float32).reshape(-1), _c(sig, np.float32).reshape(-1), nImg,
                         px.iCol, px.iRow, px.n, idim, threads)
    return out.reshape(nImg, nR, nT)


def weights_global(dvp, pR, pT, kIdx=0, nK=1, state=None):
    nImg, nR, nT = dvp.shape
    if state is None:
        state = (np.zeros(nImg * nK, np.float32), np.zeros(nImg * nK * nR, np.float32),
                 np.zeros(nImg * nK * nT, np.float32), np.full(nImg, np.nan, np.float32))
    wC, wR, wT, baseL = state
    lib().orc_weights_global(_c(dvp, np.float32).reshape(-1), nImg, nR, nT, _c(pR, np.float64),
                             _c(pT, np.float64), kIdx, nK, wC, wR, wT, baseL)
    return wC, wR, wT, baseL


def local_phase(vol, vdim, pf, quat, trans, pC, pR, pT, dat, ctf_, sig, px, idim):
    nR, nT = len(quat), len(trans)
    wC = np.zeros(1, np.float32)
    wR = np.zeros(nR, np.float32)
    wT = np.zeros(nT, np.float32)
    base = np.zeros(1, np.float32)
    dvp = np.zeros(nR * nT, np.float32)
    lib().orc_local_phase(_cf(vol).reshape(-1), vdim, pf, _c(quat, np.float64).reshape(-1), nR,
                          _c(trans, np.float64).reshape(-1), nT, float(pC), _c(pR, np.float64),
                          _c(pT, np.float64), _cf(dat), _c(ctf_, np.float32), _c(sig, np.float32),
                          px.iCol, px.iRow, px.n, idim, wC, wR, wT, base, dvp.ctypes.data)
    return wC[0], wR, wT, base[0], dvp.reshape(nR, nT)


def defocus_pre(px, attr, N):
    """CTF-search precalculation of one image: (freq, defocusP, K1, K2)."""
    freq = np.zeros(px.n, np.float32)
    dfo = np.zeros(px.n, np.float32)
    k1, k2 = _c_float(), _c_float()
    lib().orc_defocus_pre(_c(attr, np.float32), px.iCol, px.iRow, px.n, N, freq, dfo,
                          ctypes.byref(k1), ctypes.byref(k2))
    return freq, dfo, k1.value, k2.value


def ctf_search(dfo, freq, d, K1, K2, phase_shift, con_t):
    """ctfD[nD][nPxl] of one image for the defocus factors d."""
    d = _c(d, np.float64)
    out = np.zeros(len(d) * len(freq), np.float32)
    lib().orc_ctf_search(out, _c(dfo, np.float32), _c(freq, np.float32), d, len(d), K1, K2,
                         phase_shift, con_t, len(freq))
    return out.reshape(len(d), len(freq))


def local_phase_d(vol, vdim, pf, quat, trans, pC, pR, pT, pD, dat, ctfD, sig, px, idim):
    nR, nT, nD = len(quat), len(trans), len(pD)
    wC = np.zeros(1, np.float32)
    wR = np.zeros(nR, np.float32)
    wT = np.zeros(nT, np.float32)
    wD = np.zeros(nD, np.float32)
    base = np.zeros(1, np.float32)
    dvp = np.zeros(nR * nT * nD, np.float32)
    lib().orc_local_phase_d(_cf(vol).reshape(-1), vdim, pf, _c(quat, np.float64).reshape(-1), nR,
                            _c(trans, np.float64).reshape(-1), nT, nD, float(pC),
                            _c(pR, np.float64), _c(pT, np.float64), _c(pD, np.float64), _cf(dat),
                            _c(ctfD, np.float32).reshape(-1), _c(sig, np.float32), px.iCol,
                            px.iRow, px.n, idim, wC, wR, wT, wD, base, dvp.ctypes.data)
    return wC[0], wR, wT, wD, base[0], dvp.reshape(nR, nT, nD)


def local_phase2d_d(img, vdim, pf, rot, trans, pC, pR, pT, pD, dat, ctfD, sig, px, idim):
    """The 2D (r, t, d) phase of one image: rot [nR, 2] (cos, sin)."""
    nR, nT, nD = len(rot), len(trans), len(pD)
    wC = np.zeros(1, np.float32)
    wR = np.zeros(nR, np.float32)
    wT = np.zeros(nT, np.float32)
    wD = np.zeros(nD, np.float32)
    base = np.zeros(1, np.float32)
    dvp = np.zeros(nR * nT * nD, np.float32)
    lib().orc_local_phase2d_d(_cf(img).reshape(-1), vdim, pf, _c(rot, np.float64).reshape(-1), nR,
                              _c(trans, np.float64).reshape(-1), nT, nD, float(pC),
                              _c(pR, np.float64), _c(pT, np.float64), _c(pD, np.float64),
                              _cf(dat), _c(ctfD, np.float32).reshape(-1), _c(sig, np.float32),
                              px.iCol, px.iRow, px.n, idim, wC, wR, wT, wD, base, dvp.ctypes.data)
    return wC[0], wR, wT, wD, base[0], dvp.reshape(nR, nT, nD)


def insert_batch_d(vdim, pf, dat, attr, nD, quat, trans, offS, w, px, idim):
    """CTF-search insert: attr [nImg, 8], nD [nImg, mReco]."""
    nImg, mReco = quat.shape[0], quat.shape[1]
    size = (vdim // 2 + 1) * vdim * vdim
    F = np.zeros(2 * size, np.float32)
    T = np.zeros(size, np.float32)
    O = np.zeros(3, np.float64)
    cnt = np.zeros(1, np.int64)
    lib().orc_insert_batch_d(F, T, O, cnt, vdim, pf, _cf(dat).reshape(-1),
                             _c(attr, np.float32).reshape(-1), _c(nD, np.float64).reshape(-1),
                             _c(quat, np.float64).reshape(-1), _c(trans, np.float64).reshape(-1),
                             _c(offS, np.float64).reshape(-1), _c(w, np.float32), nImg, mReco,
                             px.iCol, px.iRow, px.n, idim)
    return F.view(np.complex64), T, O, int(cnt[0])


def resample(w, u, n_out, u0):
    anc = np.zeros(n_out, np.int32)
    wout = np.zeros(n_out, np.float64)
    imax = lib().orc_resample(len(w), _c(w, np.float64), _c(u, np.float64), n_out, float(u0), anc, wout)
    return anc, wout, imax


def insert3d(F, T, vdim, src, ctf_, mat, w, px):
    lib().orc_insert3d(F, T, vdim, _cf(src), _c(ctf_, np.float32), _c(mat, np.float64), float(w),
                       _c(px.iColPad, np.int32), _c(px.iRowPad, np.int32), px.n)


def insert_batch(vdim, pf, dat, ctf_, quat, trans, offS, w, px, idim, F=None, T=None):
    nImg, mReco = quat.shape[0], quat.shape[1]
    size = (vdim // 2 + 1) * vdim * vdim
    F = np.zeros(2 * size, np.float32) if F is None else F
    T = np.zeros(size, np.float32) if T is None else T
    O = np.zeros(3, np.float64)
    cnt = np.zeros(1, np.int64)
    lib().orc_insert_batch(F, T, O, cnt, vdim, pf, _cf(dat).reshape(-1), _c(ctf_, np.float32).reshape(-1),
                           _c(quat, np.float64).reshape(-1), _c(trans, np.float64).reshape(-1),
                           _c(offS, np.float64).reshape(-1), _c(w, np.float32), nImg, mReco,
                           px.iCol, px.iRow, px.n, idim)
    return F.view(np.complex64), T, O, int(cnt[0])


def project2d(img, vdim, pf, cs, px):
    out = np.zeros(2 * px.n, np.float32)
    lib().orc_project2d(out, _cf(img).reshape(-1), vdim, pf, _c(cs, np.float64), px.iCol, px.iRow,
                        px.n)
    return out.view(np.complex64)


def insert2d_batch(vdim, pf, dat, ctf_, rot, trans, offS, w, nc, px, idim, nK=1):
    """rot / trans: [nImg, mReco, 2]; nc: [nImg, mReco] int32 or None."""
    nImg, mReco = rot.shape[0], rot.shape[1]
    size = (vdim // 2 + 1) * vdim
    F = np.zeros(2 * size * nK, np.float32)
    T = np.zeros(size * nK, np.float32)
    O = np.zeros(2 * nK, np.float64)
    cnt = np.zeros(nK, np.int64)
    ncp = None if nc is None else np.ascontiguousarray(nc, np.int32)
    lib().orc_insert2d_batch(F, T, O, cnt, vdim, pf, _cf(dat).reshape(-1),
                             _c(ctf_, np.float32).reshape(-1), _c(rot, np.float64).reshape(-1),
                             _c(trans, np.float64).reshape(-1), _c(offS, np.float64).reshape(-1),
                             _c(w, np.float32), None if ncp is None else ncp.ctypes.data, nImg, mReco,
                             px.iCol, px.iRow, px.n, idim)
    return F.view(np.complex64), T, O, cnt


def fsc(A, B, vdim, n_shell):
    out = np.zeros(n_shell, np.float64)
    lib().orc_fsc(out, n_shell, _cf(A).reshape(-1), _cf(B).reshape(-1), vdim)
    return out
