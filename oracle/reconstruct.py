"""numpy restatement of the reconstruction solve (row f1), TEST INFRASTRUCTURE
ONLY (tests/ and bench.py's CPU leg), never imported by thunder_amd.

Reconstructor::reconstruct (src/Reconstructor.cpp:1129-1831) for 3D with the
trilinear kernel and the reference's Config.h switches
(RECONSTRUCTOR_WIENER_FILTER_FSC, RECONSTRUCTOR_CHECK_C_MAX,
RECONSTRUCTOR_CORRECT_CONVOLUTION_KERNEL + RECONSTRUCTOR_TRILINEAR_KERNEL,
FUNCTIONS_MKB_ORDER_0), in float64 with numpy's FFT (FFTW conventions of
src/FFT.cpp: forward unnormalised, backward scaled by 1/size):
  MAP Wiener factor :1150-1279, W / T init :1288-1331, grid-correction
  balancing :1356-1552 (convoluteC :2595-2675, checkC :2522-2593, constants
  include/Reconstructor.h:61-75), no-grid-correction W :1553-1587, F W ->
  real space -> VOL_EXTRACT_RL -> / TIK_RL :1669-1818.
reconstruct2d: the MODE_2D branches of the same function (rings instead of
shells, IMG_EXTRACT_RL), one class image.
The MKB real-space kernel is tabulated like TabFunction (src/TabFunction.cpp:
TabFunction::init / operator(): 1e5 + 1 samples on [0, 1], nearest entry) with
closed forms of the half-integer Bessel functions (MKB_RL_R2,
src/Functions/Functions.cpp; GSL 2.4's gsl_sf_bessel_Inu / Jnu / I0 at order
1.5 and 0)."""
import math

import numpy as np

TAB_N = 100000


def bessel_i0(x):
    s, t, k = 1.0, 1.0, 1
    while True:
        t *= (x * x / 4.0) / (k * k)
        s += t
        k += 1
        if t < 1e-17 * s or k > 300:
            return s


def _nu15_over(v, modified):
    """I_{3/2}(v) / v^1.5 or J_{3/2}(v) / v^1.5 (vectorised)."""
    v = np.asarray(v, np.float64)
    out = np.empty_like(v)
    small = v < 0.5
    vs = v[small]
    g25 = math.gamma(2.5)
    term = np.full_like(vs, 1.0 / (2.0 ** 1.5 * g25))
    acc = term.copy()
    for k in range(1, 30):
        term = term * ((1.0 if modified else -1.0) * (vs * vs / 4.0) / (k * (k + 1.5)))
        acc += term
    out[small] = acc
    vb = v[~small]
    c = np.sqrt(2.0 / (np.pi * vb)) / vb ** 1.5
    out[~small] = c * ((np.cosh(vb) - np.sinh(vb) / vb) if modified else (np.sin(vb) / vb - np.cos(vb)))
    return out


def mkb_rl_r2(r2, a, alpha):
    r2 = np.asarray(r2, np.float64)
    u2 = (2 * np.pi * a) ** 2 * r2
    inside = u2 <= alpha * alpha
    v = np.sqrt(np.abs(alpha * alpha - u2))
    out = np.where(inside, _nu15_over(v, True), _nu15_over(v, False))
    return (2 * np.pi) ** 1.5 * a ** 3 / bessel_i0(alpha) * out


def _ft_quad(vdim):
    i = np.arange(vdim // 2 + 1)
    j = np.fft.fftfreq(vdim, 1.0 / vdim).astype(np.int64)
    return (j[:, None, None] ** 2 + j[None, :, None] ** 2 + i[None, None, :] ** 2)   # [k][j][i]


def _rl_quad(n):
    c = np.fft.fftfreq(n, 1.0 / n).astype(np.int64)
    return c[:, None, None] ** 2 + c[None, :, None] ** 2 + c[None, None, :] ** 2


def reconstruct(F, T, N, pf=2, a=1.9, alpha=15.0, grid_corr=True, max_radius=0, fsc=None,
                join_half=False):
    """F: [vdim, vdim, vdim/2+1] complex, T: same shape real.  Returns
    (map [N, N, N] real space, origin at index 0; iterations; diffs)."""
    vdim = pf * N
    F = np.asarray(F, np.complex128)
    T = np.array(T, np.float64)
    maxR = max_radius if max_radius > 0 else N // 2 - int(math.ceil(a))
    quad = _ft_quad(vdim)
    inside = quad < (maxR * pf) ** 2
    if fsc is not None:
        lo, hi = (5 * pf) ** 2, (maxR * pf) ** 2
        m = (quad >= lo) & (quad < hi)
        u = np.rint(np.sqrt(quad[m].astype(np.float64))).astype(np.int64)
        idx = u // pf
        f = np.where(idx >= len(fsc), 0.0, np.asarray(fsc)[np.minimum(idx, len(fsc) - 1)])
        f = np.clip(f, 1e-3, 1 - 1e-3)
        if join_half:
            f = np.sqrt(2 * f / (1 + f))
        T[m] = T[m] / f
    W = inside.astype(np.float64)
    T = np.maximum(T, 1e-25)
    diffs = []
    m = 0
    if grid_corr:
        tab = mkb_rl_r2(np.arange(TAB_N + 1) * 1e-5, a, alpha).astype(np.float32).astype(np.float64)
        nf = float(mkb_rl_r2(np.array([0.0]), a, alpha)[0])
        kern = tab[np.minimum(np.rint((_rl_quad(vdim) / float(vdim * vdim)) / 1e-5).astype(np.int64),
                              TAB_N)] / nf
        diff_prev = diff = np.finfo(np.float32).max
        n_no = 0
        for m in range(30):
            C = T * W
            c = np.fft.irfftn(C, s=(vdim, vdim, vdim)) * kern
            C = np.fft.rfftn(c)
            a_ = np.abs(C)
            W = np.where(inside, W / np.maximum(a_, 1e-6), W)
            diff_prev, diff = diff, float(np.max(np.abs(a_[inside] - 1)))
            diffs.append(diff)
            n_no = n_no + 1 if diff > diff_prev * 0.95 else 0
            if diff < 1e-2 or (m >= 10 and n_no == 2):
                m += 1
                break
        else:
            m = 30
    else:
        W = np.where(inside, 1.0 / np.maximum(np.abs(T), 1e-6), W)
    pad = np.where(inside, F * W, 0)
    rl = np.fft.irfftn(pad, s=(vdim, vdim, vdim))
    c = np.fft.fftfreq(N, 1.0 / N).astype(np.int64)
    box = rl[np.ix_(c % vdim, c % vdim, c % vdim)]
    r = np.sqrt(_rl_quad(N).astype(np.float64)) / vdim
    x = np.pi * r
    j0 = np.where(x == 0, 1.0, np.sin(x) / np.where(x == 0, 1.0, x))
    return box / (j0 * j0), m, diffs


def _ft_quad2(vdim):
    i = np.arange(vdim // 2 + 1)
    j = np.fft.fftfreq(vdim, 1.0 / vdim).astype(np.int64)
    return j[:, None] ** 2 + i[None, :] ** 2                  # [j][i]


def _rl_quad2(n):
    c = np.fft.fftfreq(n, 1.0 / n).astype(np.int64)
    return c[:, None] ** 2 + c[None, :] ** 2


def reconstruct2d(F, T, N, pf=2, a=1.9, alpha=15.0, grid_corr=True, max_radius=0, fsc=None,
                  join_half=False):
    """F: [vdim, vdim/2+1] complex, T: same shape real (one class).  Returns
    (image [N, N] real space, origin at index 0; iterations; diffs)."""
    vdim = pf * N
    F = np.asarray(F, np.complex128)
    T = np.array(T, np.float64)
    maxR = max_radius if max_radius > 0 else N // 2 - int(math.ceil(a))
    quad = _ft_quad2(vdim)
    inside = quad < (maxR * pf) ** 2
    if fsc is not None:
        lo, hi = (5 * pf) ** 2, (maxR * pf) ** 2
        m = (quad >= lo) & (quad < hi)
        u = np.rint(np.sqrt(quad[m].astype(np.float64))).astype(np.int64)
        idx = u // pf
        f = np.where(idx >= len(fsc), 0.0, np.asarray(fsc)[np.minimum(idx, len(fsc) - 1)])
        f = np.clip(f, 1e-3, 1 - 1e-3)
        if join_half:
            f = np.sqrt(2 * f / (1 + f))
        T[m] = T[m] / f
    W = inside.astype(np.float64)
    T = np.maximum(T, 1e-25)
    diffs = []
    m = 0
    if grid_corr:
        tab = mkb_rl_r2(np.arange(TAB_N + 1) * 1e-5, a, alpha).astype(np.float32).astype(np.float64)
        nf = float(mkb_rl_r2(np.array([0.0]), a, alpha)[0])
        kern = tab[np.minimum(np.rint((_rl_quad2(vdim) / float(vdim * vdim)) / 1e-5).astype(np.int64),
                              TAB_N)] / nf
        diff_prev = diff = np.finfo(np.float32).max
        n_no = 0
        for m in range(30):
            C = T * W
            c = np.fft.irfftn(C, s=(vdim, vdim)) * kern
            C = np.fft.rfftn(c)
            a_ = np.abs(C)
            W = np.where(inside, W / np.maximum(a_, 1e-6), W)
            diff_prev, diff = diff, float(np.max(np.abs(a_[inside] - 1)))
            diffs.append(diff)
            n_no = n_no + 1 if diff > diff_prev * 0.95 else 0
            if diff < 1e-2 or (m >= 10 and n_no == 2):
                m += 1
                break
        else:
            m = 30
    else:
        W = np.where(inside, 1.0 / np.maximum(np.abs(T), 1e-6), W)
    pad = np.where(inside, F * W, 0)
    rl = np.fft.irfftn(pad, s=(vdim, vdim))
    c = np.fft.fftfreq(N, 1.0 / N).astype(np.int64)
    box = rl[np.ix_(c % vdim, c % vdim)]
    r = np.sqrt(_rl_quad2(N).astype(np.float64)) / vdim
    x = np.pi * r
    j0 = np.where(x == 0, 1.0, np.sin(x) / np.where(x == 0, 1.0, x))
    return box / (j0 * j0), m, diffs
