"""Seeded synthetic cryo-EM stacks of the shapes in BASELINE.json.

There is no network and no dataset: the bench and the tests build a volume of
Gaussian blobs, pad it x pf and Fourier transform it into the half-complex
projectee layout [vdim][vdim][vdim/2+1] (what Projector::setProjectee,
src/Projector.cpp:123-148, hands to the search), then CTF-modulated noisy
projections at a chosen SNR.  The global sample set follows Particle::reset
(src/Particle.cpp:87-169): ACG(identity) = uniform quaternions, translations
from a bivariate Gaussian of width transS, translation prior 1 / pdf
(balanceWeight, src/Particle.cpp:2340-2375), rotation prior 1 / nR.
"""
import math

import numpy as np
import torch

CHI2_QINV_HALF_2DOF = -2.0 * math.log(0.5)   # gsl_cdf_chisq_Qinv(0.5, 2)


def n_trans_global(trans_s=10.0, trans_search_factor=0.25):
    """nT of src/Optimiser.cpp:1732-1737."""
    return max(30, int(round(math.pi * (trans_s * CHI2_QINV_HALF_2DOF) ** 2 * trans_search_factor)))


def blob_volume(N, n_blobs=40, seed=1, device="cpu", sym_R=None):
    """Real-space N^3 float32 volume of Gaussian blobs inside radius 0.35 N;
    sym_R ([n, 3, 3], the non-identity elements of a point group, e.g.
    ops.symmetry("C4")[0]): every blob is repeated at R c for every element,
    so V(R x) = V(x) about the box centre (x, y, z = column, row, slice)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    centers = (torch.rand(n_blobs, 3, generator=g, dtype=torch.float64) * 2 - 1)
    centers = centers / centers.norm(dim=1, keepdim=True).clamp(min=1) * 0.35 * N * torch.rand(
        n_blobs, 1, generator=g, dtype=torch.float64)
    widths = 1.0 + torch.rand(n_blobs, generator=g, dtype=torch.float64) * (N / 32.0)
    amps = 0.5 + torch.rand(n_blobs, generator=g, dtype=torch.float64)
    if sym_R is not None and len(sym_R):
        Rs = torch.as_tensor(np.asarray(sym_R, np.float64))
        centers = torch.cat([centers] + [centers @ R.T for R in Rs])
        widths = widths.repeat(len(Rs) + 1)
        amps = amps.repeat(len(Rs) + 1)
    ax = torch.arange(N, dtype=torch.float32, device=device) - N // 2
    vol = torch.zeros(N, N, N, dtype=torch.float32, device=device)
    zz, yy, xx = ax.view(N, 1, 1), ax.view(1, N, 1), ax.view(1, 1, N)
    for c, wd, a in zip(centers.tolist(), widths.tolist(), amps.tolist()):
        r2 = (xx - c[0]) ** 2 + (yy - c[1]) ** 2 + (zz - c[2]) ** 2
        vol += float(a) * torch.exp(-r2 / (2 * wd * wd))
    return vol


def projectee(vol, pf=2):
    """Pad x pf (object centred on the origin, i.e. ifftshifted) and FFT into
    the half-complex [vdim][vdim][vdim/2+1] complex64 layout of Volume."""
    N = vol.shape[0]
    vdim = pf * N
    pad = torch.zeros(vdim, vdim, vdim, dtype=torch.float32, device=vol.device)
    o = (vdim - N) // 2
    pad[o:o + N, o:o + N, o:o + N] = vol
    pad = torch.fft.ifftshift(pad)
    ft = torch.fft.rfftn(pad)                      # [k][j][i], i in [0, vdim/2]
    return (ft / float(N ** 1.5)).to(torch.complex64).contiguous()


def uniform_quaternions(n, rng):
    q = rng.standard_normal((n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    return q


def clustered_quaternions(n_img, n_r, spread_deg, rng):
    """Particle clouds [n_img, n_r, 4]: every image's rotations are small
    perturbations (per-axis std ~ spread_deg) of one uniform pose."""
    base = uniform_quaternions(n_img, rng)
    d = rng.standard_normal((n_img, n_r, 4)) * np.radians(spread_deg) / 2
    d[..., 0] = 1.0
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    w0, x0, y0, z0 = [base[:, None, k] for k in range(4)]
    w1, x1, y1, z1 = [d[..., k] for k in range(4)]
    return np.ascontiguousarray(np.stack(
        [w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1, w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
         w0 * y1 - x0 * z1 + y0 * w1 + z0 * x1, w0 * z1 + x0 * y1 - y0 * x1 + z0 * w1], -1))


def global_sample_set(nR, trans_s=10.0, trans_search_factor=0.25, seed=2):
    """(quat [nR,4], trans [nT,2], pR [nR], pT [nT]) of Particle::reset for 3D, C1."""
    rng = np.random.default_rng(seed)
    quat = uniform_quaternions(nR, rng)
    nT = n_trans_global(trans_s, trans_search_factor)
    trans = rng.standard_normal((nT, 2)) * trans_s
    m = trans.mean(axis=0)
    s = trans.std(axis=0, ddof=1)
    pdf = np.exp(-0.5 * (((trans - m) / s) ** 2).sum(axis=1)) / (2 * math.pi * s[0] * s[1])
    pT = 1.0 / pdf
    pT /= pT.sum()
    pR = np.full(nR, 1.0 / nR)
    return quat, trans, pR, pT


def ctf_attrs(n, seed=5, pixel_size=1.32):
    """[n, 8] float32 {pixelSize, voltage(V), dU, dV (A), theta, Cs (A), ampC, phaseShift}."""
    rng = np.random.default_rng(seed)
    a = np.zeros((n, 8), np.float32)
    a[:, 0] = pixel_size
    a[:, 1] = 300e3
    a[:, 2] = rng.uniform(15000, 30000, n)
    a[:, 3] = a[:, 2] - rng.uniform(0, 500, n)
    a[:, 4] = rng.uniform(0, math.pi, n)
    a[:, 5] = 2.7e7
    a[:, 6] = 0.1
    a[:, 7] = 0.0
    return a


def noisy_images(signal, iSig, n_shell, snr=0.05, seed=6, white=False):
    """signal: complex [nImg, nPxl] (ctf * shifted projection).  Returns
    (dat, sigRcp) with per-shell noise power sigma^2 = <|signal|^2>_shell / snr
    (white: one sigma^2 = <|signal|^2> / snr over the pixel set, the
    micrograph-like case where the high shells are noise-dominated) and
    sigRcp = -1 / (2 sigma^2) (the _sigRcp of src/Optimiser.cpp:5242)."""
    dev = signal.device
    sh = torch.as_tensor(iSig, dtype=torch.long, device=dev)
    p = (signal.real ** 2 + signal.imag ** 2).mean(dim=0)
    num = torch.zeros(n_shell, dtype=torch.float64, device=dev).index_add_(0, sh, p.double())
    cnt = torch.zeros(n_shell, dtype=torch.float64, device=dev).index_add_(
        0, sh, torch.ones_like(p, dtype=torch.float64))
    shell_pow = (num / cnt.clamp(min=1)).clamp(min=1e-12)
    sigma2 = (shell_pow / snr).float()[sh]                     # [nPxl]
    if white:
        sigma2 = torch.full_like(sigma2, float(p.mean()) / snr)
    g = torch.Generator(device=dev).manual_seed(seed)
    noise = torch.complex(torch.randn(signal.shape, generator=g, device=dev),
                          torch.randn(signal.shape, generator=g, device=dev))
    dat = (signal + noise * torch.sqrt(sigma2 / 2)).to(torch.complex64).contiguous()
    sig = (-0.5 / sigma2).expand(signal.shape[0], -1).contiguous()
    return dat, sig
