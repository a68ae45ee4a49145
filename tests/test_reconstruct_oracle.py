"""CPU checks of the f1 restatement (oracle/reconstruct.py): the MKB kernel's
half-integer Bessel closed forms against scipy.special (an independent
implementation of the functions GSL 2.4 evaluates in MKB_RL_R2), and the
solve's identities (no grid correction: the map is IFFT(F / T) in the sphere,
kernel-corrected)."""
import numpy as np
import scipy.special as sp

from oracle import reconstruct as rc


def test_mkb_kernel_matches_scipy_bessel():
    a, alpha = 1.9, 15.0
    r2 = np.linspace(0, 1, 2001)
    got = rc.mkb_rl_r2(r2, a, alpha)
    u2 = (2 * np.pi * a) ** 2 * r2
    v = np.sqrt(np.abs(alpha ** 2 - u2))
    with np.errstate(invalid="ignore", divide="ignore"):
        ref = np.where(u2 <= alpha ** 2, sp.iv(1.5, v), sp.jv(1.5, v)) / v ** 1.5
    ref = (2 * np.pi) ** 1.5 * a ** 3 / sp.i0(alpha) * ref
    ok = v > 1e-3                       # scipy's 0 / 0 at the switch point
    assert np.allclose(got[ok], ref[ok], rtol=1e-9, atol=1e-12 * np.abs(ref).max())
    assert abs(rc.bessel_i0(alpha) - sp.i0(alpha)) < 1e-12 * sp.i0(alpha)


def test_no_grid_correction_inverts_T():
    N, pf = 16, 2
    vdim = N * pf
    rng = np.random.default_rng(3)
    x = rng.standard_normal((vdim, vdim, vdim))
    X = np.fft.rfftn(x)
    T = rng.uniform(0.5, 2.0, X.shape)
    got, it, _ = rc.reconstruct(X * T, T, N, pf, grid_corr=False)
    quad = rc._ft_quad(vdim)
    maxR = N // 2 - 2
    ref_rl = np.fft.irfftn(np.where(quad < (maxR * pf) ** 2, X, 0), s=(vdim,) * 3)
    c = np.fft.fftfreq(N, 1.0 / N).astype(int)
    box = ref_rl[np.ix_(c % vdim, c % vdim, c % vdim)]
    r = np.sqrt(rc._rl_quad(N).astype(float)) / vdim
    j0 = np.where(r == 0, 1.0, np.sin(np.pi * r) / np.where(r == 0, 1, np.pi * r))
    assert it == 0
    assert np.allclose(got, box / j0 ** 2, atol=1e-10)


def test_grid_correction_balances_C():
    N, pf = 16, 2
    vdim = N * pf
    rng = np.random.default_rng(4)
    T = rng.uniform(0.5, 2.0, (vdim, vdim, vdim // 2 + 1))
    F = np.zeros_like(T, dtype=complex)
    _, it, diffs = rc.reconstruct(F, T, N, pf, grid_corr=True)
    assert 1 <= it <= 30 and len(diffs) == it
    assert diffs[-1] < diffs[0]


def test_2d_no_grid_correction_inverts_T():
    """MODE_2D restatement: without grid correction the class image is the
    inverse FFT of F / T in the disc, IMG_EXTRACT_RL'd and kernel-corrected."""
    N, pf = 32, 2
    vdim = N * pf
    rng = np.random.default_rng(5)
    X = np.fft.rfftn(rng.standard_normal((vdim, vdim)))
    T = rng.uniform(0.5, 2.0, X.shape)
    got, it, _ = rc.reconstruct2d(X * T, T, N, pf, grid_corr=False)
    quad = rc._ft_quad2(vdim)
    maxR = N // 2 - 2
    ref_rl = np.fft.irfftn(np.where(quad < (maxR * pf) ** 2, X, 0), s=(vdim, vdim))
    c = np.fft.fftfreq(N, 1.0 / N).astype(int)
    box = ref_rl[np.ix_(c % vdim, c % vdim)]
    r = np.sqrt(rc._rl_quad2(N).astype(float)) / vdim
    j0 = np.where(r == 0, 1.0, np.sin(np.pi * r) / np.where(r == 0, 1, np.pi * r))
    assert it == 0
    assert np.allclose(got, box / j0 ** 2, atol=1e-10)


def test_2d_grid_correction_balances_C():
    N, pf = 32, 2
    vdim = N * pf
    rng = np.random.default_rng(6)
    T = rng.uniform(0.5, 2.0, (vdim, vdim // 2 + 1))
    _, it, diffs = rc.reconstruct2d(np.zeros_like(T, dtype=complex), T, N, pf, grid_corr=True)
    assert 1 <= it <= 30 and len(diffs) == it
    assert diffs[-1] < diffs[0]
