"""numpy restatement of the deterministic particle-filter statistics (a10).

TEST INFRASTRUCTURE ONLY (tests/ import it; the product path never does).
Parity unpinned: the reference ships no fixtures for these functions; each
function restates the reference source it cites, and tests/test_oracle.py
pins the closed-form cases (an exact ACG sample's scatter, rank-1 clouds).
"""
import numpy as np

PEAK_FACTOR_MAX, PEAK_FACTOR_MIN, PEAK_FACTOR_BASE = 0.5, 1e-3, 2   # include/Particle.h:52-57
PERTURB_K_MAX = 1.0                                                  # include/Particle.h:64


def qmul(a, b):
    """quaternion_mul (src/Geometry/Euler.cpp), Hamilton product, rows."""
    a, b = np.atleast_2d(a), np.atleast_2d(b)
    w = a[:, 0] * b[:, 0] - a[:, 1] * b[:, 1] - a[:, 2] * b[:, 2] - a[:, 3] * b[:, 3]
    x = a[:, 0] * b[:, 1] + a[:, 1] * b[:, 0] + a[:, 2] * b[:, 3] - a[:, 3] * b[:, 2]
    y = a[:, 0] * b[:, 2] - a[:, 1] * b[:, 3] + a[:, 2] * b[:, 0] + a[:, 3] * b[:, 1]
    z = a[:, 0] * b[:, 3] + a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1] + a[:, 3] * b[:, 0]
    return np.stack([w, x, y, z], axis=1)


def conj(q):
    return q * np.array([1.0, -1.0, -1.0, -1.0])


def infer_acg(Q, max_it=None):
    """inferACG(dmat44&, const dmat4&), src/Geometry/DirectionalStat.cpp:93-145:
    Tyler's fixed point B = 4/nf sum q q^T / (q^T A^-1 q), from B = I, while
    sum|A - B| > 1e-3; returns the last A.  A NaN criterion (a singular A on a
    degenerate cloud) ends the loop like the reference's `while`.  max_it caps
    the iterations as the driver's perturbation mean does (acgIters)."""
    B = np.eye(4)
    it = 0
    while max_it is None or it < max_it:
        it += 1
        A = B
        with np.errstate(all="ignore"):
            Ai = np.linalg.inv(A) if np.all(np.isfinite(A)) and abs(np.linalg.det(A)) > 0 else \
                np.full((4, 4), np.nan)
            u = np.einsum("ij,jk,ik->i", Q, Ai, Q)
            B = np.einsum("ij,ik->jk", Q / u[:, None], Q)
            nf = np.sum(1.0 / u)
            B = B * (4.0 / nf)
        crit = np.abs(A - B).sum()
        if not crit > 1e-3:
            return A
    return A


def principal_axis(A):
    """Eigenvector of the largest eigenvalue (inferACG(dvec4&, ...),
    DirectionalStat.cpp:224-251), unit norm; sign free."""
    w, V = np.linalg.eigh(A)
    return V[:, np.argmax(w)]


def cal_vari_rot(Q):
    """Particle::calVari(PAR_R), 3D, PARTICLE_ROT_MEAN_USING_STAT_CAL_VARI
    (src/Particle.cpp:1011-1098): de-mean by the ACG principal axis, then
    k_j = A(j, j) / A(0, 0) of inferACG on the de-meaned cloud (:184-222)."""
    mean = principal_axis(infer_acg(Q))
    A = infer_acg(qmul(conj(mean)[None, :], Q))
    return A[1, 1] / A[0, 0], A[2, 2] / A[0, 0], A[3, 3] / A[0, 0]


def cal_vari_trans(T):
    """Particle::calVari(PAR_T) (src/Particle.cpp:1101-1121): gsl_stats_sd."""
    return float(np.std(T[:, 0], ddof=1)), float(np.std(T[:, 1], ddof=1))


def cal_vari_defocus(d):
    """Particle::calVari(PAR_D) (src/Particle.cpp:1120-1141, ZERO_MEAN off):
    gsl_stats_sd, 0 for a single sample."""
    d = np.asarray(d, np.float64)
    return 0.0 if d.size == 1 else float(np.std(d, ddof=1))


def balance_defocus(d):
    """Particle::balanceWeight(PAR_D) (src/Particle.cpp:2374-2409): w_i =
    1 / N(d_i - m; 0, s) with the sample mean m and gsl_stats_sd_m s, 1 when
    s == 0; returned normalised (normW)."""
    d = np.asarray(d, np.float64)
    m = d.mean()
    s = 0.0 if d.size == 1 else np.sqrt(np.sum((d - m) ** 2) / (d.size - 1))
    if s == 0:
        w = np.ones_like(d)
    else:
        w = 1.0 / (np.exp(-0.5 * ((d - m) / s) ** 2) / (s * np.sqrt(2 * np.pi)))
    return w / w.sum()


def pdf_acg(x, A):
    """pdfACG (DirectionalStat.cpp:19-24): det(A)^-1/2 (x^T A^-1 x)^-2."""
    Ai = np.linalg.inv(A)
    return np.linalg.det(A) ** -0.5 * np.einsum("ij,jk,ik->i", x, Ai, x) ** -2


def balance_rot(Q):
    """Particle::balanceWeight(PAR_R), 3D (src/Particle.cpp:2330-2340):
    w_i = 1 / pdfACG(q_i, inferACG(Q)); returned normalised to sum 1."""
    w = 1.0 / pdf_acg(Q, infer_acg(Q))
    return w / w.sum()


def peak_factor_rot(u):
    """Particle::setPeakFactor(PAR_R), 3D (src/Particle.cpp:1920-1925)."""
    s = np.sort(np.asarray(u, np.float64))[::-1]
    return max(PEAK_FACTOR_MIN, min(PEAK_FACTOR_MAX, s[len(s) // PEAK_FACTOR_BASE ** 3] / s[0]))


def keep_half_height(u, peak):
    """Particle::keepHalfHeightPeak (src/Particle.cpp:1964-1984)."""
    u = np.asarray(u, np.float64)
    hh = u.max() * peak
    return np.where(u < hh, 0.0, u - hh)


# ---------------------------------------------------------------- MODE_2D
# 2D rotations are Particle::_r rows (cos, sin, 0, 0) (sampleVMS(dmat4&),
# src/Geometry/DirectionalStat.cpp:320-332).

def vms_kappa(k):
    """The concentration of sampleVMS / pdfVMS from the dispersion k
    (DirectionalStat.cpp:256, 269)."""
    return (1 - k) * (1 + 2 * k - k * k) / k / (2 - k)


def infer_vms(R):
    """inferVMS(dvec2& mu, double& k, src) (DirectionalStat.cpp:334-357): the
    normalised resultant mu and k = 1 - |resultant| / n."""
    R = np.asarray(R, np.float64)
    mu = np.array([R[:, 0].sum(), R[:, 1].sum()])
    n = np.hypot(mu[0], mu[1])
    return mu / n, 1.0 - n / len(R)


def cal_vari_rot2d(R):
    """Particle::calVari(PAR_R), MODE_2D (src/Particle.cpp:1013-1016): k1."""
    return infer_vms(R)[1]


def pdf_vms(x, mu, k):
    """pdfVMS (DirectionalStat.cpp:252-262), rows x."""
    from math import factorial
    kappa = vms_kappa(k)
    x = np.asarray(x, np.float64)[:, :2]
    if kappa < 5:
        i0 = sum((kappa / 2) ** (2 * m) / factorial(m) ** 2 for m in range(40))   # gsl_sf_bessel_I0
        return np.exp(kappa * (x @ mu)) / (2 * np.pi * i0)
    sd = np.sqrt(1.0 / kappa)
    d = np.hypot(x[:, 0] - mu[0], x[:, 1] - mu[1])
    return np.exp(-d * d / (2 * sd * sd)) / (np.sqrt(2 * np.pi) * sd)


def balance_rot2d(R):
    """Particle::balanceWeight(PAR_R), MODE_2D (src/Particle.cpp:2317-2329):
    w_i = 1 / pdfVMS(r_i; inferVMS(r)); returned normalised to sum 1."""
    mu, k = infer_vms(R)
    w = 1.0 / pdf_vms(R, mu, k)
    return w / w.sum()


def peak_factor_rot2d(u):
    """Particle::setPeakFactor(PAR_R), MODE_2D (src/Particle.cpp:1920-1921):
    the (n / PEAK_FACTOR_BASE)-th largest over the largest."""
    s = np.sort(np.asarray(u, np.float64))[::-1]
    return max(PEAK_FACTOR_MIN, min(PEAK_FACTOR_MAX, s[len(s) // PEAK_FACTOR_BASE] / s[0]))


def sample_vms(rng, kappa, n):
    """sampleVMS(dmat2&, mu = (1, 0), k, n) (DirectionalStat.cpp:264-318) with
    numpy's generator: uniform directions below kappa 0.1, else Best & Fisher's
    rejection sampler for the cosine and a fair sign for the sine.  Returns
    rows (cos, sin)."""
    out = np.empty((n, 2))
    if kappa < 0.1:
        th = rng.uniform(0, 2 * np.pi, n)
        out[:, 0], out[:, 1] = np.cos(th), np.sin(th)
        return out
    a = 1 + np.sqrt(1 + 4 * kappa * kappa)
    b = (a - np.sqrt(2 * a)) / (2 * kappa)
    r = (1 + b * b) / (2 * b)
    for i in range(n):
        while True:
            z = np.cos(np.pi * rng.uniform())
            f = (1 + r * z) / (r + z)
            c = kappa * (r - f)
            u2 = rng.uniform()
            if c * (2 - c) > u2 or np.log(c / u2) + 1 - c >= 0:
                break
        d = np.sqrt((1 - f) * (f + 1))
        out[i] = (f, -d) if rng.uniform() > 0.5 else (f, d)
    return out
