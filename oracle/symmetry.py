"""numpy restatement of THUNDER's point-group symmetry, TEST INFRASTRUCTURE
ONLY (tests/ and the smoke check), never imported by thunder_amd.

  symmetry_group     symmetryGroup (src/Geometry/SymmetryFunctions.cpp:13-63)
  elements           Symmetry::init -> fillSymmetryEntry (SymmetryFunctions.cpp:
                     65-152) -> fillLR (src/Geometry/Symmetry.cpp:146-214, rotations
                     only: the reflexion / inversion branches are CLOG(FATAL)) ->
                     completePointGroup (:232-278) with novo (:216-230) and
                     SAME_MATRIX (include/Geometry/Symmetry.h:64-73, EQUAL_ACCURACY
                     1e-2, include/Macro.h:106); rotate3D(R, phi, axis) /
                     quaternion(q, R) of src/Geometry/Euler.cpp:102-123, 181-189,
                     272-281.  The L matrices are all identity for rotation-only
                     groups and are not carried.
  counterpart        symmetryCounterpart (Symmetry.cpp:309-335): of q and every
                     conj(s_i) q the one with the largest |<., anchor>|, the first
                     on ties; anchor default ANCHOR_POINT_2 = (1, 0, 0, 0).
  symmetrize_ft      SYMMETRIZE_FT (include/Geometry/Transformation.h:105-194):
                     V'(v) = V(v) + sum_i [|R_i v|^2 < r^2] V~(R_i v), V~ the
                     trilinear Fourier interpolation of Volume::getByInterpolationFT
                     (src/Image/Volume.cpp:314-338, Hermitian fold), over every
                     voxel of the half-complex grid (VOLUME_FOR_EACH_PIXEL_FT);
                     coordinates rounded to float32 (RFLOAT) as the reference's
                     getByInterpolationFT arguments, sums in float64 here.
  prepare_tf         Reconstructor::prepareTF (src/Reconstructor.cpp:1056-1091):
                     RECONSTRUCTOR_NORMALISE_T_F (1 / T[0], :2455-2479), then
                     symmetrizeT / symmetrizeF with r = maxRadius pf + 1 (:2676-2690).
  symmetrize_o       Reconstructor::symmetrizeO (:2692-2713).
"""
import math
import re

import numpy as np

PG_CN, PG_DN, PG_T, PG_O, PG_I1, PG_I2, PG_I3, PG_I4 = 202, 206, 209, 212, 216, 217, 218, 219
EQUAL_ACCURACY = 1e-2


def symmetry_group(sym):
    if re.fullmatch(r"C[0-9]+", sym):
        return PG_CN, int(sym[1:])
    if re.fullmatch(r"D[0-9]+", sym):
        return PG_DN, int(sym[1:])
    table = {"T": PG_T, "O": PG_O, "I1": PG_I1, "I2": PG_I2, "I3": PG_I3, "I4": PG_I4}
    if sym in table:
        return table[sym], -1
    raise ValueError("INVALID SYMMTRY INDEX")


def fill_entries(group, order):
    """(fold, axis) rotation operations, SymmetryFunctions.cpp:65-152."""
    if group == PG_CN:
        return [(order, (0.0, 0.0, 1.0))]
    if group == PG_DN:
        return fill_entries(PG_CN, order) + [(2, (1.0, 0.0, 0.0))]
    if group == PG_T:
        return [(3, (0.0, 0.0, 1.0)), (2, (0.0, 0.816496, 0.577350))]
    if group == PG_O:
        return [(3, (0.5773502, 0.5773502, 0.5773502)), (4, (0.0, 0.0, 1.0))]
    if group == PG_I1:
        return [(2, (1.0, 0.0, 0.0)), (5, (0.8506508, 0.0, -0.5257311)),
                (3, (0.9341724, 0.3568221, 0.0))]
    if group == PG_I2:
        return fill_entries(PG_CN, 2) + [(5, (0.5257311, 0.0, 0.8506508)),
                                         (3, (0.0, 0.3568221, 0.9341724))]
    if group == PG_I3:
        return ([(2, (-0.5257311, 0.0, 0.8506508))] + fill_entries(PG_CN, 5) +
                [(3, (-0.4911235, 0.3568221, 0.7946545))])
    if group == PG_I4:
        return [(2, (0.5257311, 0.0, 0.8506508)), (5, (0.8944272, 0.0, 0.4472136)),
                (3, (0.4911235, 0.3568221, 0.7946545))]
    raise ValueError("UNKNOWN SYMMETRY POINT GROUP")


def rotate3d_quat(q):
    """rotate3D(dmat33&, const dvec4&), Euler.cpp:181-189 (row-major 3x3)."""
    A = np.array([[0.0, -q[3], q[2]], [q[3], 0.0, -q[1]], [-q[2], q[1], 0.0]])
    return np.eye(3) + 2 * q[0] * A + 2 * (A @ A)


def rotate3d_axis(phi, axis):
    """rotate3D(dst, phi, axis) = rotate3D(quaternion(phi, axis)), Euler.cpp:102-110, 272-281."""
    s = math.sin(phi / 2)
    return rotate3d_quat(np.array([math.cos(phi / 2), s * axis[0], s * axis[1], s * axis[2]]))


def quat_from_matrix(R):
    """quaternion(dvec4&, const dmat33&), Euler.cpp:112-123."""
    q = np.array([0.5 * math.sqrt(max(0.0, 1 + R[0, 0] + R[1, 1] + R[2, 2])),
                  0.5 * math.sqrt(max(0.0, 1 + R[0, 0] - R[1, 1] - R[2, 2])),
                  0.5 * math.sqrt(max(0.0, 1 - R[0, 0] + R[1, 1] - R[2, 2])),
                  0.5 * math.sqrt(max(0.0, 1 - R[0, 0] - R[1, 1] + R[2, 2]))])
    q[1] = math.copysign(q[1], R[2, 1] - R[1, 2])
    q[2] = math.copysign(q[2], R[0, 2] - R[2, 0])
    q[3] = math.copysign(q[3], R[1, 0] - R[0, 1])
    return q


def _same(A, B):
    return bool(np.all(np.abs(A - B) <= EQUAL_ACCURACY))


def elements(sym):
    """(R [n, 3, 3] row-major, quat [n, 4]) of the non-identity symmetry
    elements in Symmetry's order (n = group order - 1)."""
    group, order = symmetry_group(sym)
    Rs, Qs = [], []

    def novo(R):
        if _same(R, np.eye(3)):
            return False
        return not any(_same(R, X) for X in Rs)

    for fold, axis in fill_entries(group, order):
        angle = np.float32(2 * math.pi / fold)      # RFLOAT (FP32 build)
        for j in range(1, fold):
            R = rotate3d_axis(float(angle * np.float32(j)), axis)
            if novo(R):
                Rs.append(R)
                Qs.append(quat_from_matrix(R))
    # completePointGroup: visit (i, j) cells of a growing table in row-major order
    done = np.zeros((len(Rs), len(Rs)), bool)
    while True:
        hit = np.argwhere(~done)
        if len(hit) == 0:
            break
        i, j = hit[0]
        done[i, j] = True
        R = Rs[i] @ Rs[j]
        if novo(R):
            Rs.append(R)
            Qs.append(quat_from_matrix(R))
            grown = np.zeros((len(Rs), len(Rs)), bool)
            grown[:done.shape[0], :done.shape[1]] = done
            done = grown
    if not Rs:
        return np.zeros((0, 3, 3)), np.zeros((0, 4))
    return np.array(Rs), np.array(Qs)


def quat_mul(a, b):
    """quaternion_mul, Euler.cpp:13-26."""
    return np.array([a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                     a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                     a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                     a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]])


def counterpart(q, quats, anchor=(1.0, 0.0, 0.0, 0.0)):
    anchor = np.asarray(anchor, np.float64)
    best, s = np.asarray(q, np.float64), abs(float(np.dot(q, anchor)))
    for sq in quats:
        p = quat_mul(sq * np.array([1.0, -1.0, -1.0, -1.0]), q)
        t = abs(float(np.dot(p, anchor)))
        if t > s:
            s, best = t, p
    return best


def symmetrise(cloud, quats, anchor=(1.0, 0.0, 0.0, 0.0)):
    """Particle::symmetrise (src/Particle.cpp:2445-2471) of one cloud [n, 4]."""
    return np.array([counterpart(q, quats, anchor) for q in cloud])


def _interp_ft(V, x, y, z):
    """getByInterpolationFT, LINEAR_INTERP, of a half-complex volume V[k][j][i]
    at float32 coordinates (arrays); Hermitian fold for x < 0."""
    vdim = V.shape[0]
    x, y, z = (np.asarray(a, np.float32).astype(np.float64) for a in (x, y, z))
    conj = ~(x >= 0)
    x, y, z = np.where(conj, -x, x), np.where(conj, -y, y), np.where(conj, -z, z)
    x0, y0, z0 = np.floor(x), np.floor(y), np.floor(z)
    dx, dy, dz = x - x0, y - y0, z - z0
    x0, y0, z0 = x0.astype(np.int64), y0.astype(np.int64), z0.astype(np.int64)
    out = np.zeros(x.shape, V.dtype)
    for kz in (0, 1):
        for jy in (0, 1):
            for ix in (0, 1):
                w = ((dx if ix else 1 - dx) * (dy if jy else 1 - dy) * (dz if kz else 1 - dz))
                out = out + w * V[(z0 + kz) % vdim, (y0 + jy) % vdim, x0 + ix]
    return np.where(conj, np.conj(out), out) if np.iscomplexobj(V) else out


def symmetrize_ft(V, Rs, r):
    """SYMMETRIZE_FT of a half-complex volume V [vdim][vdim][vdim/2+1]."""
    vdim = V.shape[0]
    i = np.arange(vdim // 2 + 1, dtype=np.float64)
    j = np.fft.fftfreq(vdim, 1.0 / vdim)
    K, J, I = np.meshgrid(j, j, i, indexing="ij")
    out = np.array(V, dtype=np.complex128 if np.iscomplexobj(V) else np.float64)
    src = out.copy()
    for R in Rs:
        ox = R[0, 0] * I + R[0, 1] * J + R[0, 2] * K
        oy = R[1, 0] * I + R[1, 1] * J + R[1, 2] * K
        oz = R[2, 0] * I + R[2, 1] * J + R[2, 2] * K
        inside = ox * ox + oy * oy + oz * oz < r * r
        val = _interp_ft(src, np.where(inside, ox, 0), np.where(inside, oy, 0), np.where(inside, oz, 0))
        out += np.where(inside, val, 0)
    return out


def prepare_tf(F, T, Rs, max_radius, pf):
    sf = 1.0 / float(T.flat[0])
    T = np.asarray(T, np.float64) * sf
    F = np.asarray(F, np.complex128) * sf
    r = max_radius * pf + 1
    return symmetrize_ft(F, Rs, r), symmetrize_ft(T, Rs, r)


def symmetrize_o(O, counter, Rs):
    o = np.asarray(O, np.float64)
    res = o.copy()
    for R in Rs:
        res = res + R @ o
    return res, counter * (1 + len(Rs))
