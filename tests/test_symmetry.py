"""Point-group symmetry on the CPU: the restatement (oracle/symmetry.py) is
pinned by known answers -- group orders, orthonormality and closure of the
elements, exact index rotations for the 90 / 180 degree groups -- and the
library's host-side group construction (thx_symmetry, no GPU needed) equals
it element by element."""
import ctypes

import numpy as np
import pytest

from oracle import symmetry as osym

ORDERS = {"C1": 1, "C2": 2, "C3": 3, "C4": 4, "C7": 7, "D2": 4, "D3": 6, "D6": 12, "T": 12,
          "O": 24, "I1": 60, "I2": 60, "I3": 60, "I4": 60}


@pytest.mark.parametrize("sym", sorted(ORDERS))
def test_oracle_group_orders_and_closure(sym):
    R, Q = osym.elements(sym)
    assert len(R) == ORDERS[sym] - 1
    allR = [np.eye(3)] + list(R)
    for r in R:
        # the reference's axes carry 7 digits: orthonormal to ~1e-5
        assert np.abs(r @ r.T - np.eye(3)).max() < 2e-5
        assert abs(np.linalg.det(r) - 1) < 2e-5
    for a in allR:                     # closure within SAME_MATRIX's 1e-2
        for b in allR:
            assert any(np.abs(a @ b - c).max() <= 1e-2 for c in allR)
    for r, q in zip(R, Q):             # quaternion(q, R) round trip
        # quaternion(dvec4&, dmat33&) takes every component's size from the
        # diagonal (sqrt(max(0, .))) and only its sign from an off-diagonal
        # difference.  Where that difference is rounding noise (the half turns)
        # the sign -- and so the rotation -- is not determined (quirk q10,
        # DESIGN.md): the round trip is checked where it is
        if not _signs_determined(r):
            continue
        assert np.abs(osym.rotate3d_quat(q) - r).max() < 5e-4
        assert abs(np.linalg.norm(q) - 1) < 1e-4


def _signs_determined(r, tol=1e-6):
    """quaternion(q, R)'s component signs come from R's antisymmetric part:
    determined where each such difference is either clearly nonzero or its
    component is 0 anyway."""
    q = osym.quat_from_matrix(r)
    diffs = (r[2, 1] - r[1, 2], r[0, 2] - r[2, 0], r[1, 0] - r[0, 1])
    return all(abs(d) > tol or abs(c) < tol for d, c in zip(diffs, q[1:]))


def test_oracle_c4_is_the_quarter_turn_about_z():
    R, _ = osym.elements("C4")
    turns = {tuple(np.rint(r).astype(int).ravel()) for r in R}
    assert turns == {(0, -1, 0, 1, 0, 0, 0, 0, 1), (-1, 0, 0, 0, -1, 0, 0, 0, 1),
                     (0, 1, 0, -1, 0, 0, 0, 0, 1)}


def _rotate_exact(V, M):
    """V(M v) by index arithmetic for an integer signed permutation M (the
    Hermitian fold where the rotated x < 0) -- SYMMETRIZE_FT's gather at
    grid points, without interpolation."""
    vdim = V.shape[0]
    i = np.arange(vdim // 2 + 1)
    j = np.fft.fftfreq(vdim, 1.0 / vdim).astype(int)
    K, J, I = np.meshgrid(j, j, i, indexing="ij")
    ox = M[0, 0] * I + M[0, 1] * J + M[0, 2] * K
    oy = M[1, 0] * I + M[1, 1] * J + M[1, 2] * K
    oz = M[2, 0] * I + M[2, 1] * J + M[2, 2] * K
    neg = ox < 0
    fx, fy, fz = np.where(neg, -ox, ox), np.where(neg, -oy, oy), np.where(neg, -oz, oz)
    val = V[fz % vdim, fy % vdim, fx]
    return np.where(neg, np.conj(val), val), ox * ox + oy * oy + oz * oz


@pytest.mark.parametrize("sym", ["C2", "C4", "D2"])
def test_oracle_symmetrize_ft_exact_on_grid_rotations(sym):
    vdim = 16
    rng = np.random.default_rng(1)
    # the transform of a real volume: Hermitian on the x = 0 plane, where the
    # (FP32-angle) rotations land on either side of the fold
    V = np.fft.rfftn(rng.standard_normal((vdim, vdim, vdim)))
    R, _ = osym.elements(sym)
    r = 6.5
    got = osym.symmetrize_ft(V, R, r)
    ref = V.astype(np.complex128).copy()
    for M in R:
        Mi = np.rint(M).astype(int)
        val, q2 = _rotate_exact(V, Mi)
        ref += np.where(q2 < r * r, val, 0)
    # the reference's rotations come from an FP32 angle: off-diagonal 8.7e-8
    assert np.abs(got - ref).max() < 1e-5 * np.abs(ref).max()


def test_oracle_counterpart_picks_the_nearest_copy():
    _, Q = osym.elements("D3")
    rng = np.random.default_rng(4)
    for _ in range(50):
        q = rng.standard_normal(4)
        q /= np.linalg.norm(q)
        a = rng.standard_normal(4)
        a /= np.linalg.norm(a)
        got = osym.counterpart(q, Q, a)
        copies = [q] + [osym.quat_mul(s * np.array([1, -1, -1, -1]), q) for s in Q]
        assert any(np.allclose(got, c) for c in copies)
        assert abs(got @ a) >= max(abs(c @ a) for c in copies) - 1e-15


@pytest.mark.parametrize("sym", ["C1", "C4", "C7", "D2", "D5", "T", "O", "I1", "I3"])
def test_library_symmetry_matches_restatement(sym):
    from thunder_amd._lib import lib
    L = lib()
    n = ctypes.c_int()
    assert L.thx_symmetry(sym.encode(), 0, None, None, ctypes.byref(n)) == 0
    Ro, Qo = osym.elements(sym)
    assert n.value == len(Ro)
    cap = max(n.value, 1)
    R = np.zeros((cap, 3, 3))
    Q = np.zeros((cap, 4))
    assert L.thx_symmetry(sym.encode(), cap, R.ctypes.data_as(ctypes.c_void_p),
                          Q.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)) == 0
    assert np.allclose(R[:n.value], Ro, rtol=0, atol=1e-12)
    for q, qo, r in zip(Q[:n.value], Qo, Ro):
        # a component near 0 is sqrt of a rounding-level difference (1e-16 ->
        # 1e-8), so the two restatements agree to 1e-7 there
        if _signs_determined(r):       # q10: undetermined signs may differ
            assert np.allclose(q, qo, rtol=0, atol=1e-7)
        else:
            assert np.allclose(np.abs(q), np.abs(qo), rtol=0, atol=1e-7)


def test_library_symmetry_rejects_unknown_groups():
    from thunder_amd._lib import lib
    n = ctypes.c_int()
    for bad in (b"X3", b"C", b"I5", b"D-2"):
        assert lib().thx_symmetry(bad, 0, None, None, ctypes.byref(n)) != 0
