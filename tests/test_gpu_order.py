"""thx_view_order (csrc/order.hip): the image order of the 3D phases, against
a numpy restatement of its key -- slice normal n = R(q) e_z (quat_to_mat of
common.h, rotate3D of src/Geometry/Euler.cpp:181-189), n_z >= 0, octahedral
map, 16-bit cells, their Hilbert index -- and a stable sort."""
import numpy as np
import pytest
import torch

from thunder_amd._lib import check, lib
from thunder_amd.ops import _ptr, _stream, workspace

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _keys(q, cells=False):
    A = np.zeros((len(q), 3, 3))
    A[:, 0, 1], A[:, 0, 2] = -q[:, 3], q[:, 2]
    A[:, 1, 0], A[:, 1, 2] = q[:, 3], -q[:, 1]
    A[:, 2, 0], A[:, 2, 1] = -q[:, 2], q[:, 1]
    R = np.eye(3)[None] + 2 * q[:, 0, None, None] * A + 2 * A @ A
    n = R[:, :, 2].copy()
    n[n[:, 2] < 0] *= -1
    s = np.abs(n[:, 0]) + np.abs(n[:, 1]) + n[:, 2]
    qu = np.clip((n[:, 0] / s + 1) * 32768, 0, 65535).astype(np.uint64)
    qv = np.clip((n[:, 1] / s + 1) * 32768, 0, 65535).astype(np.uint64)
    if cells:
        return qu.astype(np.int64), qv.astype(np.int64)
    return np.array([_hilbert(int(x), int(y)) for x, y in zip(qu, qv)], dtype=np.uint64)


def _hilbert(x, y, n=1 << 16):
    """xy -> index on the Hilbert curve of an n x n grid."""
    d, s = 0, n // 2
    while s > 0:
        rx, ry = int(x & s > 0), int(y & s > 0)
        d += s * s * ((3 * rx) ^ ry)
        if ry == 0:
            if rx == 1:
                x, y = n - 1 - x, n - 1 - y
            x, y = y, x
        s //= 2
    return d


def _order(quat):
    nImg, mLR = quat.shape[:2]
    ws = workspace(lib().thx_view_order_workspace(nImg), DEV)
    ord_ = torch.empty(nImg, dtype=torch.int32, device=DEV)
    check(lib().thx_view_order(nImg, mLR, _ptr(quat), _ptr(ord_), _ptr(ws), ws.numel(), _stream(DEV)),
          "thx_view_order")
    torch.cuda.synchronize()
    return ord_.cpu().numpy()


@pytest.mark.parametrize("nImg", [1, 1000, 12500])
def test_view_order_sorts_by_slice_normal(nImg):
    rng = np.random.default_rng(nImg)
    q = rng.standard_normal((nImg, 3, 4))
    q /= np.linalg.norm(q, axis=-1, keepdims=True)
    o = _order(torch.as_tensor(q, device=DEV))
    assert np.array_equal(np.sort(o), np.arange(nImg))          # a permutation
    k = _keys(q[:, 0])
    # sorted by the restated key; FP64 contraction differences may move a key
    # across a 2^-15 quantisation step, never more than a few in a batch
    assert np.sum(np.diff(k[o].astype(np.int64)) < 0) <= 2
    assert np.sum(k[o] != np.sort(k)) <= 4


def test_view_order_is_stable_and_sign_blind():
    # copies of one orientation keep batch order; q and -q, and the normal's
    # two signs (a half turn about the x axis) are one plane
    rng = np.random.default_rng(7)
    base = rng.standard_normal((50, 4))
    base /= np.linalg.norm(base, axis=-1, keepdims=True)
    flip = np.array([0.0, 1.0, 0.0, 0.0])      # 180 deg about x: n -> -n (in-plane change)
    def qmul(a, b):
        return np.array([a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                         a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                         a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                         a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]])
    q = np.concatenate([base, -base, np.stack([qmul(b, flip) for b in base]), base])
    o = _order(torch.as_tensor(q[:, None, :].copy(), device=DEV))
    k = _keys(q)
    assert np.array_equal(k[:50], k[50:100]) and np.array_equal(k[:50], k[150:])
    (u0, v0), (u1, v1) = _keys(q[:50], True), _keys(q[100:150], True)
    assert np.max(np.abs(u0 - u1)) <= 1 and np.max(np.abs(v0 - v1)) <= 1
    # equal keys in batch order (stable)
    pos = np.empty(len(q), dtype=int)
    pos[o] = np.arange(len(q))
    for i in range(50):
        assert pos[i] < pos[50 + i] < pos[150 + i]
