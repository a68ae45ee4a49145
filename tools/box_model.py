#!/usr/bin/env python3
"""CPU model of the local phase's LDS patch boxes on dumped clouds
(tools/dump_clouds.py): fraction of (rotation, pixel) samples whose patch box
fits the LDS capacity when the 128-rotation tile is split into Morton-ordered
groups of G rotations, each group with its own box of cap / (128 / G) voxels
(groups staged side by side) or the full cap (groups staged one after
another).  python tools/box_model.py gpurun_out/clouds.npz"""
import sys

import numpy as np


def quat_to_mat(q):
    q0, q1, q2, q3 = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    A = np.zeros(q.shape[:-1] + (3, 3))
    A[..., 0, 1], A[..., 0, 2] = -q3, q2
    A[..., 1, 0], A[..., 1, 2] = q3, -q1
    A[..., 2, 0], A[..., 2, 1] = -q2, q1
    I = np.eye(3)
    return I + 2 * q0[..., None, None] * A + 2 * A @ A


def morton_rank(q):
    a = q[0] * np.array([1, -1, -1, -1])
    b = q
    w = a[0] * b[:, 0] - a[1] * b[:, 1] - a[2] * b[:, 2] - a[3] * b[:, 3]
    x = a[0] * b[:, 1] + a[1] * b[:, 0] + a[2] * b[:, 3] - a[3] * b[:, 2]
    y = a[0] * b[:, 2] - a[1] * b[:, 3] + a[2] * b[:, 0] + a[3] * b[:, 1]
    z = a[0] * b[:, 3] + a[1] * b[:, 2] - a[2] * b[:, 1] + a[3] * b[:, 0]
    s = np.where(w < 0, -1, 1)
    v = [np.clip(((c * s) + 1) * 512, 0, 1023).astype(np.int64) for c in (x, y, z)]
    key = np.zeros(len(q), np.int64)
    for bit in range(10):
        for ax in range(3):
            key |= ((v[ax] >> bit) & 1) << (3 * bit + ax)
    return np.argsort(key, kind="stable")


def box_voxels(M, X0, X1, Y0, Y1):
    """M [g, 3, 3] rotation matrices (columns = images of x, y axes); the
    two-sided folded box of the rotated patch rectangle (k_patch_boxes)."""
    u, v = M[:, :, 0], M[:, :, 1]
    mn = u * np.where(u >= 0, X0, X1) + v * np.where(v >= 0, Y0, Y1)
    mx = u * np.where(u >= 0, X1, X0) + v * np.where(v >= 0, Y1, Y0)
    eps = 1e-3
    dims = []
    for side in (0, 1):
        if side == 0:
            sel = mx[:, 0] >= -eps
            lo, hi = mn[sel], mx[sel]
        else:
            sel = mn[:, 0] < eps
            lo, hi = -mx[sel], -mn[sel]
        if not sel.any():
            continue
        lo_i = np.floor(lo.min(0) - eps)
        lo_i[0] = max(lo_i[0], 0)
        hi_i = np.floor(hi.max(0) + eps) + 1
        dims.append(hi_i - lo_i + 1)
    if not dims:
        return 0
    d = np.max(dims, axis=0)
    nx = (int(d[0]) + 3) // 4 * 4
    return len(dims) * nx * int(d[1]) * int(d[2])


def main():
    f = np.load(sys.argv[1])
    iCol, iRow, order = f["iCol"], f["iRow"], f["order"]
    pf, CAP = 2, int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    nimg = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    for key in sorted(k for k in f.files if k.startswith("quat_k")):
        Q = f[key]
        for KC in (16, 32, 64):
            patches = []
            for c in range(0, len(order), KC):
                p = order[c:c + KC]
                p = p[p >= 0]
                if len(p):
                    patches.append((iCol[p].min() * pf, iCol[p].max() * pf, iRow[p].min() * pf,
                                    iRow[p].max() * pf, len(p)))
            res = {}
            for G in (128, 64, 32, 16):
                fit, tot, vox = 0, 0, 0
                for q in Q[:nimg]:
                    q = q[morton_rank(q)]
                    M = quat_to_mat(q)
                    for g0 in range(0, len(q), G):
                        Mg = M[g0:g0 + G]
                        for (X0, X1, Y0, Y1, n) in patches:
                            nv = box_voxels(Mg, X0, X1, Y0, Y1)
                            w = n * len(Mg)
                            tot += w
                            if nv <= CAP:
                                fit += w
                                vox += nv
                res[G] = (round(fit / tot, 3), round(vox / max(fit, 1), 2))
            print(key, f"KC={KC} G -> (staged frac, staged voxels per staged sample):", res, flush=True)


if __name__ == "__main__":
    main()
