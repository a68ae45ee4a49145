#!/usr/bin/env python3
"""CPU model of the local phase's LDS patch boxes on dumped clouds
(tools/dump_clouds.py, all 12 500 bench images): fraction of (rotation,
pixel) samples whose patch box fits the LDS box, for

  image   -- the current tile: one image's 125 rotations (Morton-ranked) per
             workgroup, one box per patch over all of them;
  groupG  -- cross-image tiles: every image's rotations sorted by the Morton
             code of their canonical quaternion (w >= 0), cut into groups of
             G, all groups of the batch sorted by their median rotation's
             code, and 128 / G consecutive groups (different images) form
             one workgroup tile with one box per patch.

An optional perturbation (--perturb DEG) widens every rotation by a random
small rotation of that scale, standing in for the phase's perturb step.
python tools/group_model.py gpurun_out/clouds.npz [cap] [perturb_deg]"""
import sys

import numpy as np

from box_model import quat_to_mat  # noqa: E402  (tools/ on sys.path when run from tools/)


def morton_abs(q):
    """Morton code of the canonical (w >= 0) quaternion's vector part."""
    s = np.where(q[..., 0] < 0, -1.0, 1.0)
    v = [np.clip((q[..., k] * s + 1) * 512, 0, 1023).astype(np.int64) for k in (1, 2, 3)]
    key = np.zeros(q.shape[:-1], np.int64)
    for bit in range(10):
        for ax in range(3):
            key |= ((v[ax] >> bit) & 1) << (3 * bit + ax)
    return key


def boxes(M, X0, X1, Y0, Y1, eps=1e-3):
    """M [nW, R, 3, 3] -> voxels of each tile's two-sided folded box (k_patch_boxes)."""
    u, v = M[..., :, 0], M[..., :, 1]
    mn = u * np.where(u >= 0, X0, X1) + v * np.where(v >= 0, Y0, Y1)
    mx = u * np.where(u >= 0, X1, X0) + v * np.where(v >= 0, Y1, Y0)
    dims, anys = [], []
    for side in (0, 1):
        if side == 0:
            sel = mx[..., 0] >= -eps
            lo, hi = mn, mx
        else:
            sel = mn[..., 0] < eps
            lo, hi = -mx, -mn
        big = 1e9
        lo_m = np.where(sel[..., None], lo, big).min(1)
        hi_m = np.where(sel[..., None], hi, -big).max(1)
        a = sel.any(1)
        lo_i = np.floor(lo_m - eps)
        lo_i[:, 0] = np.maximum(lo_i[:, 0], 0)
        hi_i = np.floor(hi_m + eps) + 1
        d = np.where(a[:, None], hi_i - lo_i + 1, 0)
        dims.append(d)
        anys.append(a)
    d = np.maximum(dims[0], dims[1])
    nx = (d[:, 0].astype(np.int64) + 3) // 4 * 4
    nx = np.where((nx // 4) % 2 == 0, nx + 4, nx)
    sp = nx * d[:, 1].astype(np.int64)
    sp += ((2 - sp % 16) + 16) % 16
    return (anys[0].astype(np.int64) + anys[1]) * sp * d[:, 2].astype(np.int64)


def perturb(Q, deg, rng):
    e = rng.standard_normal(Q.shape) * np.radians(deg) / 2
    e[..., 0] = 1.0
    e /= np.linalg.norm(e, axis=-1, keepdims=True)
    w0, x0, y0, z0 = [Q[..., k] for k in range(4)]
    w1, x1, y1, z1 = [e[..., k] for k in range(4)]
    return np.stack([w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1, w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
                     w0 * y1 - x0 * z1 + y0 * w1 + z0 * x1, w0 * z1 + x0 * y1 - y0 * x1 + z0 * w1], -1)


def tiles_image(Q):
    keys = morton_abs(Q)
    o = np.argsort(keys, axis=1, kind="stable")
    return np.take_along_axis(Q, o[..., None], 1)          # [nImg, 125, 4]


def tiles_grouped(Q, G):
    nImg, nR = Q.shape[:2]
    keys = morton_abs(Q)
    o = np.argsort(keys, axis=1, kind="stable")
    Qs = np.take_along_axis(Q, o[..., None], 1)
    ks = np.take_along_axis(keys, o, 1)
    nG = (nR + G - 1) // G
    pad = nG * G - nR
    if pad:   # short last group: repeat its last rotation (inside its own box)
        Qs = np.concatenate([Qs, np.repeat(Qs[:, -1:], pad, 1)], 1)
        ks = np.concatenate([ks, np.repeat(ks[:, -1:], pad, 1)], 1)
    grp = Qs.reshape(nImg * nG, G, 4)
    gk = ks.reshape(nImg * nG, G)[:, G // 2]
    og = np.argsort(gk, kind="stable")
    per = 128 // G
    n = (len(og) // per) * per
    return grp[og[:n]].reshape(-1, per * G, 4)


def staged_fraction(T, patches, cap, nmax=3000):
    T = T[:nmax]
    M = quat_to_mat(T)
    fit = tot = 0.0
    for (X0, X1, Y0, Y1, n) in patches:
        nv = boxes(M, X0, X1, Y0, Y1)
        w = n * T.shape[1]
        tot += w * len(nv)
        fit += w * np.sum(nv <= cap)
    return fit / tot


def main():
    f = np.load(sys.argv[1])
    cap = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    pdeg = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    iCol, iRow, order = f["iCol"], f["iRow"], f["order"]
    pf = 2
    patches = []
    for c in range(0, len(order), 16):
        p = order[c:c + 16]
        p = p[p >= 0]
        if len(p):
            patches.append((iCol[p].min() * pf, iCol[p].max() * pf, iRow[p].min() * pf,
                            iRow[p].max() * pf, len(p)))
    rng = np.random.default_rng(0)
    for key in sorted(k for k in f.files if k.startswith("quat_k")):
        Q = f[key].astype(np.float64)
        Q /= np.linalg.norm(Q, axis=-1, keepdims=True)
        if pdeg > 0:
            Q = perturb(Q, pdeg, rng)
        res = {"image": round(staged_fraction(tiles_image(Q), patches, cap), 3)}
        for G in (16, 32, 64):
            res[f"group{G}"] = round(staged_fraction(tiles_grouped(Q, G), patches, cap), 3)
        print(key, f"cap={cap} perturb={pdeg}", res, flush=True)


if __name__ == "__main__":
    main()
