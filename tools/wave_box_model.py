#!/usr/bin/env python3
"""Patch-box sizes of the local phase on the clouds the phase evaluates
(tools/dump_clouds.py -> clouds_eval.npz): for each (image, 16-pixel patch),
the folded LDS box (k_patch_boxes' rule) over all 125 rotations (the shared
box) and over each wave's 16 Morton-ranked rotations (a per-wave box), as
quantiles and as the fraction of samples whose box fits a capacity; plus the
distinct voxels the samples' taps actually touch (the reuse an ideal cache
would see).   python tools/wave_box_model.py clouds_eval.npz [nImg]"""
import sys

import numpy as np

from box_model import quat_to_mat  # noqa: E402
from group_model import boxes, tiles_image  # noqa: E402


def main():
    f = np.load(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    iCol, iRow, order = f["iCol"], f["iRow"], f["order"]
    pf = 2
    patches = []
    for c in range(0, len(order), 16):
        p = order[c:c + 16]
        p = p[p >= 0]
        patches.append(p)
    for key in sorted(k for k in f.files if k.startswith("quat_k")):
        Q = f[key][:n].astype(np.float64)
        Q /= np.linalg.norm(Q, axis=-1, keepdims=True)
        T = tiles_image(Q)                                   # [n, 125, 4] Morton-ranked
        T = np.concatenate([T, np.repeat(T[:, -1:], 3, 1)], 1)   # 128 slots
        M = quat_to_mat(T)                                   # [n, 128, 3, 3]
        shared, wave, distinct = [], [], []
        for p in patches:
            X0, X1 = iCol[p].min() * pf, iCol[p].max() * pf
            Y0, Y1 = iRow[p].min() * pf, iRow[p].max() * pf
            shared.append(boxes(M, X0, X1, Y0, Y1))
            wave.append(boxes(M.reshape(-1, 16, 3, 3), X0, X1, Y0, Y1).reshape(n, 8))
        shared = np.stack(shared, 1)      # [n, nC]
        wave = np.stack(wave, 1)          # [n, nC, 8]
        # distinct tap voxels per (image, patch) for the first 40 images
        pts = np.stack([iCol * pf, iRow * pf, np.zeros_like(iCol)], 1).astype(np.float64)
        for l in range(min(n, 40)):
            R = M[l, :125]
            for p in patches[::5]:
                c = np.einsum("rij,pj->rpi", R, pts[p]).reshape(-1, 3)
                c = np.where(c[:, :1] < 0, -c, c)
                b = np.floor(c).astype(np.int64)
                taps = (b[:, None, :] + np.array([[i, j, k] for i in (0, 1) for j in (0, 1)
                                                  for k in (0, 1)])[None]).reshape(-1, 3)
                distinct.append(len(np.unique(taps, axis=0)) / (len(p) * 125))
        q = lambda a: [int(x) for x in np.quantile(a, [0.1, 0.5, 0.9])]
        res = {"shared_q10_50_90": q(shared), "wave_q10_50_90": q(wave),
               "distinct_voxels_per_sample": round(float(np.mean(distinct)), 3)}
        for cap in (1024, 2048, 4096, 8192, 16384):
            res[f"shared<={cap}"] = round(float(np.mean(shared <= cap)), 3)
            res[f"wave<={cap}"] = round(float(np.mean(wave <= cap)), 3)
        print(key, res, flush=True)


if __name__ == "__main__":
    main()
