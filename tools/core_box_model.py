#!/usr/bin/env python3
"""CPU model: fraction of the local phase's (rotation, pixel) samples that an
LDS patch box can serve when the box holds only the tile's CORE rotations
(rotated patch centre within +-D voxels of the mean centre, largest D whose
hull fits the cap) and the outliers gather from L2, against the current
all-or-nothing box.  python tools/core_box_model.py gpurun_out/clouds.npz [cap] [nimg]"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from box_model import box_voxels, quat_to_mat  # noqa: E402


def main():
    f = np.load(sys.argv[1])
    iCol, iRow, order = f["iCol"], f["iRow"], f["order"]
    pf, KC = 2, 16
    CAP = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    nimg = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    Ds = (16, 12, 8, 6, 5, 4, 3, 2.5, 2, 1.5, 1, 0.5)
    patches = []
    for c in range(0, len(order), KC):
        p = order[c:c + KC]
        p = p[p >= 0]
        if len(p):
            patches.append((iCol[p].min() * pf, iCol[p].max() * pf, iRow[p].min() * pf,
                            iRow[p].max() * pf, len(p)))
    for key in sorted(k for k in f.files if k.startswith("quat_k")):
        Q = f[key]
        full = core = tot = 0
        for q in Q[:nimg]:
            M = quat_to_mat(q)
            u, v = M[:, :, 0], M[:, :, 1]
            for (X0, X1, Y0, Y1, n) in patches:
                w = n * len(M)
                tot += w
                if box_voxels(M, X0, X1, Y0, Y1) <= CAP:
                    full += w
                    core += w
                    continue
                cx, cy = 0.5 * (X0 + X1), 0.5 * (Y0 + Y1)
                c = u * cx + v * cy                      # rotated patch centres [nR, 3]
                c = np.where(c[:, :1] < 0, -c, c)        # folded side
                m = np.median(c, axis=0)
                d = np.abs(c - m).max(1)
                for D in Ds:
                    sel = d <= D
                    if sel.sum() and box_voxels(M[sel], X0, X1, Y0, Y1) <= CAP:
                        core += n * sel.sum()
                        break
        print(key, f"cap {CAP}: all-or-nothing staged {full / tot:.3f}, core box staged {core / tot:.3f}",
              flush=True)


if __name__ == "__main__":
    main()
