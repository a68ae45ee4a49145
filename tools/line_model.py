"""Cache-line model of the full-resolution local phase (box 256, pf 2,
rU 126: pixels 2 projectee voxels apart) -- how many distinct 128-B lines a
rotation-pixel sample needs if the cache keeps lines for

  * one wave instruction of the current lane mapping (cells: 16 rotations x 1
    pixel; y-pair pair form: 8 rotations x 4 pixels, two slice loads),
  * one workgroup iteration (all 125 rotations x 32 pixels of a chunk),
  * W consecutive chunks (W = 4 .. 64),
  * the whole image (all rotations, all pixels: the floor of any schedule
    that keeps each image's lines until its last use).

The projectee layouts are the kernels' own: the cell-expanded copy (64-B cell
per base voxel, thx_volume_cells) and the z-interleaved y-pair copy
(thx_volume_ypair).  Clouds: Gaussian perturbations of one random pose
(sigma 1.5 / 2 / 3 degrees per axis) or uniformly random rotations, as
bench.local_roofline draws them.

    python tools/line_model.py [--images 2] > profiles/r06_line_model.json
"""
import argparse
import json

import numpy as np

HALF = 256             # projectee half size at box 256, pf 2
NC, VD = HALF + 1, 2 * HALF


def qmat(q):
    a, b, c, d = q.T
    return np.stack([np.stack([a * a + b * b - c * c - d * d, 2 * (b * c - a * d), 2 * (b * d + a * c)], -1),
                     np.stack([2 * (b * c + a * d), a * a - b * b + c * c - d * d, 2 * (c * d - a * b)], -1),
                     np.stack([2 * (b * d - a * c), 2 * (c * d + a * b), a * a - b * b - c * c + d * d], -1)],
                    -2)


def cloud(rng, n, spread):
    if spread is None:
        q = rng.normal(size=(n, 4))
        return qmat(q / np.linalg.norm(q, axis=1, keepdims=True))
    c = rng.normal(size=4)
    C = qmat((c / np.linalg.norm(c))[None])[0]
    ang = np.deg2rad(spread) * rng.normal(size=(n, 3))
    th = np.linalg.norm(ang, axis=1, keepdims=True)
    q = np.concatenate([np.cos(th / 2), ang / np.maximum(th, 1e-12) * np.sin(th / 2)], 1)
    return qmat(q) @ C


def tile_order(ru):
    """thx_pixel_tile_order: serpentine rows of 4 x 4 squares, 2 x 2 quads inside."""
    ii, jj = np.meshgrid(np.arange(0, ru + 1), np.arange(-ru, ru + 1), indexing="ij")
    m = (ii ** 2 + jj ** 2 < ru ** 2) & ~((ii == 0) & (jj < 0))
    ic, ir = ii[m], jj[m]
    ntc = (ic.max() - ic.min()) // 4 + 1
    tr, tc0 = (ir - ir.min()) // 4, (ic - ic.min()) // 4
    key = tr * ntc + np.where(tr & 1, ntc - 1 - tc0, tc0)
    lc, lr = (ic - ic.min()) % 4, (ir - ir.min()) % 4
    sub = ((lr // 2) * 2 + lc // 2) * 4 + (lr % 2) * 2 + lc % 2
    o = np.lexsort((sub, key))
    return np.stack([ic[o], ir[o]], 1).astype(float) * 2      # projectee coordinates (pf 2)


def base(R, px):
    p = px @ R[:, :2].T
    p[p[:, 0] < 0] *= -1                                    # Hermitian fold
    return np.floor(p).astype(np.int64)


def lines_cells(f):
    return [(((f[:, 2] % VD) * VD + f[:, 1] % VD) * NC + f[:, 0]) * 64 // 128]


def lines_ypair(f):
    out = []
    for dz in (0, 1):                                        # one load per slice
        z, y = (f[:, 2] + dz) % VD, f[:, 1] % VD
        e = [((((z >> 1) * VD + y) * NC + f[:, 0] + dx) * 2 + (z & 1)) * 16 // 128 for dx in (0, 1)]
        out.append(np.concatenate(e))
    return out


def model(rng, spread, layout, n_img, ru=126, nrot=125, chunk=32):
    px = tile_order(ru)
    fn = lines_cells if layout == "cells" else lines_ypair
    inst = 0
    windows = {1: 0, 4: 0, 16: 0, 64: 0}
    image = 0
    ns = 0
    for _ in range(n_img):
        R = cloud(rng, nrot, spread)
        F = np.stack([base(R[r], px) for r in range(nrot)])   # [rot][px][3]
        chunks = []
        for c0 in range(0, len(px), chunk):
            s = set()
            for r0 in range(0, nrot, 16):                     # the workgroup's waves
                blk = F[r0:r0 + 16, c0:c0 + chunk]
                if layout == "cells":                         # 16 rotations x 1 pixel
                    for p in range(blk.shape[1]):
                        ls = fn(blk[:, p])[0]
                        inst += len(set(ls.tolist()))
                        s.update(ls.tolist())
                else:                                         # 8 rotations x 4 pixels, 2 slices
                    for h in (0, 8):
                        for p0 in range(0, blk.shape[1], 4):
                            for ls in fn(blk[h:h + 8, p0:p0 + 4].reshape(-1, 3)):
                                inst += len(set(ls.tolist()))
                                s.update(ls.tolist())
            chunks.append(s)
        for w in windows:
            for k in range(0, len(chunks), w):
                windows[w] += len(set().union(*chunks[k:k + w]))
        image += len(set().union(*chunks))
        ns += nrot * len(px)
    return {"per_instruction": inst / ns,
            **{f"window_{w}_chunks": v / ns for w, v in windows.items()},
            "whole_image": image / ns}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=2)
    a = ap.parse_args()
    rng = np.random.default_rng(7)
    rows = []
    for spread in (1.5, 2.0, 3.0, None):
        for layout in ("cells", "ypair"):
            r = model(rng, spread, layout, a.images)
            rows.append({"spread_deg": spread if spread else "uniform", "layout": layout,
                         **{k: round(v, 3) for k, v in r.items()}})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
