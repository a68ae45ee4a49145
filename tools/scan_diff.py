"""Where two global-scan variants differ: dvp dumps (thx_global_scan_dvp) of
bf16x3 and bf16x6 with and without the guard on one 64-image tile, per image
row.  Debug tool.

    python tools/scan_diff.py [--images 64] [--snr 0.05]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import make_stack  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--images", type=int, default=64)
    p.add_argument("--snr", type=float, default=0.05)
    p.add_argument("--nr", type=int, default=2000)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    N, pf = 256, 2
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    q, t, pR, pT = synth.global_sample_set(a.nr, seed=2)
    px, dat, ctf, sig, *_ = make_stack(N, pf, 24, 1, a.images, dev, seed=9, vol=vol, snr=a.snr)
    rotP = ops.project3d(vol, ops.rotmat(torch.as_tensor(q, device=dev)), px)
    traP = ops.trans_table(torch.as_tensor(t, device=dev), px)
    pRd, pTd = torch.as_tensor(pR, device=dev), torch.as_tensor(pT, device=dev)
    d0 = ops.dvp(rotP, traP, dat, ctf, sig).cpu().numpy().astype(np.float64)
    runs = {}
    for name, algo, guard in (("x3", 2, 0.0), ("x6", 4, 0.0), ("x6g", 4, 4.0), ("x6g_again", 4, 4.0)):
        runs[name] = ops.global_scan(rotP, traP, dat, ctf, sig, pRd, pTd, algo=algo, guard=guard,
                                     want_dvp=True)[4].cpu().numpy().astype(np.float64)
    for name, d in runs.items():
        rel = np.abs(d - d0) / np.abs(d0)
        per_row = rel.reshape(a.images, -1).max(1)
        bad = np.nonzero(per_row > 1e-5)[0]
        worst = np.unravel_index(rel.argmax(), rel.shape)
        print(json.dumps({"run": name, "max_rel_vs_direct": float(rel.max()),
                          "worst_lrt": [int(x) for x in worst],
                          "rows_over_1e-5": bad.tolist()[:64],
                          "per_row_max": [float(f"{x:.2e}") for x in per_row]}), flush=True)
    print(json.dumps({"x6g_deterministic": bool(np.array_equal(runs["x6g"], runs["x6g_again"]))}))
    marg = {a_: [x.cpu().numpy().astype(np.float64) for x in
                 ops.global_scan(rotP, traP, dat, ctf, sig, pRd, pTd, algo=a_)] for a_ in (0, 2, 4)}
    for a_ in (2, 4):
        out = {"marginals_algo": a_}
        for k, name in ((0, "wC"), (1, "wR"), (2, "wT"), (3, "base")):
            x, y = marg[a_][k].reshape(a.images, -1), marg[0][k].reshape(a.images, -1)
            m = np.abs(y) >= 1e-4 * np.abs(y).max(axis=-1, keepdims=True)
            out[name] = float((np.abs(x - y)[m] / np.abs(y[m])).max())
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
