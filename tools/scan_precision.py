"""Global-scan precision and speed probe (C3 shape: box 256, nR 2000, nT 151,
rU 24).  For SNR 0.05 (bench stack) and SNR 20 (grid poses) it compares every
sample's dvp of each split algorithm, with and without the cancellation
guard, with the CPU restatement (orc.dvp_global), and times the scan on
--images images per algorithm.  One JSON line per measurement.

    python tools/scan_precision.py [--images 4096] [--check 8]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from bench import make_stack, timed_events  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--images", type=int, default=4096)
    p.add_argument("--check", type=int, default=8)
    p.add_argument("--algos", default="2,4")
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    from oracle import oracle as orc
    from test_gpu_driver import grid_images
    orc.build()
    dev = torch.device("cuda", 0)
    N, pf = 256, 2
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    q, t, pR, pT = gset = synth.global_sample_set(2000, seed=2)
    pxh = orc.pixel_set(N, pf, 24, 1)
    px, dat, ctf, sig, *_ = make_stack(N, pf, 24, 1, max(a.images, a.check), dev, seed=19, vol=vol)
    rotP = ops.project3d(vol, ops.rotmat(torch.as_tensor(q, device=dev)), px)
    traP = ops.trans_table(torch.as_tensor(t, device=dev), px)
    pRd, pTd = torch.as_tensor(pR, device=dev), torch.as_tensor(pT, device=dev)
    algos = [int(x) for x in a.algos.split(",")]
    stacks = {"snr0.05": (dat[:a.check].contiguous(), ctf[:a.check].contiguous(),
                          sig[:a.check].contiguous())}
    g = grid_images(vol[None].contiguous(), px, gset, a.check, seed=70, snr=20.0)
    stacks["snr20"] = g[:3]
    vnp = vol.cpu().numpy()
    for name, (d_, c_, s_) in stacks.items():
        ref = orc.dvp_global(vnp, pf * N, pf, q, t, d_.cpu().numpy(), c_.cpu().numpy(),
                             s_.cpu().numpy(), pxh, N, threads=16)
        ref64 = ref.astype(np.float64)
        for algo in algos:
            for guard in (0.0, 4.0):
                out = ops.global_scan(rotP, traP, d_, c_, s_, pRd, pTd, algo=algo, guard=guard,
                                      want_dvp=True)
                dv = out[4].cpu().numpy().astype(np.float64)
                rel = np.abs(dv - ref64) / np.abs(ref64)
                top = np.argsort(-rel.reshape(-1))[:3]
                print(json.dumps({"stack": name, "algo": algo, "guard": guard,
                                  "max_rel": float(rel.max()), "p99_rel": float(np.quantile(rel, 0.99)),
                                  "median_rel": float(np.median(rel)),
                                  "n_over_1e5": int((rel > 1e-5).sum()),
                                  "worst": [[int(i), float(ref64.reshape(-1)[i]),
                                             float(dv.reshape(-1)[i])] for i in top],
                                  "dvp_range": [float(ref64.min()), float(ref64.max())]}),
                      flush=True)
    st = torch.cuda.current_stream(dev)
    n = a.images
    for algo in algos + [1]:
        sec = timed_events(lambda: ops.global_scan(rotP, traP, dat[:n], ctf[:n], sig[:n], pRd, pTd,
                                                   algo=algo), a.reps, st)
        print(json.dumps({"timing": True, "algo": algo, "images": n, "ms": sec * 1e3,
                          "ms_per_12500": sec * 1e3 * 12500 / n}), flush=True)


if __name__ == "__main__":
    main()
