#!/usr/bin/env python3
"""Pose recovery of the expectation driver on a high-SNR synthetic stack:
angle of the global scan's best rotation and of the driver's top particle
to the true pose, after 0 / 1 / 3 / 10 particle-filter phases.

  python tools/diag_expect.py [--box 64 --ru 12 --snr 20 --images 96 --nr 1500]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_stack  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402


def angle_deg(qa, qb):
    c = (qa * qb).sum(-1).abs().clamp(max=1)
    return torch.rad2deg(2 * torch.acos(c))


def stats(e):
    q = torch.tensor([0.1, 0.5, 0.9], dtype=e.dtype, device=e.device)
    return [round(float(v), 2) for v in torch.quantile(e, q)] + [round(float((e > 20).double().mean()), 3)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--box", type=int, default=64)
    p.add_argument("--ru", type=int, default=12)
    p.add_argument("--snr", type=float, default=20.0)
    p.add_argument("--images", type=int, default=96)
    p.add_argument("--nr", type=int, default=1500)
    p.add_argument("--algo", type=int, default=2)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    N, pf = a.box, 2
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    px, dat, ctf, sig, qtrue, ttrue = make_stack(N, pf, a.ru, 1, a.images, dev, seed=21, snr=a.snr,
                                                 vol=vol)
    gset = synth.global_sample_set(a.nr, seed=2)
    q, t, pR, pT = gset
    gq = torch.as_tensor(q, device=dev)
    rotP = ops.project3d(vol, ops.rotmat(gq), px)
    traP = ops.trans_table(torch.as_tensor(t, device=dev), px)
    wC, wR, wT, base = ops.global_scan(rotP, traP, dat, ctf, sig, torch.as_tensor(pR, device=dev),
                                       torch.as_tensor(pT, device=dev), algo=a.algo)
    best = wR.reshape(a.images, -1).argmax(-1)
    nearest = angle_deg(gq[None, :, :], qtrue[:, None, :]).min(-1).values
    out = {"scan_best_err_p10_p50_p90_fracgt20": stats(angle_deg(gq[best], qtrue)),
           "grid_nearest_err": stats(nearest),
           "scan_best_trans_err_p50": float((torch.as_tensor(t, device=dev)[wT.reshape(a.images, -1)
                                                                          .argmax(-1)] - ttrue)
                                           .norm(dim=-1).median())}
    # likelihood of the true pose vs the scan's pick (direct dvp, translation = truth)
    for n_phase in (0, 1, 3, 10):
        e = ex.Expectation(vol, px, gset, n_phase=n_phase, algo=a.algo, seed=5)
        quat, trans, pRo, pTo, score = e.run(dat, ctf, sig)[:5]
        out[f"phase{n_phase}_mode_err"] = stats(angle_deg(ex.cloud_mode(quat), qtrue))
        out[f"phase{n_phase}_idx0_err"] = stats(angle_deg(quat[:, 0], qtrue))
        out[f"phase{n_phase}_trans_err_p50"] = float((trans[:, 0] - ttrue).norm(dim=-1).median())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
