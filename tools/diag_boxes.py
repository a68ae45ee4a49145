#!/usr/bin/env python3
"""Patch-box statistics of the bench's own particle clouds: run the bench's
expectation (C3, 4096 images) for k phases and report the LDS box sizes
k_patch_boxes computes for the clouds the next phase would start from, plus
the phase time of k_local_fused on them.
  python tools/diag_boxes.py [--images 4096]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_stack, timed_events  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import synth  # noqa: E402
from tools.microbench import box_stats  # noqa: E402
from thunder_amd import ops  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--images", type=int, default=4096)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    N, pf = 256, 2
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    gset = synth.global_sample_set(2000, seed=2)
    px, dat, ctf, sig, *_ = make_stack(N, pf, 24, 1, a.images, dev, seed=5, vol=vol)
    st = torch.cuda.current_stream(dev)
    for k in (0, 1, 3, 6, 10):
        e = ex.Expectation(vol, px, gset, n_phase=k, seed=7)
        quat, trans, pR, pT = [x.clone() for x in e.run(dat, ctf, sig)[:4]]
        pC = torch.ones(a.images, dtype=torch.float64, device=dev)
        out = {"after_phases": k}
        out.update(box_stats(vol, quat, trans, pC, pR, pT, dat, ctf, sig, px))
        sec = timed_events(lambda: ops.local_phase(vol, quat, trans, pC, pR, pT, dat, ctf, sig, px), 3, st)
        q0 = ex.cloud_mode(quat)
        ang = torch.rad2deg(2 * torch.acos((quat * q0[:, None, :]).sum(-1).abs().clamp(max=1)))
        qs = torch.tensor([0.1, 0.5, 0.9], dtype=ang.dtype, device=dev)
        out["max_spread_p10_p50_p90"] = [round(float(v), 1) for v in torch.quantile(ang.max(1).values, qs)]
        out["p90_spread_p10_p50_p90"] = [round(float(v), 1) for v in
                                         torch.quantile(torch.quantile(ang, 0.9, dim=1), qs)]
        out["phase_ms"] = sec * 1e3
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
