#!/usr/bin/env python3
"""Throughput of the expectation at the other BASELINE.json configurations
(one MI355X; the headline C3 line is bench.py's).  One JSON line per config:

  C2  3D refine, box 128, nR 500 -> 1500 (the 3D clamp), 151 translations,
      rU 12, 10 phases of 125 x 9
  C4  3D classification, K = 4, box 200, nR 2000, rU 19, class scan + reseed
      + 10 phases on the drawn class
  C5  3D local search, box 512, 200 x 9 particles, full resolution rU 254
      (nPxl 100 928), 3 phases (MIN_N_PHASE_PER_ITER_LOCAL)
  CS  SEARCH_TYPE_CTF at the C3 shape: local search with 9 defocus samples,
      3 phases

Synthetic data (seeded blob volumes, CTF-modulated noisy projections);
images/s = images / wall time of one expectation call (inputs resident).

  python tools/config_bench.py [--only C2,C4,C5,CS]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_stack  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402


def wall(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def global_cfg(name, N, mS, rU, rL, n_img, K, dev):
    vols = [synth.projectee(synth.blob_volume(N, seed=11 + k, device=dev), 2) for k in range(K)]
    vol = vols[0] if K == 1 else torch.stack(vols).contiguous()
    px, dat, ctf, sig, _, _ = make_stack(N, 2, rU, rL, n_img, dev, vol=vols[0])
    mS2, nR, nT = ops.global_sample_sizes(mS)
    gset = tuple(x.cpu().numpy() for x in ops.global_sample_set(nR, nT, 10.0, 2, dev))
    e = ex.Expectation(vol, px, gset, n_phase=10, seed=7)
    out = [None]

    def run():
        out[0] = e.run(dat, ctf, sig, out=out[0])
    sec = wall(run)
    return {"config": name, "box": N, "K": K, "mS": mS, "nR": nR, "nT": nT, "nPxl": px.n,
            "images": n_img, "phases": 10, "s_per_call": sec, "images_per_s": n_img / sec}


def local_cfg(name, N, rU, rL, n_img, mR, mT, dev, mLD=0, spread=3.0, cells=False):
    vol = synth.projectee(synth.blob_volume(N, seed=21, device=dev), 2)
    vc = ops.volume_cells(vol) if cells else None
    px, dat, ctf, sig, qtrue, ttrue = make_stack(N, 2, rU, rL, n_img, dev, vol=vol)
    rng = np.random.default_rng(5)
    q0 = torch.as_tensor(synth.clustered_quaternions(n_img, mR, spread, rng), device=dev)
    t0 = ttrue[:, None, :] + torch.as_tensor(rng.uniform(-1, 1, (n_img, mT, 2)), device=dev)
    pR0 = torch.full((n_img, mR), 1.0 / mR, dtype=torch.float64, device=dev)
    pT0 = torch.full((n_img, mT), 1.0 / mT, dtype=torch.float64, device=dev)
    e = ex.Expectation(vol, px, None, mLR=mR, mLT=mT, n_phase=3, seed=7,
                       search="ctf" if mLD else "local", mLD=max(mLD, 1), cells=vc)
    attrs = torch.as_tensor(synth.ctf_attrs(n_img, seed=6), device=dev)

    def run():
        st = (q0.clone(), t0.clone().contiguous(), pR0.clone(), pT0.clone())
        if mLD:
            e.run_ctf(dat, attrs, sig, st)
        else:
            e.run(dat, ctf, sig, state=st)
    sec = wall(run)
    algo = n_img * 3 * (64.0 * mR * px.n + 16.0 * px.n)   # SURVEY 8(d) bytes, 3 phases
    return {"config": name, "box": N, "search": "ctf" if mLD else "local", "mLR": mR, "mLT": mT,
            "mLD": mLD, "nPxl": px.n, "images": n_img, "phases": 3, "cloud_spread_deg": spread,
            "projectee": "cells" if cells else "half-complex", "s_per_call": sec,
            "images_per_s": n_img / sec, "algorithmic_GBps_incl_pf": algo / sec / 1e9}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--only", default="C2,C4,C5,C5cells,C5n,C5ncells,CS")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    jobs = {
        "C2": lambda: global_cfg("C2", 128, 500, 12, 0, 8192, 1, dev),
        "C4": lambda: global_cfg("C4", 200, 2000, 19, 1, 4096, 4, dev),
        "C5": lambda: local_cfg("C5", 512, 254, 3, 256, 200, 9, dev),
        "C5cells": lambda: local_cfg("C5", 512, 254, 3, 256, 200, 9, dev, cells=True),
        "C5n": lambda: local_cfg("C5", 512, 254, 3, 256, 200, 9, dev, spread=1.0),
        "C5ncells": lambda: local_cfg("C5", 512, 254, 3, 256, 200, 9, dev, spread=1.0, cells=True),
        "CS": lambda: local_cfg("CS (C3 shape)", 256, 24, 1, 4096, 125, 9, dev, mLD=9),
    }
    for k in a.only.split(","):
        try:
            r = jobs[k]()
        except Exception as exc:   # report and go on with the next config
            r = {"config": k, "error": f"{type(exc).__name__}: {exc}"}
        print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
