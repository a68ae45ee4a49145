#!/usr/bin/env python3
"""Diagnostic: cycles per staged patch iteration of k_local_fused, split by
phase (box write + image tile, barrier 1, prefetch issue, gathers, barrier 2),
for waves 0 (stager) and 7.  Needs a library built with -DTHX_LOCAL_STAMPS=1
(tools/build_define.sh stamps local.hip -DTHX_LOCAL_STAMPS=1; THX_LIB=...).
  python tools/local_stamps.py [--spread 1.5 --images 4096]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_stack  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402
from thunder_amd._lib import lib  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--spread", type=float, default=1.5)
    p.add_argument("--images", type=int, default=4096)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    N, pf = 256, 2
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    px, dat, ctf, sig, _, _ = make_stack(N, pf, 24, 1, a.images, dev, vol=vol)
    rng = np.random.default_rng(3)
    mR, mT = 125, 9
    q = synth.clustered_quaternions(a.images, mR, a.spread, rng)
    quat = torch.as_tensor(np.ascontiguousarray(q), device=dev)
    trans = torch.as_tensor(rng.standard_normal((a.images, mT, 2)), device=dev)
    pC = torch.ones(a.images, dtype=torch.float64, device=dev)
    pR = torch.full((a.images, mR), 1.0 / mR, dtype=torch.float64, device=dev)
    pT = torch.full((a.images, mT), 1.0 / mT, dtype=torch.float64, device=dev)
    L = lib()
    L.thx_debug_local_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 12)()
    ops.local_phase(vol, quat, trans, pC, pR, pT, dat, ctf, sig, px)
    torch.cuda.synchronize()
    L.thx_debug_local_stamps(buf, 1)
    ops.local_phase(vol, quat, trans, pC, pR, pT, dat, ctf, sig, px)
    torch.cuda.synchronize()
    L.thx_debug_local_stamps(buf, 0)
    names = ["box_write+tile", "barrier1", "prefetch_issue", "gathers", "barrier2"]
    out = {"spread": a.spread, "images": a.images}
    for w, base in (("wave0", 0), ("wave7", 6)):
        n = max(buf[base + 5], 1)
        out[w] = {k: round(buf[base + i] / n, 1) for i, k in enumerate(names)}
        out[w]["staged_iterations"] = buf[base + 5]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
