#!/usr/bin/env python3
"""Per-iteration cost of the inferACG fixed point (thx_pf_acg_mean) on
synthetic clouds: 12 500 images of 125 particles, either 125 distinct
clustered quaternions or a few distinct ancestors repeated (the clouds that
run the fixed point to its cap), timed at several iteration caps.
    python tools/pf_probe.py [--dump DIR]   (DIR: every call's means, .npy, to
    compare two libraries bit for bit)"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from thunder_amd import ops, synth  # noqa: E402
from thunder_amd._lib import check, lib  # noqa: E402

dev = torch.device("cuda", 0)
n, m = 12500, 125
rng = np.random.default_rng(1)
st = torch.cuda.current_stream(dev)


DUMP = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None


def timed(quat, cap, reps=5, tag=""):
    mq = torch.empty(n, 4, dtype=torch.float64, device=dev)
    it = torch.empty(n, dtype=torch.int32, device=dev)
    f = lambda: check(lib().thx_pf_acg_mean(n, m, ops._ptr(quat), cap, ops._ptr(mq), ops._ptr(it),
                                            ctypes.c_void_p(st.cuda_stream)), "acg")
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        f()
    b.record(st)
    torch.cuda.synchronize()
    h = it.cpu().numpy()
    if DUMP:
        os.makedirs(DUMP, exist_ok=True)
        np.save(os.path.join(DUMP, f"{tag}_cap{cap}_mean.npy"), mq.cpu().numpy())
        np.save(os.path.join(DUMP, f"{tag}_cap{cap}_iters.npy"), h)
    return a.elapsed_time(b) / reps, float(np.median(h)), int(h.max())


clouds = {}
clouds["distinct_3deg"] = synth.clustered_quaternions(n, m, 3.0, rng)
for d in (1, 4, 7, 16):
    base = synth.clustered_quaternions(n, d, 3.0, rng)
    idx = np.sort(rng.integers(0, d, size=(n, m)), axis=1)
    clouds[f"ancestors_{d}"] = np.take_along_axis(base, idx[..., None].repeat(4, -1), axis=1)
for name, q in clouds.items():
    quat = torch.as_tensor(np.ascontiguousarray(q), device=dev)
    for cap in (10, 100, 256):
        ms, p50, mx = timed(quat, cap, tag=name)
        print(json.dumps({"lib": os.path.basename(os.environ.get("THX_LIB", "prod")),
                          "cloud": name, "cap": cap, "ms": round(ms, 4), "iters_p50": p50,
                          "iters_max": mx}), flush=True)
