#!/usr/bin/env python3
"""Timing of the particle statistics kernels (thx_pf_calvari / balance_rot)
on 12500 images x 125 particles for several cloud shapes."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import timed_events  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402

dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)
n, m = 12500, 125
st = torch.cuda.current_stream(dev)
trans = torch.as_tensor(rng.standard_normal((n, 9, 2)), device=dev)
for name in ("cluster3", "cluster30", "dup3", "dup1"):
    if name.startswith("cluster"):
        q = synth.clustered_quaternions(n, m, float(name[7:]), rng)
    else:
        nd = int(name[3:])
        base = synth.clustered_quaternions(n, nd, 3.0, rng)
        q = base[np.arange(n)[:, None], rng.integers(0, nd, (n, m))]
    q = torch.as_tensor(np.ascontiguousarray(q), device=dev)
    tc = timed_events(lambda: ops.pf_calvari(q, trans), 3, st)
    tb = timed_events(lambda: ops.pf_balance_rot(q), 3, st)
    print(json.dumps({"cloud": name, "calvari_ms": tc * 1e3, "balance_ms": tb * 1e3}), flush=True)
