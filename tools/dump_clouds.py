#!/usr/bin/env python3
"""Dump the bench's particle clouds (C3 stack, 12 500 images) as the local
phase evaluates them -- after each phase's perturbation -- for CPU-side
analysis of the patch boxes (tools/box_model.py, tools/group_model.py) and
for replay in tools/microbench.py --clouds.  Needs a THX_DUMP_QUAT build of
optimiser.hip (thx_debug_quat_sink):

  tools/build_define.sh dumpq optimiser.hip -DTHX_DUMP_QUAT=1
  THX_LIB=thunder_amd/ab/lib_dumpq.so python tools/dump_clouds.py [n_images_kept]

-> gpurun_out/clouds_eval.npz with quat_k{k} [n, 125, 4] float16 for phases
k = 0, 2, 5, 9 of the bench's 10 (the first n images of the 12 500)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_stack  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402
from thunder_amd._lib import lib  # noqa: E402

PHASES = (0, 2, 5, 9)


def main():
    keep = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev = torch.device("cuda", 0)
    N, pf, nImg, mR = 256, 2, 12500, 125
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    _, nR, nT = ops.global_sample_sizes(2000)   # as bench.py
    gset = tuple(x.cpu().numpy() for x in ops.global_sample_set(nR, nT, 10.0, 2, dev))
    px, dat, ctf, sig, *_ = make_stack(N, pf, 24, 1, nImg, dev, seed=5, vol=vol)
    sink = torch.zeros(len(PHASES), nImg, mR, 4, dtype=torch.float64, device=dev)
    mask = sum(1 << k for k in PHASES)
    lib().thx_debug_quat_sink(ctypes.c_void_p(sink.data_ptr()), ctypes.c_uint(mask))
    e = ex.Expectation(vol, px, gset, n_phase=10, algo=2, seed=7, shuffle=True,
                       perturb_mean="acg", acg_iters=100, large_first=False)
    e.run(dat, ctf, sig)
    torch.cuda.synchronize()
    lib().thx_debug_quat_sink(None, ctypes.c_uint(0))
    out = {"iCol": px.iCol, "iRow": px.iRow, "order": px.order}
    for j, k in enumerate(PHASES):
        out[f"quat_k{k}"] = sink[j, :keep].cpu().numpy().astype(np.float16)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                     "gpurun_out", "clouds_eval.npz"), **out)
    print("ok", flush=True)


if __name__ == "__main__":
    main()
