#!/usr/bin/env python3
"""Dump the bench's particle clouds (C3 stack, 12 500 images) after k phases
(all images, float16) for CPU-side analysis of the local phase's patch boxes
(tools/box_model.py, tools/group_model.py): gpurun_out/clouds.npz with
quat_k{k} [12500, 125, 4]."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_stack  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    N, pf = 256, 2
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    gset = synth.global_sample_set(2000, seed=2)
    px, dat, ctf, sig, *_ = make_stack(N, pf, 24, 1, 12500, dev, seed=5, vol=vol)
    out = {"iCol": px.iCol, "iRow": px.iRow, "order": px.order}
    sel = torch.arange(0, 12500, 1, device=dev)
    for k in (0, 2, 5, 9):
        e = ex.Expectation(vol, px, gset, n_phase=k, seed=7)
        q = e.run(dat, ctf, sig)[0]
        out[f"quat_k{k}"] = q[sel].cpu().numpy().astype(np.float16)
        print(k, flush=True)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                     "gpurun_out", "clouds.npz"), **out)


if __name__ == "__main__":
    main()
