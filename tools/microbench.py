#!/usr/bin/env python3
"""Kernel micro-benchmarks for profiling (rocprofv3 target), not the headline bench.

  python tools/microbench.py local  [--box 256 --ru 24 --images 4096 --cells 0]
  python tools/microbench.py scan   [--algo 2 --images 4096]
  python tools/microbench.py insert [--images 1024 --mreco 100]
Prints one JSON line with the per-launch time measured with HIP events.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_stack, timed_events  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402


def box_stats(vol, quat, trans, pC, pR, pT, dat, ctf, sig, px, rec_ints=20, rt=128, kc=16):
    """Patch-box voxel counts from the records k_patch_boxes leaves at the
    start of the workspace (dvp passed explicitly, so the records come first)."""
    from thunder_amd.ops import _ptr, _stream, workspace
    from thunder_amd._lib import check, lib
    nImg, nR, nT = quat.shape[0], quat.shape[1], trans.shape[1]
    dev = dat.device
    d = torch.empty(nImg, nR, nT, dtype=torch.float32, device=dev)
    w = [torch.empty(nImg, *s, dtype=torch.float32, device=dev) for s in ((), (nR,), (nT,), ())]
    ws = workspace(lib().thx_local_phase_workspace(nImg, nR, nT, len(px.order)), dev)
    ws.zero_()
    check(lib().thx_local_phase(_ptr(vol), 0, vol.shape[0], px.pf, _ptr(quat), nR, _ptr(trans), nT,
                                _ptr(pC), _ptr(pR), _ptr(pT), _ptr(dat), _ptr(ctf), _ptr(sig),
                                _ptr(px.d_iCol), _ptr(px.d_iRow), _ptr(px.d_order), len(px.order),
                                px.n, px.idim, nImg, _ptr(w[0]), _ptr(w[1]), _ptr(w[2]), _ptr(w[3]),
                                _ptr(d), _ptr(ws), ws.numel(), _stream(dev)), "thx_local_phase")
    torch.cuda.synchronize()
    nC = (len(px.order) + kc - 1) // kc
    nRT = (nR + rt - 1) // rt
    rec = ws.view(torch.int32)[:nImg * nRT * nC * rec_ints].view(nImg, nRT, nC, rec_ints)
    tot = rec[..., 10].double().flatten()
    q = torch.tensor([0.1, 0.5, 0.9], dtype=torch.float64, device=dev)
    return {"box_voxels_p10_p50_p90": [int(v) for v in torch.quantile(tot, q)],
            "staged_frac": {str(c): float((tot <= c).double().mean()) for c in (4096, 8192, 16384, 32768)}}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("what", choices=["local", "scan", "insert"])
    p.add_argument("--box", type=int, default=256)
    p.add_argument("--ru", type=int, default=24)
    p.add_argument("--images", type=int, default=4096)
    p.add_argument("--cells", type=int, default=0)
    p.add_argument("--ypair", type=int, default=0, help="local: gather from ops.volume_ypair(vol)")
    p.add_argument("--algo", type=int, default=4)
    p.add_argument("--guard", type=float, default=None, help="scan: cancellation guard (None: the default 4, 0: off)")
    p.add_argument("--nr", type=int, default=2000)
    p.add_argument("--mreco", type=int, default=100)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--tiled", type=int, default=1,
                   help="local: 1 = tile visiting order (LDS-staged patches), 0 = set order")
    p.add_argument("--stats", type=int, default=0,
                   help="local: report patch-box sizes (voxels per LDS neighbourhood)")
    p.add_argument("--nd", type=int, default=0,
                   help="local: CTF search over nd defocus samples (thx_local_phase_d), 0 = off")
    p.add_argument("--spread", type=float, default=3.0,
                   help="local: rotation spread (deg) of each image's cloud, 0 = uniform")
    p.add_argument("--clouds", default="",
                   help="local: npz of quaternion clouds (quat_k<k>: [images, 125, 4]) instead of synthetic ones")
    p.add_argument("--k", type=int, default=0, help="local: phase of --clouds (quat_k<k>)")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    N, pf = a.box, 2
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    px, dat, ctf, sig, qtrue, ttrue = make_stack(N, pf, a.ru, 1, a.images, dev, vol=vol)
    st = torch.cuda.current_stream(dev)
    rng = np.random.default_rng(3)
    out = {"what": a.what, "box": N, "rU": a.ru, "nPxl": px.n, "images": a.images}
    if a.what == "local":
        mR, mT = 125, 9
        if a.clouds:       # the bench's own clouds at phase k
            q = np.load(a.clouds)[f"quat_k{a.k}"][:a.images].astype(np.float64)
            q /= np.linalg.norm(q, axis=-1, keepdims=True)
            assert q.shape == (a.images, mR, 4), q.shape
            out.update(clouds=a.clouds, k=a.k)
        elif a.spread > 0:   # particle clouds: perturbations of one pose per image
            q = synth.clustered_quaternions(a.images, mR, a.spread, rng)
        else:
            q = synth.uniform_quaternions(a.images * mR, rng).reshape(a.images, mR, 4)
        quat = torch.as_tensor(np.ascontiguousarray(q), device=dev)
        trans = torch.as_tensor(rng.standard_normal((a.images, mT, 2)), device=dev)
        pC = torch.ones(a.images, dtype=torch.float64, device=dev)
        pR = torch.full((a.images, mR), 1.0 / mR, dtype=torch.float64, device=dev)
        pT = torch.full((a.images, mT), 1.0 / mT, dtype=torch.float64, device=dev)
        cells = ops.volume_cells(vol) if a.cells else None
        ypair = ops.volume_ypair(vol) if a.ypair else None
        out.update(cells=a.cells, ypair=a.ypair)
        if a.nd > 0:
            dD = torch.as_tensor(1 + rng.standard_normal((a.images, a.nd)) * 0.01, device=dev)
            ctfD = (ctf[:, None, :] * (1 + 0.01 * torch.arange(a.nd, device=dev)[None, :, None]))
            ctfD = ctfD.float().contiguous()
            pD = torch.full((a.images, a.nd), 1.0 / a.nd, dtype=torch.float64, device=dev)
            sec = timed_events(lambda: ops.local_phase_d(vol, quat, trans, pC, pR, pT, pD, dat, ctfD,
                                                         sig, px, cells=cells),
                               a.reps, st)
            out["nd"] = a.nd
            del dD
        else:
            sec = timed_events(lambda: ops.local_phase(vol, quat, trans, pC, pR, pT, dat, ctf, sig,
                                                       px, cells=cells, tiled=bool(a.tiled),
                                                       ypair=ypair),
                               a.reps, st)
        if a.stats:
            out.update(box_stats(vol, quat, trans, pC, pR, pT, dat, ctf, sig, px))
        out.update(ms=sec * 1e3, us_per_image_phase=sec / a.images * 1e6,
                   algo_GBps=a.images * (64.0 * mR * px.n + 16.0 * px.n) / sec / 1e9)
    elif a.what == "scan":
        q, t, pR, pT = synth.global_sample_set(a.nr, seed=2)
        rotP = ops.project3d(vol, ops.rotmat(torch.as_tensor(q, device=dev)), px)
        traP = ops.trans_table(torch.as_tensor(t, device=dev), px)
        pRd, pTd = torch.as_tensor(pR, device=dev), torch.as_tensor(pT, device=dev)
        sec = timed_events(lambda: ops.global_scan(rotP, traP, dat, ctf, sig, pRd, pTd,
                                                   algo=a.algo, guard=a.guard), a.reps, st)
        out.update(ms=sec * 1e3, us_per_image=sec / a.images * 1e6, algo=a.algo)
    else:
        rec = ex.Reconstructor(N, pf, dev)
        if a.spread > 0:   # posterior samples: a cloud around one pose per image
            q = synth.clustered_quaternions(a.images, a.mreco, a.spread, rng)
        else:
            q = synth.uniform_quaternions(a.images * a.mreco, rng).reshape(a.images, a.mreco, 4)
        quat = torch.as_tensor(np.ascontiguousarray(q), device=dev)
        trans = torch.as_tensor(rng.standard_normal((a.images, a.mreco, 2)), device=dev)
        offS = torch.zeros(a.images, 2, dtype=torch.float64, device=dev)
        w = torch.full((a.images,), 1.0 / a.mreco, dtype=torch.float32, device=dev)
        sec = timed_events(lambda: rec.insert(dat, ctf, quat, trans, offS, w, px, tiled=bool(a.tiled)),
                           a.reps, st)
        out.update(ms=sec * 1e3, images_per_s=a.images / sec)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
