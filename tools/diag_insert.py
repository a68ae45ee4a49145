#!/usr/bin/env python3
"""Insert diagnostics on the bench's own posterior samples: run the bench's
expectation (C3), draw mReco = 100 insert samples per image, and report for
one hemisphere's k_insert_patches launch the patch-box sizes, how many
workgroups fit INS_CAP in one pass / need z-chunks / fall back to direct
scatter, the upper bound of flushed voxels, and the launch time (tiled and
direct).  Optional variant libraries (tools/build_variants.sh) are timed on the
same samples: python tools/diag_insert.py [--images 12500] [--libs a b ...]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_stack, timed_events  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402
from thunder_amd._lib import SIGNATURES, lib  # noqa: E402

INS_CAP, KC, RT, REC = 5120, 16, 128, 20


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--images", type=int, default=12500)
    p.add_argument("--mreco", type=int, default=100)
    p.add_argument("--libs", nargs="*", default=[])
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    N, pf = 256, 2
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    gset = synth.global_sample_set(2000, seed=2)
    px, dat, ctf, sig, *_ = make_stack(N, pf, 24, 1, a.images, dev, seed=5, vol=vol)
    e = ex.Expectation(vol, px, gset, n_phase=10, seed=7)
    out = e.run(dat, ctf, sig)
    iq, it = ex.draw_insert_samples(out[0], out[1], a.mreco)
    h = torch.arange(0, a.images, 2, device=dev)
    d, c, q, t = dat[h].contiguous(), ctf[h].contiguous(), iq[h].contiguous(), it[h].contiguous()
    n = d.shape[0]
    off = torch.zeros(n, 2, dtype=torch.float64, device=dev)
    w = torch.full((n,), 1.0 / a.mreco, dtype=torch.float32, device=dev)
    hm = ops.HalfMap(N * pf, dev)
    st = torch.cuda.current_stream(dev)
    res = {"images_per_launch": n, "mReco": a.mreco, "nPxl": px.n}
    res["binned_ms"] = timed_events(lambda: ops.insert3d(hm, d, c, q, t, off, w, px, method="binned"),
                                    3, st) * 1e3
    res["tiled_ms"] = timed_events(lambda: ops.insert3d(hm, d, c, q, t, off, w, px, method="tiled"),
                                   3, st) * 1e3
    res["direct_ms"] = timed_events(lambda: ops.insert3d(hm, d, c, q, t, off, w, px, tiled=False),
                                    2, st) * 1e3
    # the records of this launch
    ws = ops.workspace(lib().thx_insert3d_workspace(n, a.mreco, len(px.order)), dev)
    lib().thx_insert3d_tiled(ops._ptr(hm.F), ops._ptr(hm.T), ops._ptr(hm.O), ops._ptr(hm.counter),
                             hm.vdim, pf, ops._ptr(d), ops._ptr(c), ops._ptr(q), ops._ptr(t),
                             ops._ptr(off), ops._ptr(w), None, n, a.mreco, ops._ptr(px.d_iCol),
                             ops._ptr(px.d_iRow), ops._ptr(px.d_order), len(px.order), px.n,
                             px.idim, ops._ptr(ws), ws.numel(), ops._stream(dev))
    torch.cuda.synchronize()
    nC = len(px.order) // KC
    nRT = (a.mreco + RT - 1) // RT
    rec = ws.view(torch.int32)[:n * nRT * nC * REC].view(-1, REC).cpu().numpy().astype(np.int64)
    nx, sp, ny, nv0, tot = rec[:, 6], rec[:, 7], rec[:, 8], rec[:, 9], rec[:, 10]
    nv1 = tot - nv0
    sides = (nv0 > 0).astype(int) + (nv1 > 0)
    nz = np.maximum(nv0, nv1) // np.maximum(sp, 1)
    zc = np.where(sides > 0, np.minimum(nz, INS_CAP // np.maximum(sp * np.maximum(sides, 1), 1)), 0)
    scatter = zc == 0
    one = (~scatter) & (nz <= zc)
    chunks = np.where(scatter, 0, -(-nz // np.maximum(zc, 1)))
    res["workgroups"] = int(len(rec))
    res["frac_one_pass"] = float(one.mean())
    res["frac_zchunked"] = float(((~scatter) & ~one).mean())
    res["frac_direct_scatter"] = float(scatter.mean())
    res["mean_chunks_when_chunked"] = float(chunks[(~scatter) & ~one].mean()) if ((~scatter) & ~one).any() else 0
    res["box_voxels_p10_p50_p90_p99"] = [int(v) for v in np.percentile(tot, [10, 50, 90, 99])]
    res["flush_voxels_upper_GB"] = float(tot[~scatter].sum() * 12 / 1e9)
    res["direct_scatter_samplepx"] = int(scatter.sum() * KC * a.mreco)
    qs = q.cpu().numpy()
    uniq = np.array([len(np.unique(qs[l], axis=0)) for l in range(n)])
    res["distinct_rotations_per_image_p10_p50_p90"] = [int(v) for v in np.percentile(uniq, [10, 50, 90])]
    res["box_dims_median_nx_ny_nz"] = [int(np.median(nx)), int(np.median(ny)), int(np.median(nz))]
    for name in a.libs:
        L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                     "thunder_amd", "ab", f"lib_{name}.so"))

        fn = L.thx_insert3d_tiled
        fn.restype, fn.argtypes = SIGNATURES["thx_insert3d_tiled"]
        P = ops._ptr

        def run():
            fn(P(hm.F), P(hm.T), P(hm.O), P(hm.counter), hm.vdim, pf, P(d), P(c), P(q), P(t), P(off),
               P(w), None, n, a.mreco, P(px.d_iCol), P(px.d_iRow), P(px.d_order), len(px.order),
               px.n, px.idim, P(ws), ws.numel(), None)
        res[f"tiled_ms_{name}"] = timed_events(run, 3, st) * 1e3
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
