"""Time thx_reconstruct on one 512^3-padded half-map (box 256, pf 2) and dump
what an A/B of two builds compares: iterations, the balancing diffs, and the
map's central 64^3 (float32 .npy under gpurun_out/).
    THX_LIB=... python tools/recon_time.py TAG
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from thunder_amd import ops, synth  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "prod"
N, pf = int(os.environ.get("RT_N", 256)), 2
vdim = N * pf
dev = torch.device("cuda", 0)
vol = synth.projectee(synth.blob_volume(N, n_blobs=12, seed=3, device=dev), pf)
i = torch.arange(vdim // 2 + 1, device=dev, dtype=torch.float32)
j = torch.fft.fftfreq(vdim, 1.0 / vdim, device=dev).float()
quad = j[:, None, None] ** 2 + j[None, :, None] ** 2 + i[None, None, :] ** 2
g = torch.Generator(device=dev).manual_seed(5)
T0 = (50.0 / (1.0 + quad.sqrt())) * (0.8 + 0.4 * torch.rand(quad.shape, generator=g, device=dev))
F0 = vol * T0
res = {"tag": tag, "ms": []}
for rep in range(4):
    hm = ops.HalfMap(vdim, dev)
    hm.F.copy_(F0)
    hm.T.copy_(T0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    dst, _, it, diffs = ops.reconstruct(hm, N, pf, want_ft=False)
    torch.cuda.synchronize()
    res["ms"].append((time.perf_counter() - t) * 1e3)
res["iterations"] = it
res["diffs"] = diffs
c = N // 2
box = dst.cpu().numpy()
res["max_abs"] = float(np.abs(box).max())
out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", f"recon_{tag}.npy")
np.save(out, np.fft.fftshift(box)[c - 32:c + 32, c - 32:c + 32, c - 32:c + 32].astype(np.float32))
print(res)
