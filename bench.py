#!/usr/bin/env python3
"""Headline benchmark: particle-images/s through expectation (box 256, 2000
rotation samples), BASELINE.json metric, on N GPUs of one node.

One step = the expectation of one batch of synthetic particle images per GPU,
inputs resident in HBM: global scan over nR = 2000 rotations x nT = 151
translations at the global-search radius (rU = 24, nPxl = 870), reseed, then
10 particle-filter phases (mLR = 125, mLT = 9) -- SURVEY.md §8(d).  Weak
scaling: every rank owns its own batch (gold-standard hemisphere = rank % 2),
no collective on the expectation path.  Insert (mReco = 100) and the RCCL
half-map all-reduce are timed separately and reported as extra fields.

Launch: python bench.py [--gpus 1 --steps K --warmup W]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402
from thunder_amd._lib import lib  # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3    # MI355X_MICROARCH.md, dense f32 MFMA (= VALU)
PEAK_HBM_GBS = 8000.0            # MI355X_MICROARCH.md, HBM3E spec
PEAK_BF16_MFMA_TFLOPS = 2500.0   # MI355X_MICROARCH.md, dense bf16 MFMA
ROOF_IMAGES = 4096               # images per global-scan launch in the roofline measurement


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--images", type=int, default=12500, help="particle images per GPU per step")
    p.add_argument("--chunk", type=int, default=0,
                   help="images per expectation launch (0: the whole batch in one launch; "
                        "288 GB of HBM holds the workspaces of all 12500)")
    p.add_argument("--box", type=int, default=256)
    p.add_argument("--nr", type=int, default=2000)
    p.add_argument("--phases", type=int, default=10)
    p.add_argument("--algo", type=int, default=2,
                   help="global-scan algorithm: 0 direct, 1 FP32 MFMA, 2 bf16x3 MFMA")
    p.add_argument("--shuffle", type=int, default=1,
                   help="1: shuffle the support before resampling (Particle::resample)")
    p.add_argument("--perturb-mean", default="acg", choices=["acg", "top"],
                   help="acg: inferACG mean of the cloud (the reference's compiled switch "
                        "PARTICLE_ROT_MEAN_USING_STAT_PERTURB); top: the top particle")
    p.add_argument("--acg-iters", type=int, default=100, help="inferACG fixed-point iteration cap")
    p.add_argument("--large-first", type=int, default=0,
                   help="1: OPTIMISER_GLOBAL_PERTURB_LARGE (off in the reference's Config.h)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-extras", action="store_true", help="skip insert / all-reduce / local roofline")
    return p.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def make_stack(N, pf, rU, rL, n_img, device, seed=5, snr=0.05, vol=None):
    """Synthetic images: ctf * shift(t_true) * P_Rtrue(vol) + noise."""
    px = ops.PixelSet(N, pf, rU, rL, device=device)
    rng = np.random.default_rng(seed)
    qtrue = torch.as_tensor(synth.uniform_quaternions(n_img, rng), device=device)
    ttrue = torch.as_tensor(rng.standard_normal((n_img, 2)) * 3.0, device=device)
    attrs = torch.as_tensor(synth.ctf_attrs(n_img, seed=seed + 1), device=device)
    ctf = ops.ctf(attrs, px)
    sig = torch.empty(n_img, px.n, dtype=torch.complex64, device=device)
    for l0 in range(0, n_img, 8192):
        l1 = min(n_img, l0 + 8192)
        P = ops.project3d(vol, ops.rotmat(qtrue[l0:l1].contiguous()), px)
        Tt = ops.trans_table(ttrue[l0:l1].contiguous(), px)
        sig[l0:l1] = ctf[l0:l1] * P * Tt
    dat, sigRcp = synth.noisy_images(sig, px.iSig, N // 2 + 1, snr=snr, seed=seed + 2)
    return px, dat, ctf, sigRcp, qtrue, ttrue


def pmc_traffic():
    """HBM bytes per launch of the roofline launch sequences, measured by the
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench (tools/gpu_round.sh
    pmc -> tools/traffic.py -> profiles/rNN_traffic.json, the newest round)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")))
    if not files:
        return {}, None
    with open(files[-1]) as f:
        return json.load(f), os.path.relpath(files[-1], ROOT)


def timed_events(fn, reps, stream):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record(stream)
    for _ in range(reps):
        fn()
    e.record(stream)
    e.synchronize()
    return s.elapsed_time(e) / reps / 1e3


def scan_roofline(vol, px, gset, dat, ctf, sig, algo, reps=3):
    """Average duration of the global-scan launch sequence (HIP events on the
    launch stream) priced against the matrix-core roof of its dtype:
    algo 1 = FP32 MFMA (4 flop per image x rotation x translation x pixel),
    algo 2 = bf16 MFMA, three products per FP32 product (12 bf16 flop)."""
    dev = dat.device
    q, t, pR, pT = gset
    nImg, nR, nT = dat.shape[0], len(q), len(t)
    rotP = ops.project3d(vol, ops.rotmat(torch.as_tensor(q, device=dev)), px)
    traP = ops.trans_table(torch.as_tensor(t, device=dev), px)
    pRd, pTd = torch.as_tensor(pR, device=dev), torch.as_tensor(pT, device=dev)
    st = torch.cuda.current_stream(dev)
    sec = timed_events(lambda: ops.global_scan(rotP, traP, dat, ctf, sig, pRd, pTd, algo=algo),
                       reps, st)
    pad = lambda v, m: (v + m - 1) // m * m
    elems = float(pad(nImg, 64)) * pad(nR, 4) * pad(nT, 32) * pad(px.n, 16)
    issued = (12.0 if algo == 2 else 4.0) * elems
    peak = PEAK_BF16_MFMA_TFLOPS if algo == 2 else PEAK_FP32_MFMA_TFLOPS
    algorithmic = 15.0 * nImg * nR * nT * px.n      # SURVEY §8(d), direct formulation
    return sec, issued, algorithmic, peak


def local_roofline(vol, N, pf, device, n_img=512, reps=3):
    """Full-resolution particle-filter phase (nPxl = 24746 at box 256,
    mLR = 125, mLT = 9): HBM bytes 64 * mLR * nPxl + 16 * nPxl per image-phase."""
    rU = N // 2 - 2
    px, dat, ctf, sig, qtrue, ttrue = make_stack(N, pf, rU, 1, n_img, device, seed=17, vol=vol)
    rng = np.random.default_rng(3)
    mR, mT = 125, 9
    quat = torch.as_tensor(synth.uniform_quaternions(n_img * mR, rng).reshape(n_img, mR, 4),
                           device=device)
    trans = torch.as_tensor(rng.standard_normal((n_img, mT, 2)), device=device)
    pC = torch.ones(n_img, dtype=torch.float64, device=device)
    pR = torch.full((n_img, mR), 1.0 / mR, dtype=torch.float64, device=device)
    pT = torch.full((n_img, mT), 1.0 / mT, dtype=torch.float64, device=device)
    st = torch.cuda.current_stream(device)
    cells = ops.volume_cells(vol)
    sec = timed_events(lambda: ops.local_phase(vol, quat, trans, pC, pR, pT, dat, ctf, sig, px,
                                               cells=cells), reps, st)
    sec_plain = timed_events(lambda: ops.local_phase(vol, quat, trans, pC, pR, pT, dat, ctf, sig,
                                                     px), reps, st)
    del cells
    algo_bytes = n_img * (64.0 * mR * px.n + 16.0 * px.n)
    return sec, algo_bytes, px.n, sec_plain


def cpu_baseline(vol_np, N, pf, gset, dat, ctf, sig, px_host, seconds):
    """The C restatement (oracle/, OpenMP) on the host cores, same workload
    shape, bounded sample of images (test infrastructure as CPU baseline)."""
    from oracle import oracle as orc
    threads = min(16, os.cpu_count() or 1)
    q, t, pR, pT = gset
    vdim = pf * N
    rng = np.random.default_rng(0)

    def run(n):
        t0 = time.perf_counter()
        d = orc.dvp_global(vol_np, vdim, pf, q, t, dat[:n], ctf[:n], sig[:n], px_host, N,
                           threads=threads)
        orc.weights_global(d, pR, pT)
        # 10 local phases per image (125 x 9 samples), likelihood + marginals
        for l in range(n):
            for _ in range(10):
                lq = synth.uniform_quaternions(125, rng)
                lt = rng.standard_normal((9, 2))
                orc.local_phase(vol_np, vdim, pf, lq, lt, 1.0, np.full(125, 1 / 125),
                                np.full(9, 1 / 9), dat[l], ctf[l], sig[l], px_host, N)
        return time.perf_counter() - t0

    n = 2
    dt = run(n)
    n2 = max(2, min(len(dat), int(n * seconds / max(dt, 1e-3))))
    if n2 > n:
        dt = run(n2)
        n = n2
    return {"value": n / dt, "unit": "particle-images/s", "cores": threads, "kind": "port",
            "sample": f"{n} images x (global scan nR={len(q)} nT={len(t)} nPxl={px_host.n} + "
                      f"10 local phases 125x9), OpenMP {threads} threads, {dt:.1f} s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    lib()   # fail loudly if the HIP library is missing

    N, pf, rU, rL = a.box, 2, 24, 1
    log(rank, f"[bench] building synthetic volume N={N} pf={pf}")
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    gset = synth.global_sample_set(a.nr, seed=2)
    px, dat, ctf, sig, qtrue, ttrue = make_stack(N, pf, rU, rL, a.images, dev, seed=5 + 101 * rank,
                                                 vol=vol)
    e = ex.Expectation(vol, px, gset, n_phase=a.phases, algo=a.algo, seed=7 + rank,
                       shuffle=bool(a.shuffle), perturb_mean=a.perturb_mean, acg_iters=a.acg_iters,
                       large_first=bool(a.large_first))
    chunk = a.chunk or a.images
    chunks = [(l0, min(a.images, l0 + chunk)) for l0 in range(0, a.images, chunk)]
    outs = [None] * len(chunks)

    def step():
        for c, (l0, l1) in enumerate(chunks):
            outs[c] = e.run(dat[l0:l1], ctf[l0:l1], sig[l0:l1], out=outs[c])

    log(rank, f"[bench] nPxl={px.n} nR={a.nr} nT={len(gset[1])} images/gpu={a.images}")
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ms_per_step = el / a.steps * 1e3
    value = a.gpus * a.images * a.steps / el

    # accuracy sanity of the timed path: top rotation vs true pose
    res = {}
    if rank == 0:
        # (off-grid poses: a 2000-rotation grid at the 15 A scan resolution
        # leaves about half the modes in a wrong basin; tools/diag_expect.py)
        qa = outs[0][0]
        q0 = ex.cloud_mode(qa)
        qt = qtrue[:q0.shape[0]]
        cosang = (q0 * qt).sum(-1).abs().clamp(max=1)
        res["median_pose_error_deg"] = float(torch.rad2deg(2 * torch.acos(cosang)).median())
        # final particle-cloud spread: angle of every rotation sample to the cloud mode
        ca = (qa * q0[:, None, :]).sum(-1).abs().clamp(max=1)
        ang = torch.rad2deg(2 * torch.acos(ca))
        qs = torch.tensor([0.1, 0.5, 0.9], dtype=ang.dtype, device=ang.device)
        res["cloud_spread_deg"] = {
            "median_p10_p50_p90": [round(float(v), 2) for v in torch.quantile(ang.median(1).values, qs)],
            "max_p10_p50_p90": [round(float(v), 2) for v in torch.quantile(ang.max(1).values, qs)]}

    extras = {}
    traffic, traffic_src = pmc_traffic()

    def launch_traffic(key, ok):
        t = traffic.get(key) if ok else None
        return (t["traffic_bytes"], f"{traffic_src}: {key}") if t else (None, None)

    if not a.no_extras:
        # dominant kernel: the global scan
        nRoof = min(ROOF_IMAGES, a.images)
        sec, issued, algorithmic, peak = scan_roofline(vol, px, gset, dat[:nRoof],
                                                       ctf[:nRoof], sig[:nRoof], a.algo)
        kname = {1: "k_scan_mfma (fp32 32x32x2)", 2: "k_scan_split<BF16X3> (bf16 32x32x16, 3-product split)"}
        tr, tr_src = launch_traffic("scan_4096", a.algo == 2 and nRoof == 4096
                                    and a.nr == 2000 and N == 256)
        extras["roofline"] = {"bound": "mfma", "achieved": issued / sec / 1e12,
                              "peak": peak, "unit": "TFLOP/s",
                              "frac": issued / sec / 1e12 / peak, "traffic": tr,
                              "traffic_unit": "bytes per launch (HBM, PMC)", "traffic_source": tr_src,
                              "kernel": f"global scan {kname.get(a.algo, a.algo)} + prep + combine",
                              "launch_ms": sec * 1e3, "images_per_launch": nRoof,
                              "algorithmic_equiv_tflops": algorithmic / sec / 1e12,
                              "note": "achieved = issued matrix-core flops after the expansion of "
                                      "|d-cTP|^2 into a GEMM (4 fp32 flop, or 3x4 bf16 flop, per "
                                      "image x rotation x translation x pixel); "
                                      "algorithmic_equiv uses the direct 15-flop count of SURVEY "
                                      "8(d) and can exceed the FP32 VALU peak"}
        lsec, lbytes, lnpx, lsec_plain = local_roofline(vol, N, pf, dev)
        tr, tr_src = launch_traffic("local_fullres_512", N == 256)
        extras["roofline_local"] = {"bound": "hbm", "achieved": lbytes / lsec / 1e9,
                                    "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                    "frac": lbytes / lsec / 1e9 / PEAK_HBM_GBS, "traffic": tr,
                                    "traffic_unit": "bytes per launch (HBM, PMC)",
                                    "traffic_source": tr_src,
                                    "algorithmic_bytes": lbytes,
                                    "kernel": f"local phase full-res (nPxl={lnpx}, 125x9, 512 "
                                              "images, cell-expanded projectee)",
                                    "launch_ms": lsec * 1e3,
                                    "launch_ms_halfcomplex_layout": lsec_plain * 1e3}
        # insert (mReco = 100) + half-map all-reduce over the hemisphere
        rec = ex.Reconstructor(N, pf, dev)
        quat, trans = outs[0][0], outs[0][1]
        iq, it = ex.draw_insert_samples(quat, trans, 100)
        nI = iq.shape[0]
        offS = torch.zeros(nI, 2, dtype=torch.float64, device=dev)
        w = torch.full((nI,), 1.0 / 100, dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream(dev)
        isec = timed_events(lambda: rec.insert(dat[:nI], ctf[:nI], iq, it, offS, w, px), 2, st)
        extras["insert_images_per_s"] = a.gpus * nI / isec
        if dist:
            groups = [dist.new_group([r for r in range(world) if r % 2 == h]) for h in (0, 1)]
            g = groups[rank % 2]
            torch.cuda.synchronize()
            dist.barrier()
            t1 = time.perf_counter()
            ex.halfmap_allreduce(rec.hm, group=g)
            torch.cuda.synchronize()
            extras["allreduce_ms"] = (time.perf_counter() - t1) * 1e3
            extras["allreduce_bytes"] = (rec.hm.F.numel() * 8 + rec.hm.T.numel() * 4)
        else:
            extras["allreduce_ms"] = 0.0

    if rank == 0 and not a.no_cpu_baseline:
        vol_np = vol.cpu().numpy()
        n_cpu = 256
        from oracle import oracle as orc
        pxh = orc.pixel_set(N, pf, rU, rL)
        extras["cpu_baseline"] = cpu_baseline(vol_np, N, pf, gset, dat[:n_cpu].cpu().numpy(),
                                              ctf[:n_cpu].cpu().numpy(), sig[:n_cpu].cpu().numpy(),
                                              pxh, a.cpu_seconds)

    if rank == 0:
        line = {"metric": "particle-images/sec through expectation (box 256, 2000 rot samples)",
                "value": value, "unit": "particle-images/s", "n_gpus": a.gpus, "steps": a.steps,
                "warmup": a.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic (seeded Gaussian-blob volume, CTF-modulated noisy projections, SNR 0.05)",
                "config": {"workload": f"C3: 3D refine box {N}, {a.nr} rotation x {len(gset[1])} "
                                       f"translation global scan at rU={rU} (nPxl={px.n}) + "
                                       f"{a.phases} particle-filter phases (125 x 9)",
                           "images_per_gpu": a.images, "global_batch": a.images * a.gpus,
                           "box": N, "pf": pf, "nR": a.nr, "nT": len(gset[1]), "nPxl": px.n,
                           "parallelism": f"dp{a.gpus} (hemisphere = rank % 2)"},
                **res, **extras}
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
