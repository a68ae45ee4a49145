#!/usr/bin/env python3
"""Is a two-half phase pipeline worth building?  Times the particle-filter
phase loop alone (a local search: no scan, no reseed) at the bench's shape,
starting from the bench's post-scan clouds:

  full  -- one call over all images (the production shape),
  seq   -- two calls over the two halves, one after the other,
  conc  -- the two half calls on two HIP streams from two host threads, so
           each half's particle-filter chain can run under the other half's
           local kernel.

conc < full says the overlap pays; one JSON line per (case, rep).
    python tools/half_probe.py [--images 12500] [--phases 10] [--reps 3]"""
import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from thunder_amd import expectation as ex  # noqa: E402
from thunder_amd import ops, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=12500)
    ap.add_argument("--phases", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    N, pf, rU, rL = 256, 2, 24, 1
    vol = synth.projectee(synth.blob_volume(N, seed=1, device=dev), pf)
    _, nR, nT = ops.global_sample_sizes(2000)
    gset = tuple(x.cpu().numpy() for x in ops.global_sample_set(nR, nT, 10.0, 2, dev))
    px, dat, ctf, sig, _, _ = bench.make_stack(N, pf, rU, rL, a.images, dev, vol=vol)
    eg = ex.Expectation(vol, px, gset, n_phase=1, seed=11)
    start = [t.clone() for t in eg.run(dat, ctf, sig)[:4]]
    el = ex.Expectation(vol, px, None, n_phase=a.phases, search="local", seed=11)
    n, h = a.images, a.images // 2
    halves = ((0, h), (h, n))
    streams = [torch.cuda.Stream(dev) for _ in halves]

    def fresh():
        return [t.clone() for t in start]

    def run(st, l0, l1):
        el.run(dat[l0:l1], ctf[l0:l1], sig[l0:l1], state=[t[l0:l1] for t in st])

    def conc(st):
        cur = torch.cuda.current_stream(dev)
        for s in streams:
            s.wait_stream(cur)

        def go(k):
            with torch.cuda.stream(streams[k]):
                run(st, *halves[k])
        th = [threading.Thread(target=go, args=(k,)) for k in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for s in streams:
            cur.wait_stream(s)

    cases = {"full": lambda st: run(st, 0, n),
             "seq": lambda st: [run(st, l0, l1) for l0, l1 in halves],
             "conc": conc}
    ref = None
    for rep in range(a.reps + 1):
        for name, f in cases.items():
            st = fresh()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f(st)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            same = None       # the half calls draw per call-local image index
            if name == "seq":
                ref = st
            elif name == "conc" and ref is not None:
                same = all(torch.equal(x, y) for x, y in zip(st, ref))
            if rep:        # rep 0 warms up
                print(json.dumps({"case": name, "rep": rep, "images": n, "phases": a.phases,
                                  "ms": round(ms, 3), "conc_same_as_seq": same}), flush=True)


if __name__ == "__main__":
    main()
