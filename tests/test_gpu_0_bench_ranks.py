"""The N > 1 bench path, rehearsed on one GPU: bench.py --gpus 2 under
torch.distributed.run with THX_BENCH_BACKEND=gloo for the bench's own
collectives (timing max, RCCL unique-id broadcast), both ranks on device 0,
the hemisphere round end through thx_halfmap_allreduce / thx_halfmap_sendrecv
on one-rank RCCL communicators (thunder_amd/hemisphere.py).  It is the driver's
8-GPU SCALE command on a tiny configuration.

This file sorts first among the GPU tests: the ranks are started before this
pytest process touches the GPU (a process that has initialised the GPU must
not start programs here), and the test skips if something already did."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_rehearsal():
    import torch
    if torch.cuda.is_initialized():
        pytest.skip("this process already initialised the GPU; run the file on its own")
    env = dict(os.environ, THX_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29517", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--box", "128", "--nr", "500",
           "--images", "256", "--phases", "2", "--no-cpu-baseline", "--no-rooflines"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["scaling"] == "weak"
    assert "allreduce_ms" in d and d["allreduce_ranks_per_hemisphere"] == 1
    assert d["allreduce_transport"] in ("rccl", "torch")
    assert "reconstructed_fsc_shells_4_16_32_64" in d
