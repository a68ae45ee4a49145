"""world_size-2 gloo checks of the multi-GPU plumbing on CPU.

The expectation path shards particles with no collective (weak scaling); the
only exchange is the per-hemisphere half-map sum at the end of a round
(ncclAllReduce of F/T/O/counter, gpu/src/cuthunder.cu:5903-5993), done here
by thunder_amd.expectation.halfmap_allreduce over the hemisphere group.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class CpuHalfMap:
    def __init__(self, vdim, seed):
        g = torch.Generator().manual_seed(seed)
        self.F = torch.complex(torch.randn(vdim, vdim, vdim // 2 + 1, generator=g),
                               torch.randn(vdim, vdim, vdim // 2 + 1, generator=g))
        self.T = torch.rand(vdim, vdim, vdim // 2 + 1, generator=g)
        self.O = torch.randn(3, dtype=torch.float64, generator=g)
        self.counter = torch.tensor([7 + seed], dtype=torch.int32)


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from thunder_amd.expectation import halfmap_allreduce, hemisphere_groups, hemisphere_shard
    hm = CpuHalfMap(8, seed=rank)
    # hemisphere groups: every rank creates both (collective), uses its own
    groups = hemisphere_groups(world)
    halfmap_allreduce(hm, group=groups[rank % 2])
    full = CpuHalfMap(8, seed=rank)
    dist.all_reduce(full.T)          # world-wide reference sum
    out[rank] = (hm.F.clone(), hm.T.clone(), hm.O.clone(), int(hm.counter.item()),
                 full.T.clone(), list(hemisphere_shard(100, world, rank)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_halfmap_allreduce_per_hemisphere(world):
    port = free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    for rank in range(world):
        F, T, O, c, Tall, idx = out[rank]
        members = [r for r in range(world) if r % 2 == rank % 2]
        refs = [CpuHalfMap(8, seed=r) for r in members]
        assert torch.allclose(F, sum(h.F for h in refs), atol=1e-5)
        assert torch.allclose(T, sum(h.T for h in refs), atol=1e-5)
        assert torch.allclose(O, sum(h.O for h in refs))
        assert c == sum(int(h.counter.item()) for h in refs)
        assert torch.allclose(Tall, sum(CpuHalfMap(8, seed=r).T for r in range(world)), atol=1e-5)
    # the shards cover every image once, hemispheres alternate
    allidx = sorted(i for r in range(world) for i in out[r][5])
    assert allidx == list(range(100))
    for r in range(world):
        assert all(i % 2 == r % 2 for i in out[r][5])
