"""The end of a round across ranks: the gold-standard hemispheres' half-map
reduction, reconstruction on each hemisphere's lead, the hand-over of
hemisphere B's map to hemisphere A's lead and the FSC there.

Mirrors the reference's round end: Reconstructor::allReduceF/T/O and the
NCCL all-reduce inside cuthunder::InsertFT (src/Reconstructor.cpp:2350-2520,
gpu/src/cuthunder.cu:5903-5993) per hemisphere, then
Model::compareTwoHemispheres (src/Model.cpp:307-852: the master receives
hemisphere A's and B's maps with MPI_Recv_Large and calls FSC,
src/Functions/Spectrum.cpp:302-337).  Here rank 0 leads hemisphere A and
computes the FSC; rank 1 leads hemisphere B (hemisphere = rank % 2,
src/Parallel.cpp:26-53).

Two transports, one code path: "rccl" (device tensors, the C-ABI's
thx_halfmap_allreduce / thx_halfmap_sendrecv over xGMI) and "torch"
(torch.distributed on whatever backend the process group has -- gloo with CPU
tensors in the CPU tests, or a one-GPU rehearsal of several ranks).  The
reconstruction and FSC are passed in, so the CPU tests can plug the float64
restatement (oracle/reconstruct.py) where the GPU run uses thx_reconstruct /
thx_fsc.
"""
import torch

from . import ops


def hemisphere(rank):
    """0 = hemisphere A (even ranks), 1 = B (odd ranks)."""
    return rank % 2


def leads(world):
    """(A lead, B lead): the first rank of each hemisphere."""
    return (0, 1) if world > 1 else (0, 0)


class RoundEnd:
    """Collective set-up of the groups / communicators a round end needs.
    Every rank of the job constructs it (torch.distributed.new_group is
    collective)."""

    def __init__(self, world, rank, transport="rccl", device=None):
        import torch.distributed as dist
        if transport not in ("rccl", "torch"):
            raise ValueError("transport: 'rccl' or 'torch'")
        self.world, self.rank, self.transport = world, rank, transport
        self.device = device
        # (world 1: hemisphere B has no rank, and no group)
        self.hemi_groups = [dist.new_group([r for r in range(world) if r % 2 == h])
                            if h < world else None for h in (0, 1)]
        self.lead_group = dist.new_group(list(leads(world))) if world > 1 else None
        self.hemi_comm = self.lead_comm = None
        if transport == "rccl":
            self.hemi_comm = ops.RcclComm.from_group(self.hemi_groups[hemisphere(rank)], device)
            if self.lead_group is not None and rank in leads(world):
                self.lead_comm = ops.RcclComm.from_group(self.lead_group, device)

    @property
    def is_lead(self):
        return self.rank in leads(self.world)

    def reduce(self, hm):
        """a13: the sum of F, T, O, counter over this rank's hemisphere, in place."""
        import torch.distributed as dist
        if self.transport == "rccl":
            if self.hemi_comm.nranks > 1:
                self.hemi_comm.allreduce(hm)
            return hm
        g = self.hemi_groups[hemisphere(self.rank)]
        if dist.get_world_size(g) > 1:
            for t in (hm.F, hm.T, hm.O, hm.counter):
                h = self._staged(t)
                dist.all_reduce(h, op=dist.ReduceOp.SUM, group=g)
                if h is not t:
                    t.copy_(h)
        return hm

    @staticmethod
    def _staged(t):
        """gloo moves host tensors: device tensors go through a host copy."""
        import torch.distributed as dist
        return t.cpu() if t.is_cuda and dist.get_backend() == "gloo" else t

    def exchange(self, mine):
        """The leads' hand-over: hemisphere B's lead sends `mine` (its
        reconstructed map, any float / complex tensor) to hemisphere A's lead,
        which returns (A, B); the B lead returns None; other ranks must not
        call it.  One rank holds both hemispheres when world == 1."""
        import torch.distributed as dist
        a, b = leads(self.world)
        if self.world == 1:
            raise ValueError("world 1: both hemispheres are local, nothing to exchange")
        if self.rank not in (a, b):
            raise ValueError("exchange: only the hemisphere leads take part")
        buf = mine.contiguous()
        if self.transport == "rccl":
            f = torch.view_as_real(buf) if buf.is_complex() else buf
            if f.dtype != torch.float32:
                raise TypeError("rccl exchange moves float32 / complex64 maps")
            n = f.numel()
            if self.rank == b:
                self.lead_comm.sendrecv(send=f, peer_send=0)
                return None
            other = torch.empty_like(buf)
            o = torch.view_as_real(other) if other.is_complex() else other
            self.lead_comm.sendrecv(recv=o, peer_recv=1, n_recv=n)
            return buf, other
        if self.rank == b:
            dist.send(self._staged(buf), dst=a)
            return None
        other = self._staged(torch.empty_like(buf))
        dist.recv(other, src=b)
        return buf, other.to(buf.device)

    def close(self):
        for c in (self.hemi_comm, self.lead_comm):
            if c is not None:
                c.close()


def round_end(hm, re, reconstruct, fsc):
    """Reduce this rank's half-map over its hemisphere, reconstruct on the
    hemisphere leads, hand B's map to A's lead; returns the FSC on rank 0
    (None elsewhere).  reconstruct(hm) -> map (Fourier, half-complex);
    fsc(A, B) -> per-shell FSC."""
    re.reduce(hm)
    if not re.is_lead:
        return None
    mine = reconstruct(hm)
    got = re.exchange(mine)
    if got is None:
        return None
    return fsc(*got)
