"""One-process-per-GPU sharded Preconditioning over torch.distributed (RCCL).

Rank g owns a Morton range of level-0 blocks (include/mas_capi.h, mas_shard_*).
Per apply the only exchange is one allgather of the padded level-1 residual
segments (~64 KB per rank at 1M over xGMI); every rank writes z for its own
vertices.  The r vector is replicated on every rank (the caller's layout);
z is owner-computes.

Overlap (default with RCCL): the allgather is started asynchronously (it runs
on the process group's own stream once the restrict is done), the rank's
level-0 block solves (z = Z0) are enqueued behind it on the apply stream, and
only then does the apply stream wait for the allgather and run the coarse
levels + prolongation (mas_apply_shard_fine / _complete).  The level-0 work
(~15 us per rank at N = 8, 1M) thus hides the collective's latency instead of
following it.  Bitwise equal to the serial form.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class ShardedApply:
    def __init__(self, P, rank: int, world: int, group=None, device=None, overlap=None):
        self.P, self.rank, self.world, self.group = P, rank, world, group
        # one rank has no collective to hide: the serial form saves the prolongation pass
        self.overlap = world > 1 if overlap is None else bool(overlap)
        self.plan = P.shard_setup(rank, world)
        seg = self.plan["seg_max"]
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.seg = torch.zeros((seg, 4), dtype=torch.float32, device=dev)
        self.gathered = torch.zeros((world * seg, 4), dtype=torch.float32, device=dev)
        self.graph = None
        self.graph_args = None

    def _gather(self, s, async_op):
        """Allgather of the level-1 segments on stream s; returns the pending work (RCCL, async) or None."""
        with torch.cuda.stream(s):
            if self.world == 1:
                self.gathered.copy_(self.seg)
            elif dist.get_backend(self.group) == "gloo":  # test path: CPU staging
                g = torch.empty((self.gathered.shape[0], 4), dtype=torch.float32)
                dist.all_gather_into_tensor(g, self.seg.cpu(), group=self.group)
                self.gathered.copy_(g)
            else:  # RCCL over xGMI
                return dist.all_gather_into_tensor(self.gathered, self.seg, group=self.group, async_op=async_op)
        return None

    def _step(self, z, r, s, overlap=None):
        overlap = self.overlap if overlap is None else overlap
        self.P.shard_restrict(self.rank, self.world, r, self.seg, s.cuda_stream)
        if not overlap:
            self._gather(s, async_op=False)
            self.P.shard_finish(self.rank, self.world, self.gathered, r, z, s.cuda_stream)
            return
        work = self._gather(s, async_op=True)
        self.P.shard_fine(self.rank, self.world, r, z, s.cuda_stream)   # runs while the allgather is in flight
        if work is not None:
            with torch.cuda.stream(s):
                work.wait()                                             # the apply stream waits for the collective
        self.P.shard_complete(self.rank, self.world, self.gathered, z, s.cuda_stream)

    def capture(self, z, r, stream):
        """Record one apply (restrict, RCCL allgather, finish) as a HIP graph:
        later calls with the same z, r replay it, which removes the per-kernel
        host launch cost that dominates once the per-rank work is ~50 us.
        Call after at least one eager apply (lazy communicator / table setup)."""
        if self.world > 1 and dist.get_backend(self.group) == "gloo":
            raise RuntimeError("graph capture needs the nccl (RCCL) backend")
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            self._step(z, r, stream, overlap=False)
        torch.cuda.synchronize()
        self.graph, self.graph_args = g, (z.data_ptr(), r.data_ptr())

    def __call__(self, z, r, stream=None):
        """z, r: torch cuda float32 [nV, 4]; runs on `stream` (torch.cuda.Stream) or the current stream."""
        s = stream if stream is not None else torch.cuda.current_stream()
        if self.graph is not None and self.graph_args == (z.data_ptr(), r.data_ptr()):
            self.graph.replay()
        else:
            self._step(z, r, s)
