"""One-process-per-GPU sharded Preconditioning over torch.distributed (RCCL).

Rank g owns a Morton range of level-0 blocks (include/mas_capi.h, mas_shard_*).
Per apply the only exchange is one allgather of the padded level-1 residual
segments (~64 KB per rank at 1M over xGMI); every rank writes z for its own
vertices.  The r vector is replicated on every rank (the caller's layout);
z is owner-computes.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class ShardedApply:
    def __init__(self, P, rank: int, world: int, group=None, device=None):
        self.P, self.rank, self.world, self.group = P, rank, world, group
        self.plan = P.shard_setup(rank, world)
        seg = self.plan["seg_max"]
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.seg = torch.zeros((seg, 4), dtype=torch.float32, device=dev)
        self.gathered = torch.zeros((world * seg, 4), dtype=torch.float32, device=dev)
        self.graph = None
        self.graph_args = None

    def _step(self, z, r, s):
        self.P.shard_restrict(self.rank, self.world, r, self.seg, s.cuda_stream)
        with torch.cuda.stream(s):
            if self.world == 1:
                self.gathered.copy_(self.seg)
            elif dist.get_backend(self.group) == "gloo":  # test path: CPU staging
                g = torch.empty((self.gathered.shape[0], 4), dtype=torch.float32)
                dist.all_gather_into_tensor(g, self.seg.cpu(), group=self.group)
                self.gathered.copy_(g)
            else:  # RCCL over xGMI
                dist.all_gather_into_tensor(self.gathered, self.seg, group=self.group)
        self.P.shard_finish(self.rank, self.world, self.gathered, r, z, s.cuda_stream)

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
            self._step(z, r, stream)
        torch.cuda.synchronize()
        self.graph, self.graph_args = g, (z.data_ptr(), r.data_ptr())

    def __call__(self, z, r, stream=None):
        """z, r: torch cuda float32 [nV, 4]; runs on `stream` (torch.cuda.Stream) or the current stream."""
        s = stream if stream is not None else torch.cuda.current_stream()
        if self.graph is not None and self.graph_args == (z.data_ptr(), r.data_ptr()):
            self.graph.replay()
        else:
            self._step(z, r, s)
