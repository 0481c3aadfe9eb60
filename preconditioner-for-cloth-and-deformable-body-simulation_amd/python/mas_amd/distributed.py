"""One-process-per-GPU sharded Preconditioning (RCCL over xGMI).

Rank g owns a Morton range of level-0 blocks (include/mas_capi.h, mas_shard_*).
Per apply the only exchange is one allgather of the padded level-1 residual
segments (~64 KB per rank at 1M); every rank writes z for its own vertices.
The r vector is replicated on every rank (the caller's layout); z is
owner-computes.

Every apply is ONE library call per rank, the same entry point a C/C++
simulator uses (mas_shard_apply_device / mas_shard_apply_rccl): the library
restricts the rank's level-1 segment, runs the allgather on its own
communication stream while the rank's level-0 block solves run on the apply
stream, then the coarse levels and the prolongation.  The collective is
either
  * transport="torch": an allgather hook the library calls, issued through
    torch.distributed on `group` (nccl = RCCL; gloo stages through the host,
    for CPU-side tests of the protocol), or
  * transport="rccl": the handle's own RCCL communicator (mas_rccl_init), its
    unique id broadcast over `group` once.
Both are bitwise equal to the unsharded apply on the union of the ranks'
vertices.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class _DeviceArray:
    """A raw device pointer as a torch view (__cuda_array_interface__, no copy)."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 2,
                                         "strides": None}


def device_view(ptr: int, n: int, device) -> torch.Tensor:
    return torch.as_tensor(_DeviceArray(ptr, n), device=device)


def exchange_coarse_rows(P, group=None, device=None) -> bool:
    """The second half of a sharded Prepare (include/mas_capi.h ABI 5): one
    allgather of every rank's coarse-row segment over `group` (nccl = RCCL;
    gloo stages through the host), then mas_prepare_shard_complete.  Every
    rank calls it after its Prepare; returns False when nothing was pending
    (unsharded, or the exchange ran inside Prepare over the handle's RCCL
    communicator)."""
    seg = P.prepare_shard_rows() if P.rows_pending else None
    if seg is None:
        return False
    ptr, nbytes = seg
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    world = dist.get_world_size(group)
    n = nbytes // 4
    src = device_view(ptr, n, dev)
    if dist.get_backend(group) == "gloo":
        torch.cuda.synchronize(dev)
        g = torch.empty(n * world, dtype=torch.float32)
        dist.all_gather_into_tensor(g, src.cpu(), group=group)
        gathered = g.to(dev)
    else:
        gathered = torch.empty(n * world, dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(gathered, src, group=group)
    P.prepare_shard_complete(gathered, torch.cuda.current_stream(dev).cuda_stream)
    return True


class ShardedApply:
    def __init__(self, P, rank: int, world: int, group=None, device=None, overlap=None, transport="torch"):
        self.P, self.rank, self.world, self.group = P, rank, world, group
        self.overlap = world > 1  # the library overlaps the level-0 solves with the gather when there is one
        self.plan = P.shard_setup(rank, world)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.transport = transport
        self.backend = dist.get_backend(group) if (world > 1 or dist.is_initialized()) else None
        if transport == "rccl":
            import mas_amd
            uid = [mas_amd.rccl_unique_id() if rank == 0 else None]
            if world > 1:  # the 128-byte id travels over the existing group once
                dist.broadcast_object_list(uid, src=0, group=group)
            P.rccl_init(uid[0], rank, world)
        elif transport != "torch":
            raise ValueError(f"transport must be 'torch' or 'rccl', not {transport!r}")
        seg = self.plan["seg_max"]
        # explicit-step buffers (graph capture only)
        self.seg = torch.zeros((seg, 4), dtype=torch.float32, device=self.device)
        self.gathered = torch.zeros((world * seg, 4), dtype=torch.float32, device=self.device)
        self.graph = None
        self.graph_args = None

    # -- the allgather hook the library calls (transport="torch") --
    def _hook(self, send, recv, nbytes, strm):
        n = nbytes // 4
        with torch.cuda.stream(torch.cuda.ExternalStream(strm, device=self.device)):
            src = device_view(send, n, self.device)
            dst = device_view(recv, n * self.world, self.device)
            if self.world == 1:
                dst.copy_(src)
            elif self.backend == "gloo":  # protocol tests: stage through the host
                torch.cuda.current_stream().synchronize()
                g = torch.empty(n * self.world, dtype=torch.float32)
                dist.all_gather_into_tensor(g, src.cpu(), group=self.group)
                dst.copy_(g)
            else:  # RCCL over xGMI, ordered on the library's communication stream
                dist.all_gather_into_tensor(dst, src, group=self.group)

    def _call(self, z, r, s):
        if self.P.rows_pending:  # the first apply after a sharded Prepare: its coarse-row exchange first
            exchange_coarse_rows(self.P, self.group, self.device)
        if self.transport == "rccl":
            self.P.shard_apply_rccl(z, r, s.cuda_stream)
        else:
            self.P.shard_apply(self.rank, self.world, z, r, allgather=self._hook, stream=s.cuda_stream)

    def _step_explicit(self, z, r, s):
        """The same apply from the step-wise entry points (restrict, gather, finish)."""
        self.P.shard_restrict(self.rank, self.world, r, self.seg, s.cuda_stream)
        with torch.cuda.stream(s):
            if self.world == 1:
                self.gathered.copy_(self.seg)
            else:
                dist.all_gather_into_tensor(self.gathered, self.seg, group=self.group)
        self.P.shard_finish(self.rank, self.world, self.gathered, r, z, s.cuda_stream)

    def capture(self, z, r, stream):
        """Record one apply as a HIP graph: later calls with the same z, r
        replay it (removes the per-kernel host launch cost).  The rccl
        transport captures the one-call apply itself (the gather on the
        library's communication stream, forked and joined inside the graph);
        the torch transport captures the step-wise form.  Call after at least
        one eager apply (buffers and tables exist by then)."""
        if self.world > 1 and self.backend == "gloo":
            raise RuntimeError("graph capture needs the nccl (RCCL) backend")
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            if self.transport == "rccl":
                self._call(z, r, stream)
            else:
                self._step_explicit(z, r, stream)
        torch.cuda.synchronize()
        self.graph, self.graph_args = g, (z.data_ptr(), r.data_ptr())

    def __call__(self, z, r, stream=None):
        """z, r: torch cuda float32 [nV, 4]; runs on `stream` (torch.cuda.Stream) or the current stream."""
        s = stream if stream is not None else torch.cuda.current_stream()
        if self.graph is not None and self.graph_args == (z.data_ptr(), r.data_ptr()):
            self.graph.replay()
        else:
            self._call(z, r, s)
