"""Steady-state Prepare of the ranks of a sharded world (mas_set_prepare_shard),
one handle per rank on one GPU, against the unsharded Prepare.  A rank's
Prepare is mas_prepare (its own coarse rows, ABI 5) + the coarse-row
allgather -- replaced here by a local copy of its own segment into a zeroed
gathered buffer (the communication is NOT in these numbers) -- +
mas_prepare_shard_complete (unpack, factor the shared blocks).
python scripts/dev/prep_shard.py [config] [world] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                "../../preconditioner-for-cloth-and-deformable-body-simulation_amd/python"))

import torch
import mas_amd
from mas_amd import meshgen
from mas_amd.distributed import device_view

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "1M+contacts"
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
mesh, cfg = meshgen.build_config(cfg_name)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None


def prep(P, rank=0, world=1):
    if contacts is None:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    else:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, contacts[0], None, None, contacts[1])
    st = P.stats()
    st["complete_ms"] = 0.0
    seg = P.prepare_shard_rows() if P.rows_pending else None
    if seg is not None:
        ptr, nbytes = seg
        n = nbytes // 4
        gathered = torch.zeros(world * n, dtype=torch.float32, device="cuda")
        gathered[rank * n:(rank + 1) * n].copy_(device_view(ptr, n, gathered.device))
        torch.cuda.synchronize()
        P.prepare_shard_complete(gathered)
        st["complete_ms"] = P.stats()["prepare_complete_ms"]
        st["seg_bytes"] = nbytes
    st["rank_ms"] = st["prepare_ms"] + st["complete_ms"]
    return st


def line(tag, st):
    return (f"{tag}: prepare {st['prepare_ms']:.3f} ms (levels {st['prepare_levels_ms']:.3f}, assemble "
            f"{st['prepare_assemble_ms']:.3f}, factor {st['prepare_factor_ms']:.3f}, "
            f"fused level-0 {st['prepare_fine_ms']:.3f} from {st['prepare_fine_start_ms']:.3f}, "
            f"hier rebuilt {st['hier_rebuilt']}, coarse split {st['coarse_split']}) + complete "
            f"{st['complete_ms']:.3f} ms = {st['rank_ms']:.3f} ms" + (f", segment {st['seg_bytes']} B" if 'seg_bytes' in st else ""))


# one handle at a time (created, measured, destroyed): every handle owns two
# or three HIP streams, and with more streams alive than GPU_MAX_HW_QUEUES
# (4) they share hardware queues, which would serialise a Prepare's overlap
tags = ["unsharded"] + [f"rank {g}/{world}" for g in range(world)]
best = {}
for i, tag in enumerate(tags):
    P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts,
                          shard=None if i == 0 else (i - 1, world))
    for _ in range(reps):
        st = prep(P, max(i - 1, 0), world if i else 1)
        if tag not in best or st["rank_ms"] < best[tag]["rank_ms"]:
            best[tag] = st
    del P
    print(line(tag, best[tag]), flush=True)
slow = max(best[t]["rank_ms"] for t in tags[1:])
print(f"{cfg_name} world {world}: slowest rank {slow:.3f} ms (Prepare + complete, allgather excluded) = "
      f"{slow / best['unsharded']['prepare_ms']:.3f} x unsharded")
