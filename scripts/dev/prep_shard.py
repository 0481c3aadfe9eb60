"""Steady-state Prepare of the ranks of a sharded world (mas_set_prepare_shard),
one handle per rank on one GPU, against the unsharded Prepare.
python scripts/dev/prep_shard.py [config] [world] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                "../../preconditioner-for-cloth-and-deformable-body-simulation_amd/python"))

import mas_amd
from mas_amd import meshgen

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "1M+contacts"
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
mesh, cfg = meshgen.build_config(cfg_name)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None


def prep(P):
    if contacts is None:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    else:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, contacts[0], None, None, contacts[1])
    return P.stats()


def line(tag, st):
    return (f"{tag}: prepare {st['prepare_ms']:.3f} ms (levels {st['prepare_levels_ms']:.3f}, assemble "
            f"{st['prepare_assemble_ms']:.3f}, factor {st['prepare_factor_ms']:.3f}, "
            f"fused level-0 {st['prepare_fine_ms']:.3f} from {st['prepare_fine_start_ms']:.3f}, "
            f"hier rebuilt {st['hier_rebuilt']})")


# one handle at a time (created, measured, destroyed): every handle owns two
# or three HIP streams, and with more streams alive than GPU_MAX_HW_QUEUES
# (4) they share hardware queues, which would serialise a Prepare's overlap
tags = ["unsharded"] + [f"rank {g}/{world}" for g in range(world)]
best = {}
for i, tag in enumerate(tags):
    P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts,
                          shard=None if i == 0 else (i - 1, world))
    for _ in range(reps):
        st = prep(P)
        if tag not in best or st["prepare_ms"] < best[tag]["prepare_ms"]:
            best[tag] = st
    del P
    print(line(tag, best[tag]), flush=True)
slow = max(best[t]["prepare_ms"] for t in tags[1:])
print(f"{cfg_name} world {world}: slowest rank {slow:.3f} ms = {slow / best['unsharded']['prepare_ms']:.3f} x unsharded")
