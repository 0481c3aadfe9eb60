"""Prepare-only driver for profiling: one config, N steady-state Prepares.
python scripts/dev/prep_only.py [config] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "../../preconditioner-for-cloth-and-deformable-body-simulation_amd/python"))

import mas_amd
from mas_amd import meshgen

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "1M+contacts"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
mesh, cfg = meshgen.build_config(cfg_name)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
# PREP_SHARD=rank,world: a sharded Prepare (mas_set_prepare_shard) of that rank
shard = tuple(int(x) for x in os.environ["PREP_SHARD"].split(",")) if os.environ.get("PREP_SHARD") else None
P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts, shard=shard)
# PREP_DEVICE=1: the Hessian from device memory (mas_prepare_device), so host
# work inside Prepare is not hidden behind the H2D copies
dev = None
if os.environ.get("PREP_DEVICE") == "1":
    import numpy as np
    import torch
    dev = tuple(torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (mesh.diag, mesh.off, mesh.starts))
    torch.cuda.synchronize()
for _ in range(reps):
    t0 = time.perf_counter()
    if dev is not None:
        if contacts is None:
            P.PreparePreconditionerDevice(*dev)
        else:
            P.PreparePreconditionerDevice(*dev, None, None, contacts[0], None, None, contacts[1])
    elif contacts is None:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    else:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, contacts[0], None, None, contacts[1])
    st = P.stats()
    print(f"prepare {st['prepare_ms']:.3f} ms (levels {st['prepare_levels_ms']:.3f}, assemble "
          f"{st['prepare_assemble_ms']:.3f}, factor {st['prepare_factor_ms']:.3f}, fused level-0 {st['prepare_fine_ms']:.3f} from {st['prepare_fine_start_ms']:.3f}, hier rebuilt {st['hier_rebuilt']}); host {1e3*(time.perf_counter()-t0):.1f} ms",
          flush=True)
