"""Fused apply diagnostics: per config and early budget, the apply time by
events, the deferred blocks and the wait give-ups of one apply."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..",
                                "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
import mas_amd  # noqa: E402
from mas_amd import meshgen  # noqa: E402

for config in sys.argv[1:] or ["256k", "1M+contacts"]:
    mesh, cfg = meshgen.build_config(config)
    contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
    for early in ("0", "64", "100000"):
        for mode in ("3", "4"):
            if mode == "3" and early != "0":
                continue
            os.environ["MAS_COARSE_MODE"] = mode
            os.environ["MAS_FUSE_EARLY"] = early
            P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts)
            r = torch.from_numpy(meshgen.residual(mesh.nV, 1)).cuda()
            z = torch.zeros_like(r)
            s = torch.cuda.Stream()
            ts = []
            for k in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                P.PreconditioningDevice(z, r, s.cuda_stream)
                e1.record(s)
                s.synchronize()
                ts.append(e0.elapsed_time(e1))
            st = P.stats()
            print(f"{config} mode {mode} early {early}: ms {['%.3f' % t for t in ts]} "
                  f"timeouts {st['wait_timeouts']}", flush=True)
            del P
