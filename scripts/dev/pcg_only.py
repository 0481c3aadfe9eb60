"""PCG-only driver for A/B runs: python scripts/dev/pcg_only.py [config] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "../../preconditioner-for-cloth-and-deformable-body-simulation_amd/python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mas_amd  # noqa: E402
from mas_amd import meshgen  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "1M+contacts"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
mesh, cfg = meshgen.build_config(cfg_name)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts)
r = torch.from_numpy(meshgen.residual(mesh.nV, 0x5EED)).cuda()
dd = torch.from_numpy(np.ascontiguousarray(mesh.diag, np.float32)).cuda()
do = torch.from_numpy(np.ascontiguousarray(mesh.off, np.float32)).cuda()
dr = torch.from_numpy(np.ascontiguousarray(mesh.starts, np.int32)).cuda()
s = torch.cuda.Stream()
torch.cuda.synchronize()
for _ in range(reps):
    for name, pre in (("mas", True), ("none", False)):
        x = torch.zeros_like(r)
        res = P.pcg_solve_device(dd, do, dr, x, r, max_iters=5000, tol=1e-5, precondition=pre, stream=s.cuda_stream)
        torch.cuda.synchronize()
        print(f"{name}: iters {res['iterations']} true_rel {res['true_rel_residual']:.3g} "
              f"ms/iter {res['solve_ms'] / max(res['iterations'], 1):.4f}", flush=True)
