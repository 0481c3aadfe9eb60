"""One 1M-vertex PCG solve (for profiling the PCG kernels alone)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
import numpy as np
import torch
import mas_amd
from mas_amd import meshgen
mesh, cfg = meshgen.build_config(sys.argv[1] if len(sys.argv) > 1 else "1M")
P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"])
dd = torch.from_numpy(np.ascontiguousarray(mesh.diag, np.float32)).cuda()
do = torch.from_numpy(np.ascontiguousarray(mesh.off, np.float32)).cuda()
dr = torch.from_numpy(np.ascontiguousarray(mesh.starts, np.int32)).cuda()
b = torch.from_numpy(meshgen.residual(mesh.nV, 1)).cuda()
x = torch.zeros_like(b)
torch.cuda.synchronize()
print(P.pcg_solve_device(dd, do, dr, x, b, max_iters=40, tol=1e-9, precondition=False))
