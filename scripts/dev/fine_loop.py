"""Applies of one BASELINE config on one handle, for PMC passes over the fine
kernel (scripts/dev/gpu_fine_pmc.sh).  argv: config [applies] ; the fine
variant comes from MAS_FINE_VARIANT as in scripts/ab_fine.py.  Prints the
event-timed fine-kernel average (mas_stats.fine_ms_avg) of the same applies."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
import torch
import mas_amd
from mas_amd import meshgen

cfgname = sys.argv[1] if len(sys.argv) > 1 else "1M+contacts"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
mesh, cfg = meshgen.build_config(cfgname)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts, device=0)
r = torch.from_numpy(meshgen.residual(mesh.nV, 0x5EED)).cuda()
z = torch.zeros_like(r)
st = torch.cuda.Stream(); torch.cuda.set_stream(st); sp = st.cuda_stream
for _ in range(5):
    P.PreconditioningDevice(z, r, sp)
torch.cuda.synchronize()
P.set_profiling(True)
for _ in range(K):
    P.PreconditioningDevice(z, r, sp)
torch.cuda.synchronize()
s = P.stats()
print(f"{cfgname} variant {os.environ.get('MAS_FINE_VARIANT', 'default')}: {K} applies, "
      f"fine {s['fine_ms_avg'] * 1e3:.1f} us avg, fine blocks {P.info()['num_fine_blocks']}", flush=True)
