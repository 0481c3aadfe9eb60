"""Applies of one BASELINE config on one handle: for PMC passes over the fine
kernel (scripts/dev/gpu_fine_pmc.sh) and for library A/Bs in separate
processes (MAS_LIB_NAME selects the build).  argv: config [applies].  The fine
variant comes from MAS_FINE_VARIANT as in scripts/ab_fine.py.  Prints one JSON
line: back-to-back ms per apply (events around the K applies), then the
per-phase averages of K profiled applies (mas_stats)."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
import numpy as np
import torch
import mas_amd
from mas_amd import meshgen

cfgname = sys.argv[1] if len(sys.argv) > 1 else "1M+contacts"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
# the mesh is cached under /tmp across the processes of one GPU call (the 4M
# tet takes ~40 s to generate on the host)
cache = f"/tmp/mas_mesh_{cfgname}.npz"
if os.path.exists(cache):
    f = np.load(cache)
    mesh, cfg = meshgen.Mesh(*(f[k] for k in ("pos", "starts", "idx", "diag", "off", "faces", "edges"))), \
        meshgen.CONFIGS[cfgname]
else:
    mesh, cfg = meshgen.build_config(cfgname)
    np.savez(cache + ".part.npz", pos=mesh.pos, starts=mesh.starts, idx=mesh.idx, diag=mesh.diag, off=mesh.off,
             faces=mesh.faces, edges=mesh.edges)
    os.replace(cache + ".part.npz", cache)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts, device=0)
r = torch.from_numpy(meshgen.residual(mesh.nV, 0x5EED)).cuda()
z = torch.zeros_like(r)
st = torch.cuda.Stream(); torch.cuda.set_stream(st); sp = st.cuda_stream
for _ in range(5):
    P.PreconditioningDevice(z, r, sp)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(K):
    P.PreconditioningDevice(z, r, sp)
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / K
P.set_profiling(True)
for _ in range(K):
    P.PreconditioningDevice(z, r, sp)
torch.cuda.synchronize()
s = P.stats()
print(json.dumps(dict(config=cfgname, lib=os.environ.get("MAS_LIB_NAME", "libmas_amd.so"),
                      fine_variant=os.environ.get("MAS_FINE_VARIANT", "default"), applies=K,
                      ms_per_apply=round(ms, 5), pre_fine_us=round(s["pre_fine_ms_avg"] * 1e3, 2),
                      fine_us=round(s["fine_ms_avg"] * 1e3, 2), post_fine_us=round(s["post_fine_ms_avg"] * 1e3, 2),
                      wait_timeouts=s["wait_timeouts"], fine_blocks=P.info()["num_fine_blocks"])), flush=True)
