"""Apply time against time since the first apply: batches of B back-to-back
applies (events around each batch) for S seconds on one handle; prints the
ms per apply of every batch.  Shows whether a short run (bench.py's driver
command: 5 warm-up + 20 timed applies) sees the same per-apply time as a long
one.  argv: config [seconds] [batch]."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
import numpy as np
import torch
import mas_amd
from mas_amd import meshgen

cfgname = sys.argv[1] if len(sys.argv) > 1 else "1M+contacts"
S = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
B = int(sys.argv[3]) if len(sys.argv) > 3 else 20
cache = f"/tmp/mas_mesh_{cfgname}.npz"
if os.path.exists(cache):
    f = np.load(cache)
    mesh, cfg = meshgen.Mesh(*(f[k] for k in ("pos", "starts", "idx", "diag", "off", "faces", "edges"))), \
        meshgen.CONFIGS[cfgname]
else:
    mesh, cfg = meshgen.build_config(cfgname)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts, device=0)
r = torch.from_numpy(meshgen.residual(mesh.nV, 0x5EED)).cuda()
z = torch.zeros_like(r)
st = torch.cuda.Stream(); torch.cuda.set_stream(st); sp = st.cuda_stream
torch.cuda.synchronize()
out, t0 = [], time.perf_counter()
while time.perf_counter() - t0 < S:
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(B):
        P.PreconditioningDevice(z, r, sp)
    e1.record(st)
    torch.cuda.synchronize()
    out.append((round(time.perf_counter() - t0, 4), round(e0.elapsed_time(e1) / B, 5)))
ms = [m for _, m in out]
print(json.dumps(dict(config=cfgname, batch=B, batches=len(out), first=out[:12], last=out[-3:],
                      median_after_1s=float(np.median([m for t, m in out if t > 1.0] or ms)))), flush=True)
