"""A/B the fine-kernel variants (MAS_FINE_VARIANT) in one process, interleaved rounds."""
import os, sys, statistics, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
import torch, numpy as np
import mas_amd
from mas_amd import meshgen

variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2").split(",")]
cfgname = sys.argv[2] if len(sys.argv) > 2 else "1M+contacts"
mesh, cfg = meshgen.build_config(cfgname)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
Ps = {}
for v in variants:
    os.environ["MAS_FINE_VARIANT"] = str(v)
    Ps[v] = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts, device=0)
r = torch.from_numpy(meshgen.residual(mesh.nV, 0x5EED)).cuda()
zs = {v: torch.zeros_like(r) for v in variants}
torch.cuda.synchronize()
st = torch.cuda.Stream(); torch.cuda.set_stream(st); sp = st.cuda_stream
K = 100
res = {v: {"step": [], "fine": []} for v in variants}
for rnd in range(8):
    for v in variants:
        P = Ps[v]
        for _ in range(10): P.PreconditioningDevice(zs[v], r, sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record(st)
        for _ in range(K): P.PreconditioningDevice(zs[v], r, sp)
        e1.record(st); torch.cuda.synchronize()
        res[v]["step"].append(e0.elapsed_time(e1) / K * 1e3)
        P.set_profiling(True)
        for _ in range(K): P.PreconditioningDevice(zs[v], r, sp)
        torch.cuda.synchronize()
        res[v]["fine"].append(P.stats()["fine_ms_avg"] * 1e3); P.set_profiling(False)
z0 = zs[variants[0]].cpu().numpy()
out = {}
for v in variants:
    zv = zs[v].cpu().numpy()
    out[v] = dict(step_us_med=statistics.median(res[v]["step"]), step_us_min=min(res[v]["step"]),
                  fine_us_med=statistics.median(res[v]["fine"]), fine_us_min=min(res[v]["fine"]),
                  bitwise_equal_to_first=bool(np.array_equal(zv, z0)))
print(json.dumps(out, indent=1))
