"""A/B library knobs (env vars read at mas_create) in one process, interleaved rounds.
usage: python scripts/ab_env.py "MAS_OVERLAP=0" "MAS_OVERLAP=1" [--config 1M+contacts]"""
import os, sys, statistics, json, argparse
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
ap = argparse.ArgumentParser(); ap.add_argument("variants", nargs="+"); ap.add_argument("--config", default="1M+contacts")
ap.add_argument("--rounds", type=int, default=8); ap.add_argument("--steps", type=int, default=100)
args = ap.parse_args()
import torch, numpy as np
import mas_amd
from mas_amd import meshgen
mesh, cfg = meshgen.build_config(args.config)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
Ps = {}
for v in args.variants:
    saved = {}
    for kv in v.split(","):
        k, val = kv.split("="); saved[k] = os.environ.get(k); os.environ[k] = val
    Ps[v] = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts, device=0)
    for k, old in saved.items():
        if old is None: os.environ.pop(k)
        else: os.environ[k] = old
r = torch.from_numpy(meshgen.residual(mesh.nV, 0x5EED)).cuda()
zs = {v: torch.zeros_like(r) for v in args.variants}
torch.cuda.synchronize()
st = torch.cuda.Stream(); torch.cuda.set_stream(st); sp = st.cuda_stream
res = {v: {"step": [], "fine": [], "pre": [], "post": []} for v in args.variants}
for rnd in range(args.rounds):
    for v in args.variants:
        P = Ps[v]
        for _ in range(10): P.PreconditioningDevice(zs[v], r, sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record(st)
        for _ in range(args.steps): P.PreconditioningDevice(zs[v], r, sp)
        e1.record(st); torch.cuda.synchronize()
        res[v]["step"].append(e0.elapsed_time(e1) / args.steps * 1e3)
        P.set_profiling(True)
        for _ in range(args.steps): P.PreconditioningDevice(zs[v], r, sp)
        torch.cuda.synchronize()
        s = P.stats(); P.set_profiling(False)
        res[v]["fine"].append(s["fine_ms_avg"] * 1e3); res[v]["pre"].append(s["pre_fine_ms_avg"] * 1e3)
        res[v]["post"].append(s["post_fine_ms_avg"] * 1e3)
z0 = zs[args.variants[0]].cpu().numpy()
out = {}
for v in args.variants:
    out[v] = {k + "_us_med": round(statistics.median(x), 2) for k, x in res[v].items()}
    out[v]["step_us_min"] = round(min(res[v]["step"]), 2)
    out[v]["bitwise_equal_to_first"] = bool(np.array_equal(zs[v].cpu().numpy(), z0))
print(json.dumps(out, indent=1))
