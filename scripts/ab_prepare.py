"""A/B Prepare variants (env knobs read at mas_create): device time per phase and
bitwise comparison of the resulting inverses / applies.
usage: python scripts/ab_prepare.py "MAS_FACTOR_VARIANT=0" "MAS_FACTOR_VARIANT=1" [--config 1M+contacts]"""
import os, sys, statistics, json, argparse
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
ap = argparse.ArgumentParser(); ap.add_argument("variants", nargs="+"); ap.add_argument("--config", default="1M+contacts")
ap.add_argument("--rounds", type=int, default=3)
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
keys = ("prepare_ms", "prepare_levels_ms", "prepare_assemble_ms", "prepare_factor_ms", "prepare_fine_ms",
        "prepare_fine_start_ms")
res = {v: {k: [] for k in keys} for v in args.variants}
for rnd in range(args.rounds):
    for v in args.variants:
        P = Ps[v]
        if contacts is None:
            P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
        else:
            P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, contacts[0], None, None, contacts[1])
        s = P.stats()
        for k in keys: res[v][k].append(s[k])
r = meshgen.residual(mesh.nV, 0x5EED)
z = {v: Ps[v].Preconditioning(None, r) for v in args.variants}
inf = Ps[args.variants[0]].info()
nblk = inf["total_clusters"] // 32
sample = sorted(set(list(range(0, min(64, nblk))) + list(range((mesh.nV + 31) // 32, nblk))))
out = {"config": args.config, "blocks_compared": len(sample)}
v0 = args.variants[0]
for v in args.variants:
    d = {k + "_med": round(statistics.median(x), 3) for k, x in res[v].items()}
    d["apply_bitwise_equal_to_first"] = bool(np.array_equal(z[v], z[v0]))
    d["inverses_bitwise_equal_to_first"] = all(np.array_equal(Ps[v].block_inverse(b), Ps[v0].block_inverse(b))
                                               for b in sample)
    out[v] = d
print(json.dumps(out, indent=1))
