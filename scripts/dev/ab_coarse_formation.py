"""A/B of the coarse blocks' inverse formation (VALU reference order vs the
matrix-core formation the level-0 blocks use by default), one library per
process (MAS_LIB_NAME).  Prints Prepare phase medians for the unsharded handle
and a world-8 rank, saves z and the coarse inverses for the comparison step.
usage: python scripts/dev/ab_coarse_formation.py TAG [config]
       python scripts/dev/ab_coarse_formation.py --compare TAG_A TAG_B"""
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                "../../preconditioner-for-cloth-and-deformable-body-simulation_amd/python"))
OUT = "gpurun_out/ab_coarse_formation"

if sys.argv[1] == "--compare":
    a, b = (np.load(f"{OUT}/{t}.npz") for t in sys.argv[2:4])
    za, zb = a["z"].astype(np.float64), b["z"].astype(np.float64)
    ia, ib = a["inv"].astype(np.float64), b["inv"].astype(np.float64)
    per_blk = np.linalg.norm((ia - ib).reshape(len(ia), -1), axis=1) / np.linalg.norm(ia.reshape(len(ia), -1), axis=1)
    print(json.dumps({"z_rel_diff": float(np.linalg.norm(za - zb) / np.linalg.norm(za)),
                      "coarse_inverse_rel_diff_max": float(per_blk.max()),
                      "coarse_blocks": int(len(ia))}))
    sys.exit(0)

import mas_amd                      # noqa: E402
from mas_amd import meshgen         # noqa: E402

tag = sys.argv[1]
cfg_name = sys.argv[2] if len(sys.argv) > 2 else "1M+contacts"
mesh, cfg = meshgen.build_config(cfg_name)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
keys = ("prepare_ms", "prepare_assemble_ms", "prepare_factor_ms", "prepare_fine_ms")
res = {}
for shard in (None, (3, 8)):
    P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts, shard=shard)
    runs = []
    for _ in range(6):
        if contacts is None:
            P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
        else:
            P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, contacts[0], None, None, contacts[1])
        runs.append(P.stats())
    res["unsharded" if shard is None else "rank3of8"] = {k: round(statistics.median(r[k] for r in runs[1:]), 4)
                                                          for k in keys}
    if shard is None:
        r = meshgen.residual(mesh.nV, 0x5EED)
        z = P.Preconditioning(None, r)
        inf = P.info()
        nfb, nblk = (mesh.nV + 31) // 32, inf["total_clusters"] // 32
        inv = np.stack([P.block_inverse(b) for b in range(nfb, nblk)])
        os.makedirs(OUT, exist_ok=True)
        np.savez(f"{OUT}/{tag}.npz", z=z, inv=inv)
    del P
print(tag, json.dumps(res), flush=True)
