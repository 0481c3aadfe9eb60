"""Round-6 planning numbers for sharding the coarse assembly:
level-1-cluster-aligned shard boundaries vs the equal split of level-0
blocks, from the oracle's level maps (CPU).  Prints, per config and world
size, the largest rank's share of level-0 blocks under each split and the
level-1 inverse bytes a rank would receive in an allgather."""
import json
import sys

import numpy as np

sys.path.insert(0, "oracle")
sys.path.insert(0, "preconditioner-for-cloth-and-deformable-body-simulation_amd/python")
from mas_amd import meshgen          # noqa: E402
from oracle import Oracle            # noqa: E402


def maps_for(name):
    mesh, cfg = meshgen.build_config(name)
    o = Oracle(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0], cfg["levels"], 8)
    o.allocate(mesh)
    if cfg["contacts"]:
        vf, vfC = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3)
        o.prepare(mesh, vf=vf, vfC=vfC)
    else:
        o.prepare(mesh)
    return mesh, o.maps()


def main(names):
    out = {}
    for name in names:
        mesh, m = maps_for(name)
        nV = mesh.nV
        nfb = (nV + 31) // 32
        ls = m["level_size"]
        ct = m["coarse_tables"]
        n1, b1 = int(ls[1][0]), int(ls[1][1])
        # first level-0 block of each level-1 cluster (level-1 nodes never leave a bank)
        first_blk = np.full((n1 + 31) // 32, nfb, np.int64)
        cl = (ct[:, 0] - b1) // 32
        np.minimum.at(first_blk, cl, np.arange(nV) // 32)
        starts = np.unique(first_blk)
        res = {"nV": nV, "level1_nodes": n1, "level1_clusters": int(starts.size),
               "level_sizes": [int(x) for x in ls[:, 0]],
               "level1_inverse_MB": round(starts.size * 96 * 97 / 2 * 4 / 1e6, 2)}
        for W in (2, 4, 8):
            eq = [r * nfb // W for r in range(W + 1)]
            al = [0] + [int(starts[np.argmin(np.abs(starts - e))]) for e in eq[1:-1]] + [nfb]
            res[f"W{W}"] = {"equal_max_share": max(np.diff(eq)) / nfb,
                            "aligned_max_share": max(np.diff(al)) / nfb,
                            "aligned_bounds": al}
        out[name] = res
        print(name, json.dumps(res), flush=True)
    return out


if __name__ == "__main__":
    main(sys.argv[1:] or ["1M+contacts", "4M-tet"])
