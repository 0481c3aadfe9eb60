"""Round-6 planning: level-0 bank boundaries at which no coarse row's subtree
is cut (every level-l node's vertices on one side, l = 1..L-1), from the
oracle's level maps (CPU), and the nearest such cut to each equal-split
boundary for world 2/4/8 (largest rank share)."""
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
    return mesh, o.maps(), o.num_levels


def ok_cuts(m, nV, L):
    ct = m["coarse_tables"]   # by sorted vertex: ancestors at levels 1..L-1
    nb = (nV + 31) // 32
    ok = np.ones(nb + 1, bool)
    for l in range(1, L):
        a = ct[:, l - 1].astype(np.int64)
        pad = np.full(nb * 32, a[-1]); pad[:nV] = a
        pre = np.maximum.accumulate(pad)[31::32]             # max anc over vertices < 32(j+1)
        suf = np.minimum.accumulate(pad[::-1])[::-1][::32]   # min anc over vertices >= 32j
        ok[1:nb] &= pre[:nb - 1] < suf[1:nb]
    return ok


def main(names):
    out = {}
    for name in names:
        mesh, m, Lv = maps_for(name)
        nV = mesh.nV
        nb = (nV + 31) // 32
        ok = ok_cuts(m, nV, Lv); L = Lv
        cand = np.flatnonzero(ok)
        res = {"nV": nV, "L": L, "ok_cuts": int(cand.size), "level_sizes": [int(x) for x in m["level_size"][:, 0]]}
        for W in (2, 4, 8):
            eq = [r * nb // W for r in range(W + 1)]
            al = [0] + [int(cand[np.argmin(np.abs(cand - e))]) for e in eq[1:-1]] + [nb]
            res[f"W{W}"] = {"aligned_max_share": round(max(np.diff(al)) / nb, 5),
                            "moved_blocks": [int(a - e) for a, e in zip(al, eq)]}
        out[name] = res
        print(name, json.dumps(res), flush=True)
    return out


if __name__ == "__main__":
    main(sys.argv[1:] or ["256k", "1M+contacts", "4M-tet"])
