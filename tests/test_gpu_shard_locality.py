"""Subtree locality of the GPU coarse assembly (the basis for sharding it,
DESIGN.md §7 "Sharding the coarse assembly"; the oracle's version is
tests/test_oracle_shard_locality.py).

For a shard's Morton range S (the equal split of level-0 blocks, as
`mas_set_prepare_shard` uses), every coarse row whose subtree lies inside S
must be bitwise unchanged when every input outside S changes: the CSR rows and
diagonals of the other vertices and the stiffness of stencils not touching S
(`PrepareHessian`, /root/reference/SeSchwarzPreconditioner.cpp:1229-1345;
`AdditionalSchwarzHessian2`, .cpp:1164-1199).  Positions and topology are the
same, so the level maps are too (asserted).  Bar: bit-exact.
"""
import numpy as np
import pytest

from conftest import cloth

pytestmark = pytest.mark.gpu


def _prepare(mesh, L, contacts):
    import mas_amd
    return mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts)


def _perturbed(mesh, contacts, inside_orig):
    import copy
    n = mesh.nV
    m = copy.copy(mesh)
    outside = np.ones(n, bool)
    outside[inside_orig] = False
    diag = mesh.diag.reshape(n, 9).copy()
    diag[outside] *= 2.0
    off = mesh.off.reshape(-1, 9).copy()
    rows = np.repeat(np.arange(n), np.diff(mesh.starts))
    off[outside[rows]] *= 2.0
    m.diag, m.off = diag.reshape(mesh.diag.shape), off.reshape(mesh.off.shape)
    if contacts is None:
        return m, None
    vf, vfC = contacts
    f = mesh.faces[vf["fId"]]
    touch = ~outside
    hit = touch[vf["vId"]] | touch[f[:, 0]] | touch[f[:, 1]] | touch[f[:, 2]]
    assert hit.any() and not hit.all()
    pvf = vf.copy()
    pvf["stiff"][~hit] *= 2.0
    return m, (pvf, vfC)


def _owned_rows(ct, L, S_mask):
    """{block: [rows]} of the coarse nodes whose whole subtree is in S."""
    owned = {}
    for lv in range(1, L):
        anc = ct[:, lv - 1]
        tot = np.bincount(anc)
        ins = np.bincount(anc[S_mask], minlength=tot.size)
        for node in np.nonzero((tot > 0) & (ins == tot))[0]:
            owned.setdefault(int(node) // 32, []).append(int(node) % 32)
    return owned


@pytest.mark.parametrize("config,rank,world", [("cloth96+contacts", 1, 3), ("1M+contacts", 3, 8)])
def test_shard_owned_coarse_rows_depend_only_on_the_shard(config, rank, world):
    from mas_amd import meshgen
    if config == "1M+contacts":
        mesh, cfg = meshgen.build_config(config)
        L, contacts = cfg["levels"], meshgen.vf_contacts(mesh, cfg["contacts"], seed=3)
    else:
        mesh, L = cloth(96), 4
        contacts = meshgen.vf_contacts(mesh, 3000)
    base = _prepare(mesh, L, contacts)
    m = base.maps()
    nV = mesh.nV
    nfb = (nV + 31) // 32
    b0, b1 = rank * nfb // world, (rank + 1) * nfb // world
    S_mask = np.zeros(nV, bool)
    S_mask[32 * b0:min(32 * b1, nV)] = True
    inside_orig = m["s2o"][S_mask]
    pm, pc = _perturbed(mesh, contacts, inside_orig)
    pert = _prepare(pm, L, pc)
    pmaps = pert.maps()
    for k in ("s2o", "going_next", "coarse_tables", "coarse_space_tables"):
        np.testing.assert_array_equal(pmaps[k], m[k])

    Lv = int(base.info()["num_levels"])
    owned = _owned_rows(m["coarse_tables"], Lv, S_mask)
    assert owned
    n_rows = 0
    for blk, rows in sorted(owned.items()):
        a, b = base.block_matrix(blk), pert.block_matrix(blk)
        for r in rows:
            np.testing.assert_array_equal(b[3 * r:3 * r + 3], a[3 * r:3 * r + 3], err_msg=f"block {blk} row {r}")
        n_rows += len(rows)
    # teeth: a coarse block of another shard changes
    others = [blk for blk in range(nfb, int(base.info()["total_clusters"]) // 32) if blk not in owned]
    assert any(not np.array_equal(base.block_matrix(blk), pert.block_matrix(blk)) for blk in others[:8])
    print(f"{config} rank {rank}/{world}: {n_rows} owned coarse rows in {len(owned)} blocks bitwise unchanged")
