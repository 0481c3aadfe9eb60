"""Subtree locality of the coarse assembly (CPU, oracle only).

The claim behind the plan to shard the coarse assembly (DESIGN.md §7,
"Sharding the coarse assembly"): every term a coarse row receives in
`PrepareHessian` (/root/reference/SeSchwarzPreconditioner.cpp:1229-1345) and
`PrepareCollisionHessian` / `AdditionalSchwarzHessian2` (.cpp:1164-1227) comes
from that row's subtree -- the CSR rows and diagonals of the vertices below it
and the contact stencils touching them -- so a rank holding one level-1
cluster's vertices can fold that cluster's level-1 block and the level-2 rows
above it bitwise by itself.

Test: scale every input outside one level-1 cluster's vertex range (CSR rows,
diagonals, and the stiffness of stencils not touching the range) and check
that the cluster's level-1 block and its level-2 rows are bitwise unchanged,
while other blocks do change.  Positions and topology are untouched, so the
level maps stay the same (asserted).
"""
import numpy as np
import pytest

from conftest import cloth, tet


def _run(mesh, L, vf=None, vfC=None):
    from oracle import Oracle
    o = Oracle(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0], L, 1)
    o.allocate(mesh)
    if vf is None:
        o.prepare(mesh)
    else:
        o.prepare(mesh, vf=vf, vfC=vfC)
    return o


def _scaled_outside(mesh, inside_orig, factor):
    """A copy of the mesh with the Hessian rows of vertices outside
    `inside_orig` (original ids) scaled by `factor`."""
    import copy
    m = copy.copy(mesh)
    n = mesh.nV
    outside = np.ones(n, bool)
    outside[inside_orig] = False
    diag = mesh.diag.reshape(n, 9).copy()
    diag[outside] *= factor
    off = mesh.off.reshape(-1, 9).copy()
    rows = np.repeat(np.arange(n), np.diff(mesh.starts))
    off[outside[rows]] *= factor
    m.diag = diag.reshape(mesh.diag.shape)
    m.off = off.reshape(mesh.off.shape)
    return m


@pytest.mark.parametrize("kind,W,L,contacts", [("cloth", 96, 4, 0), ("cloth", 96, 4, 3000), ("tet", 16, 4, 0)])
def test_coarse_rows_depend_only_on_their_subtree(kind, W, L, contacts):
    from mas_amd import meshgen
    mesh = cloth(W) if kind == "cloth" else tet(W)
    vf = vfC = None
    if contacts:
        vf, vfC = meshgen.vf_contacts(mesh, contacts)
    base = _run(mesh, L, vf, vfC)
    m = base.maps()
    assert base.num_levels >= 3
    ls = m["level_size"]
    ct = m["coarse_tables"]
    n1, b1 = int(ls[1][0]), int(ls[1][1])
    n_clusters1 = (n1 + 31) // 32
    assert n_clusters1 >= 3
    c = n_clusters1 // 2
    lo, hi = b1 + 32 * c, b1 + min(32 * (c + 1), n1)
    S = np.nonzero((ct[:, 0] >= lo) & (ct[:, 0] < hi))[0]            # sorted ids
    # the cluster's vertices are one contiguous Morton range (a shard boundary can sit there)
    assert S.size and np.array_equal(S, np.arange(S[0], S[-1] + 1))
    inside_orig = m["s2o"][S]

    pm = _scaled_outside(mesh, inside_orig, 2.0)
    pvf = vf
    if contacts:
        touch = np.zeros(mesh.nV, bool)
        touch[inside_orig] = True
        f = mesh.faces[vf["fId"]]
        hit = touch[vf["vId"]] | touch[f[:, 0]] | touch[f[:, 1]] | touch[f[:, 2]]
        assert hit.any() and not hit.all()
        pvf = vf.copy()
        pvf["stiff"][~hit] *= 2.0
    pert = _run(pm, L, pvf, vfC)
    pmaps = pert.maps()
    for k in ("s2o", "going_next", "coarse_tables", "coarse_space_tables", "level_size"):
        np.testing.assert_array_equal(pmaps[k], m[k])

    # the level-1 block of the cluster: every entry
    blk1 = lo // 32
    np.testing.assert_array_equal(pert.block_matrix(blk1), base.block_matrix(blk1))
    # the level-2 rows above it: each node's whole subtree lies in S
    owned2 = np.unique(ct[S, 1])
    for node in owned2:
        assert np.all(np.isin(np.nonzero(ct[:, 1] == node)[0], S))
        blk, row = node // 32, node % 32
        a, b = base.block_matrix(blk), pert.block_matrix(blk)
        np.testing.assert_array_equal(b[3 * row:3 * row + 3], a[3 * row:3 * row + 3])
    # teeth: a neighbouring level-1 block does change
    other = blk1 - 1 if blk1 > b1 // 32 else blk1 + 1
    assert not np.array_equal(pert.block_matrix(other), base.block_matrix(other))
