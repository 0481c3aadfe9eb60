"""Incremental level maps: a sequence of Prepares with changing
contact sets on one handle.

The handle keeps the contact-free hierarchy of its sort; each Prepare checks
on the device whether its stencils change it (k_hier_check) and reuses the
levels, the coarse edge records, the diagTable term lists and the apply tables
when they do not, or rebuilds the levels with the contacts when they do.
Bars:
  * level maps (CoarseSpaceTables, goingNext, coarseTables, the fine connect
    masks, level sizes) bit-exact against the oracle prepared from scratch
    with the same contacts, after every Prepare of the sequence;
  * z bitwise equal to a handle that rebuilds everything every Prepare
    (MAS_HIER_CACHE=0), so the reused records / term lists / apply tables are
    exactly the rebuilt ones; z within Z_TOL of the oracle;
  * mas_stats.hier_dirty_level says whether the contacts changed the
    hierarchy (and at which level), checked against the oracle's own maps.
"""
import os

import numpy as np
import pytest

from conftest import cloth
from test_gpu_parity import Z_TOL, _oracle, compare_maps, rel_err

pytestmark = pytest.mark.gpu


def _handle(mesh, L, cache=True, **kw):
    import mas_amd
    old = os.environ.get("MAS_HIER_CACHE")
    os.environ["MAS_HIER_CACHE"] = "1" if cache else "0"
    try:
        P = mas_amd.SeSchwarzPreconditioner(max_levels=L, reference_formation=True, **kw)
    finally:
        if old is None:
            del os.environ["MAS_HIER_CACHE"]
        else:
            os.environ["MAS_HIER_CACHE"] = old
    P.m_positions = mesh.pos
    P.m_neighbours = (mesh.starts, mesh.idx)
    P.m_edges = mesh.edges
    P.m_faces = mesh.faces
    P.AllocatePrecoditioner(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0])
    return P


def _prepare(P, mesh, contacts):
    if contacts is None:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    else:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, contacts[0], None, None, contacts[1])


def _level0_joining_contacts(mesh, L, count=3):
    """VF contacts whose vertex and a face vertex share a level-0 bank but lie
    in different contact-free components there (they change level 0)."""
    from mas_amd import meshgen
    m = _oracle(mesh, L).maps()
    o2s, fine = m["o2s"], m["fine_connect_mask"]
    picks = []
    fs = mesh.faces[:, :3]
    rng = np.random.default_rng(11)
    for f in rng.permutation(fs.shape[0]):
        a = o2s[fs[f, 0]]
        bank = a >> 5
        cand = [s for s in range(bank * 32, min(bank * 32 + 32, mesh.nV)) if not (fine[a] >> (s & 31)) & 1]
        if cand:
            v = int(np.nonzero(o2s == cand[0])[0][0])
            picks.append((v, int(f)))
        if len(picks) == count:
            break
    assert len(picks) == count, "no multi-component level-0 bank in this mesh"
    vf = np.zeros(count, dtype=meshgen.VF_DTYPE)
    vf["vId"] = [p[0] for p in picks]
    vf["fId"] = [p[1] for p in picks]
    vf["stiff"] = 100.0
    vf["bary"][:, 0] = 0.25
    vf["bary"][:, 1] = 0.25
    vf["normal"][:, 2] = 1.0
    cnt = np.zeros(mesh.nV + 1, np.uint32)
    cnt[mesh.nV] = count
    return vf, cnt


def _expected_dirty(mesh, L, contacts, mesh_maps):
    """The oracle's own answer: does this contact set change the hierarchy?"""
    m = _oracle(mesh, L, contacts).maps()
    same = (np.array_equal(m["coarse_space_tables"], mesh_maps["coarse_space_tables"]) and
            np.array_equal(m["fine_connect_mask"], mesh_maps["fine_connect_mask"]) and
            np.array_equal(m["level_size"], mesh_maps["level_size"]) and
            np.array_equal(m["going_next"], mesh_maps["going_next"]))
    return same


def test_contact_sequence_maps_and_z():
    from mas_amd import meshgen
    mesh = cloth(100)            # 10k vertices, 3 levels; its banks hold several components
    L = 0
    seq = [("none", None), ("vf2", meshgen.vf_contacts(mesh, 2, seed=3)),
           ("vf50", meshgen.vf_contacts(mesh, 50, seed=3)), ("vf2", meshgen.vf_contacts(mesh, 2, seed=3)),
           ("lvl0", _level0_joining_contacts(mesh, L)), ("vf50b", meshgen.vf_contacts(mesh, 50, seed=9)),
           ("none", None), ("vf2", meshgen.vf_contacts(mesh, 2, seed=3))]
    P = _handle(mesh, L)
    F = _handle(mesh, L, cache=False)
    mesh_maps = _oracle(mesh, L).maps()
    r = meshgen.residual(mesh.nV, 0x5EED)
    seen = set()
    for i, (name, c) in enumerate(seq):
        _prepare(P, mesh, c)
        _prepare(F, mesh, c)
        o = _oracle(mesh, L, c)
        compare_maps(P, o, mesh.nV)
        st = P.stats()
        nL = P.info()["num_levels"]
        clean = _expected_dirty(mesh, L, c, mesh_maps)
        assert (st["hier_dirty_level"] == nL) == clean, (name, st["hier_dirty_level"], clean)
        if name == "lvl0":
            assert st["hier_dirty_level"] == 0
        if clean and i > 0:
            assert st["hier_rebuilt"] == 0, name
        else:
            assert st["hier_rebuilt"] == 1, name
        seen.add(clean)
        assert F.stats()["hier_dirty_level"] == -1 and F.stats()["hier_rebuilt"] == 1
        z = P.Preconditioning(None, r)
        zf = F.Preconditioning(None, r)
        np.testing.assert_array_equal(z, zf)            # reused tables == rebuilt tables
        assert rel_err(z, o.apply(r)) <= Z_TOL
        print(f"{name}: dirty level {st['hier_dirty_level']} (L = {nL}), rebuilt {st['hier_rebuilt']}, "
              f"levels phase {st['prepare_levels_ms']:.3f} ms, prepare {st['prepare_ms']:.3f} ms")
    assert seen == {True, False}  # both paths ran


def test_ranges_change_invalidates_records():
    """The cached coarse records index off9 through the CSR ranges: a Prepare
    whose ranges differ (same matrices, rows stored in reverse order) must
    rebuild them -- z equal to the normal layout's, bitwise."""
    import torch
    from mas_amd import meshgen
    mesh = cloth(64)
    P = _handle(mesh, 0)
    r = meshgen.residual(mesh.nV, 5)
    _prepare(P, mesh, None)
    z0 = P.Preconditioning(None, r)
    _prepare(P, mesh, None)
    assert P.stats()["hier_rebuilt"] == 0
    np.testing.assert_array_equal(P.Preconditioning(None, r), z0)
    starts = mesh.starts.astype(np.int64)
    nnz = int(starts[-1])
    deg = np.diff(starts)
    rstarts = nnz - starts[1:]                 # row o starts where the reversed layout puts it
    off = np.zeros_like(mesh.off)
    for o in range(mesh.nV):
        off[rstarts[o]:rstarts[o] + deg[o]] = mesh.off[starts[o]:starts[o + 1]]
    ranges = np.append(rstarts, nnz).astype(np.int32)  # only [0, nV) are read as row starts
    dd = torch.from_numpy(np.ascontiguousarray(mesh.diag, np.float32)).cuda()
    do = torch.from_numpy(off).cuda()
    dr = torch.from_numpy(ranges).cuda()
    torch.cuda.synchronize()
    P.PreparePreconditionerDevice(dd, do, dr)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(P.Preconditioning(None, r), z0)
    _prepare(P, mesh, None)                    # and back
    np.testing.assert_array_equal(P.Preconditioning(None, r), z0)


@pytest.mark.parametrize("count", [100_000, 1_000])
def test_1m_contacts_reuse(count):
    """BASELINE configs[2] (1M cloth + VF contacts, 4 levels) and a 1k-contact
    variant: the contacts leave the hierarchy unchanged, so a steady-state
    Prepare reuses it -- z bitwise equal to a handle that rebuilds everything."""
    import torch
    from mas_amd import meshgen
    mesh = cloth(1024)
    c = meshgen.vf_contacts(mesh, count, seed=3)
    P = _handle(mesh, 4)
    F = _handle(mesh, 4, cache=False)
    for _ in range(3):
        _prepare(P, mesh, c)
    _prepare(F, mesh, c)
    st, sf = P.stats(), F.stats()
    assert st["hier_dirty_level"] == 4 and st["hier_rebuilt"] == 0
    r = meshgen.residual(mesh.nV, 0x5EED + 2)
    rd = torch.from_numpy(r).cuda()
    z1, z2 = torch.zeros_like(rd), torch.zeros_like(rd)
    torch.cuda.synchronize()
    P.PreconditioningDevice(z1, rd)
    F.PreconditioningDevice(z2, rd)
    torch.cuda.synchronize()
    assert torch.equal(z1, z2)
    np.testing.assert_array_equal(P.maps()["coarse_space_tables"], F.maps()["coarse_space_tables"])
    print(f"1M + {count} contacts: Prepare {st['prepare_ms']:.3f} ms (levels {st['prepare_levels_ms']:.3f}, "
          f"fused start {st['prepare_fine_start_ms']:.3f}) vs rebuilt {sf['prepare_ms']:.3f} ms "
          f"(levels {sf['prepare_levels_ms']:.3f})")
