"""The one-launch coarse form (k_coarse1.hip) and the two-pass form
(k_coarse.hip), in both of its forms, against one launch per coarse level
(k_apply.hip).

Every sum runs in the same order in both forms, so the bar is BITWISE
equality, per apply, over many back-to-back applies with a different residual
each time (a stale coarse value would show up as a mismatch in some later
apply), and the oracle bar (1e-5) for the result itself.  With the
reference's level-3 order (mas_config.reference_restriction = 1) and with
the default grouped level 3 (R3 from the children's R2).
"""
import numpy as np
import pytest

from conftest import cloth, tet

pytestmark = pytest.mark.gpu


def _handles(mesh, L, contacts, monkeypatch, grouped=False):
    """Per-level (mode 0), two-pass (2), two-pass in its occupancy form
    (SoA restriction staging, no level-3 inverse prefetch), one-launch (3),
    the wide two-pass form, and one-launch with round-robin bank waves
    (MAS_C1_CHUNK=0)."""
    import mas_amd
    hs = []
    for mode, occ, wide, chunk in ((0, 0, 0, 1), (2, 0, 0, 1), (2, 1, 0, 1), (3, 0, 0, 1), (2, 0, 1, 1), (3, 0, 0, 0)):
        monkeypatch.setenv("MAS_COARSE_MODE", str(mode))
        monkeypatch.setenv("MAS_COARSE_OCC", str(occ))
        monkeypatch.setenv("MAS_COARSE_WIDE", str(wide))
        monkeypatch.setenv("MAS_C1_CHUNK", str(chunk))
        hs.append(mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts, reference_restriction=not grouped))
        assert hs[-1].stats()["apply_mode"] == mode
    return hs


def _applies(P, rs, stream):
    import torch
    zs = [torch.zeros_like(r) for r in rs]
    torch.cuda.synchronize()
    for z, r in zip(zs, rs):          # back to back, no host sync in between
        P.PreconditioningDevice(z, r, stream.cuda_stream)
    stream.synchronize()
    return [z.cpu().numpy() for z in zs]


CASES = [("cloth", 20, 0, 0), ("cloth", 40, 2, 0), ("cloth", 100, 3, 0), ("cloth", 100, 0, 500),
         ("cloth", 33, 0, 0), ("tet", 16, 3, 0), ("tet", 12, 0, 0), ("cloth", 256, 4, 2000),
         ("cloth", 512, 3, 0), ("cloth", 512, 5, 0), ("tet", 48, 4, 0)]


@pytest.mark.parametrize("kind,W,L,nc", CASES)
@pytest.mark.parametrize("grouped", [False, True])
def test_twopass_equals_per_level(kind, W, L, nc, grouped, monkeypatch):
    import torch
    from mas_amd import meshgen
    mesh = cloth(W) if kind == "cloth" else tet(W)
    contacts = meshgen.vf_contacts(mesh, nc, seed=11) if nc else None
    P3, P2, P2o, P1, P2w, P1r = _handles(mesh, L, contacts, monkeypatch, grouped)
    rs = [torch.from_numpy(meshgen.residual(mesh.nV, 100 + k)).cuda() for k in range(24)]
    s = torch.cuda.Stream()
    z3 = _applies(P3, rs, s)
    for PX in (P2, P2o, P1, P2w, P1r):
        zf = _applies(PX, rs, s)
        for k, (a, b) in enumerate(zip(zf, z3)):
            np.testing.assert_array_equal(a, b, err_msg=f"apply {k}")
        # and again on the same handle
        zf2 = _applies(PX, rs[::-1], s)
        for k, (a, b) in enumerate(zip(zf2, z3[::-1])):
            np.testing.assert_array_equal(a, b, err_msg=f"second pass, apply {k}")


@pytest.mark.parametrize("grouped", [False, True])
def test_twopass_1m_contacts_bitwise_and_oracle(grouped, monkeypatch):
    """The bench workload: 1M cloth + 100k VF contacts, 4 levels; two-pass =
    per-level bitwise over 40 back-to-back applies, and the oracle bar."""
    import torch
    from mas_amd import meshgen
    from oracle import Oracle
    mesh = cloth(1024)
    contacts = meshgen.vf_contacts(mesh, 100_000, seed=3)
    P3, P2, P2o, P1, P2w, P1r = _handles(mesh, 4, contacts, monkeypatch, grouped)
    rs = [torch.from_numpy(meshgen.residual(mesh.nV, 0x5EED + k)).cuda() for k in range(40)]
    s = torch.cuda.Stream()
    z3 = _applies(P3, rs, s)
    for PX in (P2, P2o, P1, P2w, P1r):
        zf = _applies(PX, rs, s)
        for k, (a, b) in enumerate(zip(zf, z3)):
            np.testing.assert_array_equal(a, b, err_msg=f"apply {k}")
    o = Oracle(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0], 4, 8)
    o.allocate(mesh)
    o.prepare(mesh, vf=contacts[0], vfC=contacts[1])
    z_o = o.apply(rs[5].cpu().numpy())
    err = float(np.linalg.norm((zf[5] - z_o)[:, :3]) / np.linalg.norm(z_o[:, :3]))
    assert err <= 1e-5, err
