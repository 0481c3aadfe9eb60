"""The matrix-core inverse formation (k_factor.hip form_mfma: MAS_FACTOR_VARIANT
3 = unfused, 5 = inside the fused level-0 kernel, the library default since
round 3) against the reference-order VALU formation (mas_config
.reference_formation = 1, bitwise equal to the oracle for equal blocks).

The elimination is shared, so the two differ only in the order in which the
96 products of every inverse entry are summed.  Bars: every block's inverse
within 2e-5 relative (Frobenius) of the VALU one -- a few fp32 ulps of the
entries' magnitude -- and z = M^-1 r within the north-star 1e-5 of the oracle.
"""
import numpy as np
import pytest

from conftest import cloth, tet

pytestmark = pytest.mark.gpu


def _pair(mesh, L, contacts, monkeypatch, variant):
    import mas_amd
    monkeypatch.setenv("MAS_FACTOR_VARIANT", "2")
    P2 = mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts)
    monkeypatch.setenv("MAS_FACTOR_VARIANT", variant)
    P3 = mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts)
    return P2, P3


@pytest.mark.parametrize("variant", ["3", "5"])
@pytest.mark.parametrize("kind,W,L,nc", [("cloth", 64, 0, 200), ("tet", 16, 3, 0), ("cloth", 33, 0, 0)])
def test_mfma_inverse_matches_valu(kind, W, L, nc, variant, monkeypatch):
    from mas_amd import meshgen
    mesh = cloth(W) if kind == "cloth" else tet(W)
    contacts = meshgen.vf_contacts(mesh, nc, seed=5) if nc else None
    P2, P3 = _pair(mesh, L, contacts, monkeypatch, variant)
    worst = 0.0
    for blk in range(P2.info()["num_blocks"]):
        a, b = P2.block_inverse(blk), P3.block_inverse(blk)
        err = float(np.linalg.norm(b - a) / max(np.linalg.norm(a), 1e-30))
        worst = max(worst, err)
    print(f"{kind}{W} L={L}: worst block inverse rel. difference {worst:.2e}")
    assert worst <= 2e-5, worst


@pytest.mark.parametrize("variant", ["3", "5"])
def test_mfma_z_within_tolerance_1m_contacts(variant, monkeypatch):
    from mas_amd import meshgen
    from oracle import Oracle
    mesh = cloth(1024)
    contacts = meshgen.vf_contacts(mesh, 100_000, seed=3)
    monkeypatch.setenv("MAS_FACTOR_VARIANT", variant)
    import mas_amd
    P3 = mas_amd.from_mesh(mesh, max_levels=4, contacts=contacts)
    o = Oracle(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0], 4, 8)
    o.allocate(mesh)
    o.prepare(mesh, vf=contacts[0], vfC=contacts[1])
    r = meshgen.residual(mesh.nV, 0x5EED + 2)
    z = P3.Preconditioning(None, r)
    zo = o.apply(r)
    err = float(np.linalg.norm((z - zo)[:, :3]) / np.linalg.norm(zo[:, :3]))
    print(f"1M + contacts, MFMA formation: z rel. error vs oracle {err:.2e}")
    assert err <= 1e-5, err


def test_default_formation_blocks_256k():
    """The library default (matrix-core formation inside the fused level-0
    kernel) against the reference-order formation (mas_config
    .reference_formation = 1) block by block at BASELINE configs[1] (256k
    cloth, 3 levels): every 8th level-0 block and every coarse block within
    2e-5 relative (Frobenius)."""
    import mas_amd
    mesh = cloth(512)
    Pd = mas_amd.from_mesh(mesh, max_levels=3)
    Pr = mas_amd.from_mesh(mesh, max_levels=3, reference_formation=True)
    assert Pd.stats()["factor_formation"] == 1 and Pr.stats()["factor_formation"] == 0
    info = Pd.info()
    blocks = list(range(0, info["num_fine_blocks"], 8)) + list(range(info["num_fine_blocks"], info["num_blocks"]))
    worst = 0.0
    for blk in blocks:
        a, b = Pr.block_inverse(blk), Pd.block_inverse(blk)
        worst = max(worst, float(np.linalg.norm(b - a) / max(np.linalg.norm(a), 1e-30)))
    print(f"256k: {len(blocks)} blocks, worst inverse rel. difference {worst:.2e}")
    assert worst <= 2e-5, worst
