"""Fixture / wire format (mas_save_blob / mas_load_blob).

Bars: a restored handle applies bitwise-identically to the handle that was
saved, reports the same maps, level sizes and inverses; corrupted or
truncated blobs are rejected; a restored handle refuses Prepare until
mas_allocate; the committed golden blob (tests/golden/cloth12_L0.masblob,
scripts/make_golden_blob.py) is reproduced byte for byte on this box.
"""
import os

import numpy as np
import pytest

from conftest import REPO, cloth

pytestmark = pytest.mark.gpu


def _prepared(mesh, L=0, contacts=None, reference_formation=False):
    import mas_amd
    return mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts, reference_formation=reference_formation)


@pytest.mark.parametrize("W,L,nc", [(64, 0, 200), (100, 3, 0)])
def test_blob_roundtrip_bitwise(W, L, nc):
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(W)
    contacts = meshgen.vf_contacts(mesh, nc) if nc else None
    P = _prepared(mesh, L, contacts)
    blob = P.save_blob()
    Q = mas_amd.SeSchwarzPreconditioner()
    Q.load_blob(blob)
    ip, iq = P.info(), Q.info()
    for k in ("num_verts", "num_levels", "total_clusters", "num_blocks", "num_fine_blocks", "num_stencils"):
        assert ip[k] == iq[k], k
    np.testing.assert_array_equal(ip["level_size"], iq["level_size"])
    mp, mq = P.maps(), None
    import ctypes
    n = mesh.nV
    out = dict(morton=np.zeros(n, np.uint64), s2o=np.zeros(n, np.int32), o2s=np.zeros(n, np.int32))
    Q._check(Q._L.mas_get_maps(Q.h, *[mas_amd._ptr(out[k]) for k in ("morton", "s2o", "o2s")], None, None, None,
                               None), "get_maps")
    for k in out:
        np.testing.assert_array_equal(out[k], mp[k])
    for blk in range(ip["num_blocks"]):
        np.testing.assert_array_equal(Q.block_inverse(blk), P.block_inverse(blk))
    r = meshgen.residual(n, 31)
    np.testing.assert_array_equal(Q.Preconditioning(None, r), P.Preconditioning(None, r))
    # the blob of the restored handle is the same blob
    np.testing.assert_array_equal(Q.save_blob(), blob)
    # a restored handle has no Prepare inputs
    with pytest.raises(mas_amd.MasError, match="STATE"):
        Q.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    # ... until it is allocated again, then it behaves like a fresh handle
    Q.m_positions, Q.m_neighbours, Q.m_edges, Q.m_faces = mesh.pos, (mesh.starts, mesh.idx), mesh.edges, mesh.faces
    Q.AllocatePrecoditioner(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0])
    if contacts is None:
        Q.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    else:
        Q.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, contacts[0], None, None, contacts[1])
    np.testing.assert_allclose(Q.Preconditioning(None, r), P.Preconditioning(None, r), rtol=0, atol=1e-6)


def test_blob_rejects_damage():
    import mas_amd
    mesh = cloth(20)
    blob = _prepared(mesh).save_blob()
    Q = mas_amd.SeSchwarzPreconditioner()
    bad = blob.copy()
    bad[len(bad) // 2] ^= 0x40
    with pytest.raises(mas_amd.MasError, match="checksum"):
        Q.load_blob(bad)
    bad = blob.copy()
    bad[0] = ord("X")
    with pytest.raises(mas_amd.MasError, match="magic"):
        Q.load_blob(bad)
    with pytest.raises(mas_amd.MasError):
        Q.load_blob(blob[: len(blob) - 16])
    with pytest.raises(mas_amd.MasError, match="STATE"):
        Q.Preconditioning(None, np.zeros((mesh.nV, 4), np.float32))
    Q.load_blob(blob)  # the handle is still usable
    assert Q.info()["num_verts"] == mesh.nV


def test_golden_blob_reproduced():
    """Cross-box golden comparison: this box's Allocate + Prepare of the 12x12
    grid gives the committed blob byte for byte (maps, inverses, checksum)."""
    golden = np.fromfile(os.path.join(REPO, "tests", "golden", "cloth12_L0.masblob"), dtype=np.uint8)
    blob = _prepared(cloth(12), reference_formation=True).save_blob()   # inverses in the reference's order
    assert blob.nbytes == golden.nbytes
    np.testing.assert_array_equal(blob, golden)


def _fnv1a(buf):
    h = 1469598103934665603
    for b in buf.tobytes():
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def test_blob_rejects_out_of_range_maps():
    """A blob whose checksum is valid but whose index maps point outside the
    level table (a crafted file: FNV-1a is no tamper check) is refused before
    the handle is touched."""
    import mas_amd
    mesh = cloth(16)
    P = _prepared(mesh)
    blob = P.save_blob()
    header_bytes = int(blob[12:16].view(np.uint32)[0])
    n_sec = int(blob[128:132].view(np.int32)[0])
    table = blob[header_bytes:header_bytes + 24 * n_sec].reshape(n_sec, 24)
    sec = {int(t[:4].view(np.uint32)[0]): (int(t[8:16].view(np.uint64)[0]), int(t[16:24].view(np.uint64)[0]))
           for t in table}
    Q = mas_amd.SeSchwarzPreconditioner()
    Q.load_blob(blob)
    for sid, word in ((8, 1), (2, 5), (5, 3)):  # vmap ancestor, s2o, goingNext
        bad = blob.copy()
        nbytes, off = sec[sid]
        bad[off + 4 * word: off + 4 * word + 4] = np.array([1 << 28], np.int32).view(np.uint8)
        bad[144:152] = np.array([_fnv1a(bad[header_bytes:])], np.uint64).view(np.uint8)
        with pytest.raises(mas_amd.MasError, match="out of range"):
            Q.load_blob(bad)
        # the handle still holds the last good blob and applies
        r = np.ones((mesh.nV, 4), np.float32)
        np.testing.assert_array_equal(Q.Preconditioning(None, r), P.Preconditioning(None, r))


def test_wrappers_reject_bad_operands():
    """Shape / dtype / layout checks before the C ABI copies nV*16 bytes."""
    import torch
    import mas_amd
    mesh = cloth(16)
    P = _prepared(mesh)
    n = mesh.nV
    with pytest.raises(mas_amd.MasError, match="residual"):
        P.Preconditioning(None, np.zeros((n, 3), np.float32))
    with pytest.raises(mas_amd.MasError, match="z must be"):
        P.Preconditioning(np.zeros((n, 4), np.float64), np.zeros((n, 4), np.float32))
    with pytest.raises(mas_amd.MasError, match="csrOffDiagonals"):
        P.PreparePreconditioner(mesh.diag, mesh.off[:-1], mesh.starts)
    r = torch.zeros((n, 4), device="cuda")
    with pytest.raises(mas_amd.MasError, match="contiguous"):
        P.PreconditioningDevice(torch.zeros((4, n), device="cuda").t(), r)
    with pytest.raises(mas_amd.MasError, match="float32"):
        P.PreconditioningDevice(torch.zeros((n, 4), device="cuda", dtype=torch.float64), r)
    with pytest.raises(mas_amd.MasError, match="not on a GPU"):
        P.PreconditioningDevice(torch.zeros((n, 4)), r)
    with pytest.raises(mas_amd.MasError, match="elements"):
        P.PreconditioningDevice(torch.zeros((n - 1, 4), device="cuda"), r)
