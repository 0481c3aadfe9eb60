"""Every way Prepare can be scheduled produces the same handle, byte for byte.

Round 3 moved the level-0 work off Prepare's critical path
(`run_level0_early`, k_assemble.hip): the level-0 contact records, their sorts
and folds and the fused assemble + factor kernel start on a side queue
right after the stencils, and the coarse contact path skips the level-0
records.  The orders of every record and every sum are unchanged, so the
saved blob (maps + every packed inverse, blob.hip) must be identical whatever
the schedule: the early path queued from a second host thread or from the
level build's hook, with `od` in the early path or on the coarse chain, the
fused kernel before or after the level build, in one launch or in chunks
(round 6's default, launch_factor_fused), with or without CUs reserved,
and the round-2 late path (`keep_blocks`, which stores the level-0 blocks and so cannot start before
the levels are known).  Each handle is prepared twice (steady state), and the
apply must agree bitwise as well.
"""
import numpy as np
import pytest

from conftest import cloth, tet

pytestmark = pytest.mark.gpu

VARIANTS = [
    {},
    {"MAS_EARLY_THREAD": "0"},
    {"MAS_EARLY_OD": "1"},
    {"MAS_FUSED_AFTER_LEVELS": "1"},
    {"MAS_PREP_CU_RESERVE": "32"},
    {"MAS_FUSED_CHUNKS": "1"},
    {"MAS_FUSED_CHUNKS": "3"},
]


def _prepared(mesh, L, contacts, env, monkeypatch, keep_blocks=False):
    import mas_amd
    for k in ("MAS_EARLY_THREAD", "MAS_EARLY_OD", "MAS_FUSED_AFTER_LEVELS", "MAS_PREP_CU_RESERVE", "MAS_FUSED_CHUNKS"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    P = mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts, keep_blocks=keep_blocks)
    # a second, steady-state Prepare on the same handle
    if contacts is None:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    else:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, contacts[0], None, None, contacts[1])
    return P


def _z(P, r):
    import torch
    z = torch.zeros_like(r)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    P.PreconditioningDevice(z, r, s.cuda_stream)
    s.synchronize()
    return z.cpu().numpy()


@pytest.mark.parametrize("kind,W,L,nc", [("cloth", 256, 4, 3000), ("cloth", 100, 3, 500), ("tet", 24, 4, 0)])
def test_prepare_schedules_bitwise(kind, W, L, nc, monkeypatch):
    import torch
    from mas_amd import meshgen
    mesh = cloth(W) if kind == "cloth" else tet(W)
    contacts = meshgen.vf_contacts(mesh, nc, seed=7) if nc else None
    r = torch.from_numpy(meshgen.residual(mesh.nV, 17)).cuda()
    ref = _prepared(mesh, L, contacts, VARIANTS[0], monkeypatch)
    blob_ref, z_ref = ref.save_blob(), _z(ref, r)
    for env in VARIANTS[1:]:
        P = _prepared(mesh, L, contacts, env, monkeypatch)
        assert np.array_equal(P.save_blob(), blob_ref), env
        np.testing.assert_array_equal(_z(P, r), z_ref, err_msg=str(env))
        del P  # a CU-masked queue (the opt-in reserve) goes with its handle
    # the late path (level-0 blocks stored, fused kernel forked after the levels)
    K = _prepared(mesh, L, contacts, {}, monkeypatch, keep_blocks=True)
    np.testing.assert_array_equal(_z(K, r), z_ref)
    ib = ref.info()["num_fine_blocks"]
    for b in (0, ib // 2, ib - 1):
        np.testing.assert_array_equal(K.block_inverse(b), ref.block_inverse(b), err_msg=f"block {b}")
