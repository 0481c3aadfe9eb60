"""Loud failures (SURVEY section 5 "failure detection").

* A block whose LDL^T meets a zero, negative or non-finite pivot: with
  mas_config.strict_spd = 1 Prepare fails with MAS_ERR_NOT_SPD; by default it
  keeps going as the reference does (its method is void and divides by such
  pivots unchecked, .cpp:1406,1431) with a MasWarning.  Either way
  mas_stats.nonspd_blocks counts the blocks, the handle stays prepared, and
  the next SPD Prepare is clean.
* A bounded hand-off wait of the one-launch coarse form that gives up
  (forced here with MAS_C1_POLL_LIMIT=-1) makes the synchronous apply fail
  with MAS_ERR_HIP and is counted in mas_stats.wait_timeouts; after a device
  apply that gave up, the next device apply reports it (no stream sync).
Each case is run once.
"""
import os

import numpy as np
import pytest

from conftest import cloth

pytestmark = pytest.mark.gpu


def _handle(mesh, L=0, env=None, **kw):
    import mas_amd
    saved = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        P = mas_amd.SeSchwarzPreconditioner(max_levels=L, **kw)
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    P.m_positions = mesh.pos
    P.m_neighbours = (mesh.starts, mesh.idx)
    P.m_edges = mesh.edges
    P.m_faces = mesh.faces
    P.AllocatePrecoditioner(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0])
    return P


@pytest.mark.parametrize("strict", [True, False])
@pytest.mark.parametrize("how", ["nan", "negative"])
@pytest.mark.parametrize("reference_formation", [False, True])
def test_singular_block_is_not_spd(how, reference_formation, strict):
    import warnings
    import mas_amd
    mesh = cloth(40)
    P = _handle(mesh, reference_formation=reference_formation, strict_spd=strict)
    P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    assert P.stats()["nonspd_blocks"] == 0
    bad = mesh.diag.copy()
    v = 777
    if how == "nan":
        bad[v, 0] = np.nan
    else:
        bad[v] = -bad[v] - 50.0 * np.eye(3, dtype=np.float32).reshape(9)  # an indefinite diagonal block
    if strict:
        with pytest.raises(mas_amd.MasError, match="NOT_SPD") as e:
            P.PreparePreconditioner(bad, mesh.off, mesh.starts)
    else:  # the reference's behaviour: the Prepare goes through, the facade warns
        with pytest.warns(mas_amd.MasWarning, match="not SPD") as e:
            P.PreparePreconditioner(bad, mesh.off, mesh.starts)
        z = P.Preconditioning(None, np.ones((mesh.nV, 4), np.float32))  # the handle applies
        assert z.shape == (mesh.nV, 4)
    st = P.stats()
    assert st["nonspd_blocks"] >= 1
    print(how, reference_formation, strict, "blocks:", st["nonspd_blocks"], e)
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # an SPD Prepare again: no warning, no error
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    assert P.stats()["nonspd_blocks"] == 0


def test_forced_wait_timeout_fails_the_apply():
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(256)  # 64k vertices, L = 3: the one-launch coarse form (k_coarse1)
    r = meshgen.residual(mesh.nV, 3)
    ok = _handle(mesh, 3, env={"MAS_COARSE_MODE": "3"})
    ok.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    z = ok.Preconditioning(None, r)
    assert ok.stats()["wait_timeouts"] == 0
    P = _handle(mesh, 3, env={"MAS_COARSE_MODE": "3", "MAS_C1_POLL_LIMIT": "-1"})
    P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    assert P.stats()["apply_mode"] == 3
    with pytest.raises(mas_amd.MasError, match="gave up"):
        P.Preconditioning(None, r)
    n = P.stats()["wait_timeouts"]
    assert n >= 1
    print("timeouts counted:", n)
    # the default limit on the same handle's configuration stays silent and exact
    np.testing.assert_array_equal(ok.Preconditioning(None, r), z)
    assert ok.stats()["wait_timeouts"] == 0


def test_device_apply_giveup_reported_by_next_call():
    """mas_apply_device is asynchronous: an apply whose bounded wait gave up
    is named (MAS_ERR_HIP, its epoch) by the next apply call on the handle,
    which reads a pinned host word (no stream sync) and queues nothing; the
    call after that runs normally.  mas_get_stats counts the waits without a
    device-wide synchronisation."""
    import torch
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(256)
    r = torch.from_numpy(meshgen.residual(mesh.nV, 5)).cuda()
    z = torch.zeros_like(r)
    P = _handle(mesh, 3, env={"MAS_COARSE_MODE": "3", "MAS_C1_POLL_LIMIT": "-1"})
    P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    s = torch.cuda.Stream()
    P.PreconditioningDevice(z, r, s.cuda_stream)  # gives up on the device; the call itself returns MAS_OK
    s.synchronize()
    with pytest.raises(mas_amd.MasError, match=r"MAS_ERR_HIP.*apply #\d+ .*gave up"):
        P.PreconditioningDevice(z, r, s.cuda_stream)
    assert P.stats()["wait_timeouts"] >= 1
    P.PreconditioningDevice(z, r, s.cuda_stream)  # reported once; this one runs (and gives up again)
    s.synchronize()
    with pytest.raises(mas_amd.MasError, match="gave up"):  # the host apply names the earlier device apply first
        P.Preconditioning(None, r.cpu().numpy())


@pytest.mark.skipif("__import__('torch').cuda.device_count() < 2", reason="needs two GPUs")
def test_shard_entry_points_select_the_handle_device():
    """mas_apply_shard_* select the handle's device themselves (a caller whose
    current device is another GPU)."""
    import torch
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(128)
    P = mas_amd.from_mesh(mesh, max_levels=3, device=1)
    r = torch.from_numpy(meshgen.residual(mesh.nV, 1)).cuda(1)
    z, z_ref = torch.zeros_like(r), torch.zeros_like(r)
    P.PreconditioningDevice(z_ref, r)
    plan = P.shard_setup(0, 1)
    seg = torch.zeros((plan["seg_max"], 4), dtype=torch.float32, device="cuda:1")
    torch.cuda.set_device(0)
    P.shard_restrict(0, 1, r, seg)
    P.shard_fine(0, 1, r, z)
    P.shard_complete(0, 1, seg.clone(), z)
    torch.cuda.synchronize(1)
    assert torch.equal(z, z_ref)
