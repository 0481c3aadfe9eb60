"""Loud failures (SURVEY section 5 "failure detection").

* A block whose LDL^T meets a zero, negative or non-finite pivot makes
  Prepare fail with MAS_ERR_NOT_SPD (the reference divides by such pivots
  unchecked, .cpp:1406,1431); mas_stats.nonspd_blocks counts the blocks, the
  handle stays prepared, and the next SPD Prepare succeeds.
* A bounded hand-off wait of the one-launch coarse form that gives up
  (forced here with MAS_C1_POLL_LIMIT=-1) makes the synchronous apply fail
  with MAS_ERR_HIP and is counted in mas_stats.wait_timeouts.
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


@pytest.mark.parametrize("how", ["nan", "negative"])
@pytest.mark.parametrize("reference_formation", [False, True])
def test_singular_block_is_not_spd(how, reference_formation):
    import mas_amd
    mesh = cloth(40)
    P = _handle(mesh, reference_formation=reference_formation)
    P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    assert P.stats()["nonspd_blocks"] == 0
    bad = mesh.diag.copy()
    v = 777
    if how == "nan":
        bad[v, 0] = np.nan
    else:
        bad[v] = -bad[v] - 50.0 * np.eye(3, dtype=np.float32).reshape(9)  # an indefinite diagonal block
    with pytest.raises(mas_amd.MasError, match="NOT_SPD") as e:
        P.PreparePreconditioner(bad, mesh.off, mesh.starts)
    st = P.stats()
    assert st["nonspd_blocks"] >= 1
    print(how, reference_formation, "blocks:", st["nonspd_blocks"], e.value)
    P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)  # SPD again
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
