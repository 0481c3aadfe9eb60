"""The fused apply (coarseMode 4: coarse levels and level-0 blocks in one
launch, k_coarse1.hip k_apply_fused) against the one-launch coarse form +
k_solve_fine (coarseMode 3): z bitwise equal, at the BASELINE configs, over
repeated applies with changing residuals (the solved count is cumulative),
with fine workgroups started beside the coarse chain (MAS_FUSE_EARLY: their
waves wait for the tagged coarse Z), and without hold workgroups at all
(MAS_FUSE_HOLD=0: every fine wave may start beside the chain).
"""
import os

import numpy as np
import pytest

from conftest import cloth

pytestmark = pytest.mark.gpu


def _handle(mesh, L, mode, contacts=None, env=None, **kw):
    import mas_amd
    env = dict(env or {}, MAS_COARSE_MODE=str(mode))
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts, **kw)
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _applies(P, rs):
    import torch
    s = torch.cuda.Stream()
    out = []
    for r in rs:
        rd = torch.from_numpy(r).cuda()
        zd = torch.full_like(rd, float("nan"))
        torch.cuda.synchronize()
        P.PreconditioningDevice(zd, rd, s.cuda_stream)
        s.synchronize()
        out.append(zd.cpu().numpy())
    return out


def _compare(mesh, L, contacts=None, n=4, env=None, **kw):
    from mas_amd import meshgen
    rs = [meshgen.residual(mesh.nV, 100 + k) for k in range(n)]
    A = _handle(mesh, L, 3, contacts, **kw)
    B = _handle(mesh, L, 4, contacts, env=env, **kw)
    assert A.stats()["apply_mode"] == 3 and B.stats()["apply_mode"] == 4
    za, zb = _applies(A, rs), _applies(B, rs)
    for k, (x, y) in enumerate(zip(za, zb)):
        bad = np.flatnonzero(np.any(x.view(np.uint32) != y.view(np.uint32), axis=1))
        assert bad.size == 0, (k, bad[:5], x[bad[:3]], y[bad[:3]])
    assert B.stats()["wait_timeouts"] == 0


@pytest.mark.parametrize("config", ["256k", "1M+contacts", "4M-tet"])
def test_fused_bitwise_baseline_configs(config):
    from mas_amd import meshgen
    mesh, cfg = meshgen.build_config(config)
    contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
    _compare(mesh, cfg["levels"], contacts, n=3)


@pytest.mark.parametrize("W,L", [(256, 3), (256, 4), (200, 4), (128, 3)])
def test_fused_bitwise_small(W, L):
    _compare(cloth(W), L, n=5)


@pytest.mark.parametrize("W,L", [(256, 4), (128, 3)])
def test_fused_without_holds(W, L):
    """No hold workgroups: fine waves run beside the chain and wait for it."""
    _compare(cloth(W), L, n=3, env={"MAS_FUSE_HOLD": "0"})


def test_fused_reference_formation():
    from mas_amd import meshgen
    mesh = cloth(512)
    _compare(mesh, 3, meshgen.vf_contacts(mesh, 20000, seed=9), n=2, reference_formation=True)


@pytest.mark.parametrize("early", [64, 100000])
def test_fused_early_fine_waves(early):
    """Fine workgroups beside the coarse chain (MAS_FUSE_EARLY): their waves
    wait for the tagged coarse Z; 100000 = every fine workgroup early."""
    from mas_amd import meshgen
    mesh, cfg = meshgen.build_config("1M+contacts")
    contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3)
    _compare(mesh, cfg["levels"], contacts, n=3, env={"MAS_FUSE_EARLY": str(early)})
