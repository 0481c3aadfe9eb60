"""GPU-resident PCG (k_pcg.hip, mas_pcg_solve*) -- the caller of the apply.

Bars:
  * iteration counts within max(3, 5 %) of a float64 numpy PCG driven by the
    CPU oracle's preconditioner on the same right-hand side (the GPU loop runs
    fp32 vectors with fp64 dot products, so counts may differ by a few) --
    compared at the iteration where the recursive residual first met tol,
    which is where an fp64 PCG stops; driving the returned fp32 x's own
    residual below tol (its rounding floor is 5.9e-6 on the 100x100 grid)
    may take a few more, held to 15 % + 5;
  * the SURVEY §4 known answer: MAS / unpreconditioned iteration ratio on the
    100x100 grid in the reference's band (0.21 at 3 levels, 0.44 at 1 level);
  * the returned x satisfies ||b - A x|| <= tol ||b||: the solver replaces
    the drifting fp32 recursive residual by b - A x whenever the recursive test
    passes and stops only on the true one (the float64 recomputation here may
    differ from the fp32 one in the last digits: 1.1 tol), and the library's
    own true-residual report agrees with the float64 one;
  * the apply hooks of a solve (done flag, r.z partials) are gone afterwards:
    a plain apply after a solve equals one before it;
  * run-to-run bitwise determinism, host and device entry points equal.
"""
import numpy as np
import pytest

from conftest import cloth, tet
from test_oracle_math import _pcg_iters, hessian_sorted

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _setup(mesh, L):
    import mas_amd
    return mas_amd.from_mesh(mesh, max_levels=L)


def _true_rel_res(mesh, x, b):
    A = hessian_sorted(mesh, np.arange(mesh.nV), np.arange(mesh.nV))
    xv = x[:, :3].astype(np.float64).ravel()
    bv = b[:, :3].astype(np.float64).ravel()
    return float(np.linalg.norm(bv - A @ xv) / np.linalg.norm(bv))


# SURVEY §4 known answers (reference probe, fp64 PCG, tol 1e-5): 100^2 / L3
# 526 -> 110 (0.21), 100^2 / L1 526 -> 232 (0.44), 256^2 / L4 515 -> 93
# (0.18).  The probe's right-hand side was not recorded, so the ratio is held
# to a band around it.
@pytest.mark.parametrize("W,L,band", [(100, 3, (0.15, 0.30)), (100, 1, (0.35, 0.60)), (256, 4, (0.13, 0.25))])
def test_pcg_iterations_match_cpu_and_known_answer(W, L, band):
    from mas_amd import meshgen
    from oracle import Oracle
    mesh = cloth(W)
    P = _setup(mesh, L)
    b = meshgen.residual(mesh.nV, 0x5EED)
    x, res = P.pcg_solve(mesh.diag, mesh.off, mesh.starts, b, max_iters=3000, tol=TOL)
    assert res["converged"], res
    assert res["true_rel_residual"] <= TOL, res
    tr = _true_rel_res(mesh, x, b)
    assert tr <= 1.1 * TOL, (tr, res)
    assert abs(res["true_rel_residual"] - tr) <= 0.05 * tr + 1e-7, (res, tr)
    x0, res0 = P.pcg_solve(mesh.diag, mesh.off, mesh.starts, b, max_iters=3000, tol=TOL, precondition=False)
    assert res0["converged"], res0
    # CPU: float64 PCG with the oracle's apply
    o = Oracle(mesh.nV, 0, 0, L, 4)
    o.allocate(mesh)
    o.prepare(mesh)
    A = hessian_sorted(mesh, np.arange(mesh.nV), np.arange(mesh.nV))
    bv = b[:, :3].astype(np.float64).ravel()

    def prec(v):
        r4 = np.zeros((mesh.nV, 4), np.float32)
        r4[:, :3] = v.reshape(-1, 3)
        return o.apply(r4)[:, :3].astype(np.float64).ravel()

    it_cpu = _pcg_iters(A, bv, prec, tol=TOL)
    it_cpu0 = _pcg_iters(A, bv, lambda v: v, tol=TOL)
    for rs, ic in ((res, it_cpu), (res0, it_cpu0)):
        first = rs["first_pass_iterations"]
        assert abs(first - ic) <= max(3, 0.05 * ic), (rs, ic)
        assert first <= rs["iterations"] <= 1.15 * first + 5, rs
        assert rs["replacements"] >= 1, rs
    assert res0["true_rel_residual"] <= TOL, res0
    ratio = res["first_pass_iterations"] / res0["first_pass_iterations"]
    assert band[0] <= ratio <= band[1], (res, res0, ratio)


def test_pcg_deterministic_and_device_path():
    import torch
    from mas_amd import meshgen
    mesh = tet(12)
    P = _setup(mesh, 0)
    b = meshgen.residual(mesh.nV, 3)
    z_before = P.Preconditioning(None, b)
    x1, r1 = P.pcg_solve(mesh.diag, mesh.off, mesh.starts, b, max_iters=500, tol=TOL)
    np.testing.assert_array_equal(P.Preconditioning(None, b), z_before)
    x2, r2 = P.pcg_solve(mesh.diag, mesh.off, mesh.starts, b, max_iters=500, tol=TOL)
    # valence 14: the 16-lane SpMV over the ELL copy of the CSR blocks
    assert r1["converged"], r1
    assert _true_rel_res(mesh, x1, b) <= 1.1 * TOL
    np.testing.assert_array_equal(x1, x2)
    assert r1["iterations"] == r2["iterations"]
    dd = torch.from_numpy(np.ascontiguousarray(mesh.diag, np.float32)).cuda()
    do = torch.from_numpy(np.ascontiguousarray(mesh.off, np.float32)).cuda()
    dr = torch.from_numpy(np.ascontiguousarray(mesh.starts, np.int32)).cuda()
    db = torch.from_numpy(b).cuda()
    dx = torch.zeros_like(db)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    r3 = P.pcg_solve_device(dd, do, dr, dx, db, max_iters=500, tol=TOL, stream=s.cuda_stream)
    s.synchronize()
    np.testing.assert_array_equal(dx.cpu().numpy(), x1)
    assert r3["iterations"] == r1["iterations"]
    assert np.all(x1[:, 3] == 0)


def test_pcg_edge_cases():
    from mas_amd import meshgen
    mesh = cloth(20)
    P = _setup(mesh, 0)
    zero = np.zeros((mesh.nV, 4), np.float32)
    x, res = P.pcg_solve(mesh.diag, mesh.off, mesh.starts, zero, max_iters=100, tol=TOL)
    assert res["iterations"] == 0 and np.all(x == 0)
    b = meshgen.residual(mesh.nV, 9)
    x, res = P.pcg_solve(mesh.diag, mesh.off, mesh.starts, b, max_iters=2, tol=1e-12)
    assert res["iterations"] == 2 and not res["converged"]
    # a converged x as the initial guess stops immediately
    xs, rs = P.pcg_solve(mesh.diag, mesh.off, mesh.starts, b, max_iters=500, tol=TOL)
    x2, r2 = P.pcg_solve(mesh.diag, mesh.off, mesh.starts, b, x0=xs, max_iters=500, tol=10 * TOL)
    assert r2["iterations"] <= 1


@pytest.mark.parametrize("W,L,precondition,maxit", [(100, 3, True, 3000), (256, 4, True, 3000), (100, 3, False, 3000),
                                                    (100, 3, True, 7), (101, 3, True, 3000), (101, 3, False, 3000)])
def test_pcg_fused_p_update_bitwise(W, L, precondition, maxit, monkeypatch):
    """p = z + beta p inside the next SpMV (MAS_PCG_FUSE_P=1, the default) and
    as its own pass (0): the same iterates bit for bit -- x, the iteration
    counts, the replacements, the residuals -- also when max_iters stops the
    solve (the last decision then runs after the loop).  W = 101: an odd
    vertex count (the second p buffer's offset must stay 16-byte aligned)."""
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(W)
    b = meshgen.residual(mesh.nV, 11)
    out = []
    for fuse in ("0", "1"):
        monkeypatch.setenv("MAS_PCG_FUSE_P", fuse)
        P = mas_amd.from_mesh(mesh, max_levels=L)
        x, res = P.pcg_solve(mesh.diag, mesh.off, mesh.starts, b, max_iters=maxit, tol=TOL,
                             precondition=precondition)
        out.append((x, res))
    (x0, r0), (x1, r1) = out
    assert np.array_equal(x0.view(np.uint32), x1.view(np.uint32))
    for k in ("iterations", "converged", "replacements", "first_pass_iterations", "rel_residual", "true_rel_residual"):
        assert r0[k] == r1[k], (k, r0[k], r1[k])
    if maxit == 7:
        assert r1["iterations"] == 7 and not r1["converged"]


@pytest.mark.parametrize("W,L", [(100, 3), (256, 4)])
def test_inverse_load_policy_bitwise(W, L, monkeypatch):
    """The fine kernel's inverse loads, nontemporal (MAS_INV_RESIDENT=0) or
    default policy (1; chosen by size where the inverses fit the Infinity
    Cache): the same z and the same PCG iterates bit for bit (the r.z partials
    come from workgroups of 4 blocks either way)."""
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(W)
    b = meshgen.residual(mesh.nV, 13)
    out = []
    for res_mode in ("0", "1"):
        monkeypatch.setenv("MAS_INV_RESIDENT", res_mode)
        P = mas_amd.from_mesh(mesh, max_levels=L)
        z = P.Preconditioning(None, b)
        x, res = P.pcg_solve(mesh.diag, mesh.off, mesh.starts, b, max_iters=3000, tol=TOL)
        out.append((z, x, res))
    (z0, x0, r0), (z1, x1, r1) = out
    assert np.array_equal(z0.view(np.uint32), z1.view(np.uint32))
    assert np.array_equal(x0.view(np.uint32), x1.view(np.uint32))
    assert r0["iterations"] == r1["iterations"] and r0["true_rel_residual"] == r1["true_rel_residual"]


@pytest.mark.parametrize("kind,W,L,precondition,fuse,perturb", [
    ("cloth", 100, 3, True, "1", False), ("cloth", 256, 4, True, "1", False), ("cloth", 101, 3, False, "1", False),
    ("cloth", 100, 3, True, "0", False), ("tet", 14, 3, True, "1", False), ("cloth", 100, 3, True, "1", True)])
def test_pcg_mirrored_layout_bitwise(kind, W, L, precondition, fuse, perturb, monkeypatch):
    """The SpMV's mirrored layout (MAS_PCG_SYM=1, an A/B: a group's lower
    blocks that are bitwise transposes of an upper block in the same wave row
    are not stored; the upper block's lane forms their products, k_pcg_ell /
    k_pcg_spmv) against every block stored (0, the default): the same iterates bit for
    bit -- x, the iteration counts, the residuals -- on cloth (G = 8, a
    quarter of the slots mirrored), tet (G = 16), an odd vertex count, the
    unfused p update, and a Hessian made non-symmetric in every fifth block
    (those pairs stay stored)."""
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(W) if kind == "cloth" else tet(W)
    off = mesh.off
    if perturb:
        off = mesh.off.copy()
        off[::5] *= np.float32(1 + 2 ** -20)
    b = meshgen.residual(mesh.nV, 23)
    monkeypatch.setenv("MAS_PCG_FUSE_P", fuse)
    out = []
    for sym in ("0", "1"):
        monkeypatch.setenv("MAS_PCG_SYM", sym)
        P = mas_amd.from_mesh(mesh, max_levels=L)
        x, res = P.pcg_solve(mesh.diag, off, mesh.starts, b, max_iters=400 if perturb else 3000, tol=TOL,
                             precondition=precondition)
        out.append((x, res))
    (x0, r0), (x1, r1) = out
    assert np.array_equal(x0.view(np.uint32), x1.view(np.uint32))
    for k in ("iterations", "converged", "replacements", "first_pass_iterations", "rel_residual", "true_rel_residual"):
        assert r0[k] == r1[k], (k, r0[k], r1[k])
    if not perturb:
        assert r1["converged"]
