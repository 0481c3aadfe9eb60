"""The reference C++ surface end to end: a PCG caller compiled against
include/SeSchwarzPreconditioner.h and linked to libSeSchwarzPreconditioner.so
(the HIP path), compared with the oracle on the same inputs."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, cloth

pytestmark = pytest.mark.gpu


def test_cpp_facade_pcg(tmp_path):
    import mas_amd
    from mas_amd import meshgen
    from oracle import Oracle
    mesh = cloth(64)
    r = meshgen.residual(mesh.nV, 0x5EED)
    for name, arr in (("pos", mesh.pos), ("starts", mesh.starts), ("idx", mesh.idx), ("diag", mesh.diag),
                      ("off", mesh.off), ("r", r)):
        np.ascontiguousarray(arr).tofile(tmp_path / f"{name}.bin")
    exe = tmp_path / "facade_pcg"
    lib = os.path.dirname(mas_amd.FACADE_PATH)
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "cpp", "facade_pcg.cpp"), "-L", lib, "-lSeSchwarzPreconditioner",
                    "-lmas_amd", f"-Wl,-rpath,{lib}", "-o", str(exe)], check=True)
    try:
        out = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=90,
                             check=True).stdout
    except subprocess.TimeoutExpired as e:  # say how far it got
        raise AssertionError(f"facade_pcg timed out; stdout so far: {e.stdout!r} stderr: {e.stderr!r}")
    z = np.fromfile(tmp_path / "z.bin", dtype=np.float32).reshape(-1, 4)
    o = Oracle(mesh.nV, 0, 0, 0, 1)
    o.allocate(mesh)
    o.prepare(mesh)
    z_ref = o.apply(r)
    err = np.linalg.norm(z[:, :3] - z_ref[:, :3]) / np.linalg.norm(z_ref[:, :3])
    assert err <= 1e-5, err
    # Preconditioning / PreparePreconditioner repeated through the same host
    # arrays: bitwise the first z
    assert "host_repeat_bitwise 1" in out, out
    iters = int(out.split("pcg_iterations")[1])
    assert 20 < iters < 200, out


def _page_aligned(a):
    n = a.nbytes
    buf = np.empty(n + (-n) % 4096 + 4096, np.uint8)
    off = (-buf.ctypes.data) % 4096
    v = buf[off:off + n].view(a.dtype).reshape(a.shape)
    v[...] = a
    return v


@pytest.mark.parametrize("aligned", [True, False])
def test_host_register_bitwise(aligned):
    """mas_config.host_register = 1 (mas_capi.hip pin_host): the host arrays
    passed a second time are page-locked (page-aligned ones only) and the
    copies run from them; Prepare and apply through the same arrays three
    times give z bitwise the default handle's (pageable staging), and a fresh
    array per call (never registered) too."""
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(100)
    r = meshgen.residual(mesh.nV, 29)
    P0 = mas_amd.from_mesh(mesh, max_levels=3)
    z0 = P0.Preconditioning(None, r)
    cp = _page_aligned if aligned else (lambda a: a.copy())
    diag, off, starts, rr = cp(mesh.diag), cp(mesh.off), cp(mesh.starts), cp(r)
    z = cp(np.zeros_like(r))
    P1 = mas_amd.SeSchwarzPreconditioner(max_levels=3, host_register=True)
    P1.m_positions = mesh.pos
    P1.m_neighbours = (mesh.starts, mesh.idx)
    P1.m_edges = mesh.edges
    P1.m_faces = mesh.faces
    P1.AllocatePrecoditioner(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0])
    for _ in range(3):
        P1.PreparePreconditioner(diag, off, starts)
        z[...] = 0
        P1.Preconditioning(z, rr)
        assert np.array_equal(z.view(np.uint32), z0.view(np.uint32))
    for _ in range(2):
        zf = P1.Preconditioning(None, rr.copy())
        assert np.array_equal(zf.view(np.uint32), z0.view(np.uint32))
    del P1
    # the arrays stay usable after the handle released them
    assert np.array_equal(diag, mesh.diag)
