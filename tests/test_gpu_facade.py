"""The reference C++ surface end to end: a PCG caller compiled against
include/SeSchwarzPreconditioner.h and linked to libSeSchwarzPreconditioner.so
(the HIP path), compared with the oracle on the same inputs."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, cloth

pytestmark = pytest.mark.gpu


def _diag(pid):
    """What a stuck process is doing: each thread's state, wait channel and
    system call (/proc), and the GPU's activity."""
    lines = []
    for t in sorted(os.listdir(f"/proc/{pid}/task")):
        def rd(name):
            try:
                with open(f"/proc/{pid}/task/{t}/{name}") as f:
                    return f.read().strip()
            except OSError as e:
                return f"<{e.__class__.__name__}>"
        lines.append(f"task {t} {rd('comm')} state={rd('stat').split(') ')[-1][:1]} wchan={rd('wchan')} "
                     f"syscall={rd('syscall').split(' ')[0]}")
    for who, q in (("child", pid), ("parent", os.getpid())):
        try:
            lines.append(f"kfd queues of the {who}: {len(os.listdir(f'/sys/class/kfd/kfd/proc/{q}/queues'))}")
        except OSError as e:
            lines.append(f"kfd queues of the {who}: <{e.__class__.__name__}>")
    try:
        smi = subprocess.run(["rocm-smi", "--showuse", "--showmemuse"], capture_output=True, text=True,
                             timeout=30).stdout
        lines += [ln for ln in smi.splitlines() if "%" in ln]
    except Exception as e:  # diagnostics only
        lines.append(f"rocm-smi: {e!r}")
    return "\n".join(lines)


def _run_watched(cmd, tmp_path, limit=60, env=None):
    """Run the facade program; if it outlives `limit` s, report how far it got
    and what it is waiting in, then kill it."""
    import time
    log = tmp_path / "facade_stdout.txt"
    with open(log, "w") as f:
        p = subprocess.Popen(cmd, stdout=f, stderr=subprocess.STDOUT, env=env)
        t0 = time.time()
        while p.poll() is None and time.time() - t0 < limit:
            time.sleep(0.2)
        if p.poll() is None:
            d = _diag(p.pid)
            time.sleep(2)
            d2 = _diag(p.pid)
            p.kill()
            p.wait()
            raise AssertionError(f"facade_pcg stuck after {limit} s; output: {log.read_text()!r}\n{d}\n2 s later:\n{d2}")
    out = log.read_text()
    assert p.returncode == 0, out
    return out


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
    out = _run_watched([str(exe), str(tmp_path)], tmp_path)
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
