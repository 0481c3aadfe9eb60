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
    out = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=300, check=True).stdout
    z = np.fromfile(tmp_path / "z.bin", dtype=np.float32).reshape(-1, 4)
    o = Oracle(mesh.nV, 0, 0, 0, 1)
    o.allocate(mesh)
    o.prepare(mesh)
    z_ref = o.apply(r)
    err = np.linalg.norm(z[:, :3] - z_ref[:, :3]) / np.linalg.norm(z_ref[:, :3])
    assert err <= 1e-5, err
    # Preconditioning / PreparePreconditioner repeated through the same host
    # arrays (page-locked and cached by the library): bitwise the first z
    assert "host_repeat_bitwise 1" in out, out
    iters = int(out.split("pcg_iterations")[1])
    assert 20 < iters < 200, out
