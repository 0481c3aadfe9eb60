"""The C ABI's own collective hook from C++ (no Python in the loop): ranks as
threads on one GPU, each with its own handle, mas_shard_apply_device with a
host-staged allgather (tests/cpp/shard_threads.cpp); the union of the ranks'
z entries equals the unsharded apply bitwise."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, cloth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 3])
def test_cpp_threads_shard_apply(tmp_path, world):
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(200)
    r = meshgen.residual(mesh.nV, 0x5EED)
    for name, arr, dt in (("pos", mesh.pos, np.float32), ("starts", mesh.starts, np.int32),
                          ("idx", mesh.idx, np.int32), ("diag", mesh.diag, np.float32),
                          ("off", mesh.off, np.float32), ("r", r, np.float32)):
        np.ascontiguousarray(arr, dtype=dt).tofile(tmp_path / f"{name}.bin")
    exe = tmp_path / "shard_threads"
    lib = os.path.dirname(mas_amd.LIB_PATH)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-Wno-unused-value", "-Wno-unused-result", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "cpp", "shard_threads.cpp"), "-L", lib, "-lmas_amd",
                    f"-Wl,-rpath,{lib}", "-pthread", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), str(tmp_path), str(world)], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "BITWISE_EQUAL" in out.stdout and f"hook_calls 3" in out.stdout, out.stdout
