"""The CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer
(sanitizer builds of the CPU path).

oracle/sanitize_main.c drives Allocate -> Prepare -> Preconditioning of the
restatement built with -fsanitize=address,undefined -fno-sanitize-recover
(make -C oracle sanitize) on cases written here: cloth with each contact type
(EF, EE, VF, all three at once -- the B-3 set offsets), a tet lattice and a
non-power-of-two cloth whose banks hold several components (B-4's poorly
clustered levels), at several level counts.  Any report makes the run fail;
z must equal the regular (-O3, OpenMP) build's bit for bit.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, cloth, tet

ORACLE = os.path.join(REPO, "oracle")
EXE = os.path.join(ORACLE, "_build", "oracle_sanitize")


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], check=True)
    return EXE


def _write_case(path, mesh, L, ef=None, ee=None, vf=None, threads=2, seed=1):
    from mas_amd import meshgen
    r = meshgen.residual(mesh.nV, seed)
    hd = np.array([mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0], mesh.nnz, L,
                   0 if ef is None else ef.shape[0], 0 if ee is None else ee.shape[0],
                   0 if vf is None else vf.shape[0], threads], np.int32)
    with open(path, "wb") as f:
        for a in (hd, np.ascontiguousarray(mesh.pos, np.float32), np.ascontiguousarray(mesh.starts, np.int32),
                  np.ascontiguousarray(mesh.idx, np.int32), np.ascontiguousarray(mesh.edges, np.int32),
                  np.ascontiguousarray(mesh.faces, np.int32), np.ascontiguousarray(mesh.diag, np.float32),
                  np.ascontiguousarray(mesh.off, np.float32)):
            f.write(a.tobytes())
        for recs in (ef, ee, vf):
            if recs is not None:
                f.write(recs.tobytes())
        f.write(r.tobytes())
    return r


def _regular(mesh, L, r, ef=None, ee=None, vf=None):
    from oracle import Oracle
    o = Oracle(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0], L, 2)
    o.allocate(mesh)
    cnt = lambda n, m: None if m is None else np.append(np.zeros(n, np.uint32), np.uint32(m.shape[0]))  # noqa: E731
    nE = mesh.edges.shape[0]
    o.prepare(mesh, ef=ef, ee=ee, vf=vf, efC=cnt(nE, ef), eeC=cnt(nE, ee), vfC=cnt(mesh.nV, vf))
    return o.apply(r)


def _cases():
    from mas_amd import meshgen
    c24, c33 = cloth(24), cloth(33)
    return [
        ("cloth24-vf", c24, 0, dict(vf=meshgen.vf_contacts(c24, 60)[0])),
        ("cloth24-ef", c24, 3, dict(ef=meshgen.ef_contacts(c24, 40)[0])),
        ("cloth24-ee", c24, 2, dict(ee=meshgen.ee_contacts(c24, 40)[0])),
        ("cloth24-all", c24, 0, dict(ef=meshgen.ef_contacts(c24, 20)[0], ee=meshgen.ee_contacts(c24, 20)[0],
                                     vf=meshgen.vf_contacts(c24, 20)[0])),
        ("cloth33-vf", c33, 0, dict(vf=meshgen.vf_contacts(c33, 80, seed=9)[0])),
        ("tet8", tet(8), 0, {}),
        ("cloth5", cloth(5), 1, {}),
    ]


@pytest.mark.parametrize("idx", range(7))
def test_oracle_clean_under_asan_ubsan(exe, tmp_path, idx):
    name, mesh, L, contacts = _cases()[idx]
    case, zf = tmp_path / "case.bin", tmp_path / "z.bin"
    r = _write_case(case, mesh, L, **contacts)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="2")
    p = subprocess.run([exe, str(case), str(zf)], capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, f"{name}: rc {p.returncode}\n{p.stderr[-4000:]}"
    assert "runtime error" not in p.stderr and "Sanitizer" not in p.stderr, p.stderr[-4000:]
    z = np.fromfile(zf, np.float32).reshape(-1, 4)
    np.testing.assert_array_equal(z, _regular(mesh, L, r, **contacts))
