"""Generate the reference-pinned fixtures (tests/golden/ref_headers.json,
tests/golden/ref_morton.npz) from the reference's OWN headers.

Runs in the build container only (needs /root/reference): it builds
oracle/_ref/libref_headers.so with oracle/build_ref.sh -- oracle/ref_headers.cpp
compiled against the unmodified SeMorton.h / SeMath.h / SeMatrix.h /
SeVector.h / SeCsr.h / SeAabb.h -- and records what that code computes:

* SeMorton64::Encode on edge inputs (NaN, +-inf, +-0, denormals, 1 +- ulp,
  out-of-range) and on random points (SeMorton.h:75-101);
* Math::Clamp / Min / Max on NaN and infinity operands (SeMath.h:100-103);
* ComputeAABB + FillSortingData Morton codes (SeSchwarzPreconditioner.cpp:
  201-235) for every BASELINE config mesh (10k / 256k / 1M cloth with the
  flat-axis NaN clamp, 160^3 tet lattice) and the small parity meshes, plus a
  jittered 3-D point cloud: SHA-256 of the code array, a strided sample, the
  AABB, the number of tied codes and -- when there are no ties, so every
  correct sort gives the same order -- SHA-256 of the sorted-to-original
  permutation (DoingSort, .cpp:238-243);
* sizeof / alignof / offsetof of SeMatrix3f, Int2/Int4, Float2/3/4,
  SeMorton64 and SeCsr<int>, SeMatrix3f's element order, and SeCsr::Size /
  IdxPtr on a sample CSR;
* (tests/golden/ref_contact.npz) the contact Hessian terms of
  PrepareCollisionHessian / AdditionalSchwarzHessian2 (.cpp:1190,1208-1223)
  evaluated with the reference's own Float3 / SeMatrix3f / OuterProduct /
  Math::Square for the BASELINE contact stencils (VF of configs[2], the EF
  and EE test records), random and edge directions, stiffnesses and weights.

The outputs are data only (inputs and the reference code's outputs).

Usage: python tests/golden/make_ref_fixtures.py [--contact-only]
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))

from mas_amd import meshgen  # noqa: E402

SAMPLE_STRIDE = 997
FULL_LIMIT = 20_000          # meshes up to this size keep their full code array in the npz

# name -> generator; the BASELINE config meshes and the parity tests' small meshes
MESHES = {
    "cloth-5": lambda: meshgen.cloth_grid(5).pos,
    "cloth-12": lambda: meshgen.cloth_grid(12).pos,
    "cloth-40": lambda: meshgen.cloth_grid(40).pos,
    "cloth-100": lambda: meshgen.cloth_grid(100).pos,      # 10k config
    "cloth-512": lambda: meshgen.cloth_grid(512).pos,      # 256k config
    "cloth-1024": lambda: meshgen.cloth_grid(1024).pos,    # 1M (+contacts) config
    "tet-16": lambda: meshgen.tet_lattice(16).pos,
    "tet-160": lambda: meshgen.tet_lattice(160).pos,       # 4M tet config
    "jitter-3d": lambda: jitter_cloud(16_384, seed=0x3D),
}


def jitter_cloud(n: int, seed: int) -> np.ndarray:
    """n points: a 3-D lattice with +-0.3-spacing jitter (every axis non-degenerate)."""
    rng = np.random.default_rng(seed)
    side = int(round(n ** (1 / 3))) + 1
    g = np.stack(np.meshgrid(*[np.arange(side)] * 3, indexing="ij"), -1).reshape(-1, 3)[:n]
    p = np.zeros((n, 4), np.float32)
    p[:, :3] = (0.01 * (g + rng.uniform(-0.3, 0.3, size=(n, 3)))).astype(np.float32)
    return p


def f32bits(x) -> str:
    return "0x%08x" % int(np.float32(x).view(np.uint32))


def edge_floats() -> np.ndarray:
    one = np.float32(1.0)
    vals = [0.0, -0.0, 1.0, 0.5, 0.25, 1.0 / 3.0, 2.0, -1.0, 1e-30, -1e-30, 1e30, -1e30,
            np.nextafter(one, np.float32(2)), np.nextafter(one, np.float32(0)),
            np.float32(2097151.0 / 2097152.0), np.float32(2097150.5 / 2097152.0),
            np.float32(1.4e-45), np.float32(-1.4e-45), np.float32(1.17549435e-38),
            float("nan"), float("inf"), float("-inf")]
    return np.array(vals, dtype=np.float32)


def lib():
    so = subprocess.run([os.path.join(REPO, "oracle", "build_ref.sh")], check=True, capture_output=True,
                        text=True).stdout.strip().splitlines()[-1]
    L = ctypes.CDLL(so)
    F = ctypes.c_float
    L.refh_morton_encode.argtypes = [F, F, F]
    L.refh_morton_encode.restype = ctypes.c_uint64
    for n in ("refh_clamp",):
        getattr(L, n).argtypes = [F, F, F]
        getattr(L, n).restype = F
    for n in ("refh_min", "refh_max"):
        getattr(L, n).argtypes = [F, F]
        getattr(L, n).restype = F
    L.refh_morton_points.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.refh_layout.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_longlong)]
    L.refh_csr_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p]
    L.refh_contact_terms.argtypes = [ctypes.c_void_p, F, ctypes.c_void_p, ctypes.c_void_p]
    return L, so


def P(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def mesh_codes(L, pos):
    n = pos.shape[0]
    codes = np.zeros(n, np.uint64)
    box = np.zeros(6, np.float32)
    L.refh_morton_points(P(np.ascontiguousarray(pos, np.float32)), n, P(codes), P(box))
    return codes, box


def contact_inputs():
    """(dir [N,3], stiff [N], w [N,5]) float32: the BASELINE stencils, random, edge."""
    f = np.float32
    one = f(1.0)
    dirs, stiffs, ws = [], [], []
    # configs[2] VF stencils (meshgen.vf_contacts: bary 0.25/0.25, normal z, stiff 100, zeroed
    # records): weights -b0, -b1, -(1 - pad) (B-2, pad = 0), 1; and the fix_vf_bary form
    for w2 in (-(one - f(0.0)), -(one - f(0.25) - f(0.25))):
        dirs.append([0, 0, 1]); stiffs.append(100.0); ws.append([-0.25, -0.25, w2, 1.0, 0.0])
    # meshgen.ef_contacts: bary (0.3, 0.2, 0.25), normal (0.6, 0, 0.8), stiff 50 (.cpp:326-354)
    b0, b1, b2 = f(0.3), f(0.2), f(0.25)
    dirs.append([0.6, 0.0, 0.8]); stiffs.append(50.0); ws.append([b0, one - b0, -b1, -b2, -((one - b1) - b2)])
    # meshgen.ee_contacts: bary (0.4, 0.7), normal (0, 0.6, 0.8), stiff 80 (.cpp:355-380)
    e0, e1 = f(0.4), f(0.7)
    dirs.append([0.0, 0.6, 0.8]); stiffs.append(80.0); ws.append([e0, one - e0, -e1, -(one - e1), 0.0])
    rng = np.random.default_rng(0xC0)
    for _ in range(256):
        d = rng.normal(size=3)
        dirs.append(d / np.linalg.norm(d))
        stiffs.append(10.0 ** rng.uniform(-2, 6))
        ws.append(rng.uniform(-1, 1, size=5))
    edge_w = [0.0, -0.0, 1.0, -1.0, 0.5, 1.0 / 3.0, 1e-20, -3e-39, 1e19, 2.0 ** -75, 7.0]
    edge_d = [[0, 0, 0], [1, 0, 0], [-0.0, 1, 0], [1e-20, 1e-25, 1], [1e15, -1e15, 3e-39], [0.6, -0.8, 0.0]]
    edge_s = [0.0, 1.0, 1e-30, 1e30, 3e-39, 100.0]
    for i, d in enumerate(edge_d):
        for j, st in enumerate(edge_s):
            k = 5 * (i * len(edge_s) + j)
            dirs.append(d); stiffs.append(st)
            ws.append([edge_w[(k + q) % len(edge_w)] for q in range(5)])
    return (np.asarray(dirs, f).reshape(-1, 3), np.asarray(stiffs, f), np.asarray(ws, f).reshape(-1, 5))


def contact_fixtures(L):
    dirs, stiffs, ws = contact_inputs()
    out = np.zeros((dirs.shape[0], 234), np.float32)
    for i in range(dirs.shape[0]):
        d = np.ascontiguousarray(dirs[i])
        w = np.ascontiguousarray(ws[i])
        o = np.zeros(234, np.float32)
        L.refh_contact_terms(P(d), float(stiffs[i]), P(w), P(o))
        out[i] = o
    np.savez_compressed(os.path.join(HERE, "ref_contact.npz"), dir=dirs, stiff=stiffs, w=ws, terms=out)
    print(f"wrote tests/golden/ref_contact.npz ({dirs.shape[0]} stencils)")


def main():
    L, so = lib()
    contact_fixtures(L)
    if "--contact-only" in sys.argv:
        return
    out = {
        "generator": "tests/golden/make_ref_fixtures.py",
        "built_from": ["SeMorton.h", "SeMath.h", "SeMatrix.h", "SeVector.h", "SeCsr.h", "SeAabb.h",
                       "SePreDefine.h"],
        "compile": "oracle/build_ref.sh (clang++ -std=c++17 -DWIN32 -fms-extensions -fdeclspec "
                   "-fdelayed-template-parsing -ffp-contract=off; only prelude <math.h>)",
        "note": "outputs of the reference's own header code; floats as IEEE-754 bit patterns",
    }
    arrays = {}

    # --- Encode on edge inputs and random points -------------------------------------------
    e = edge_floats()
    grid = np.array(np.meshgrid(e, e, e, indexing="ij")).reshape(3, -1).T.astype(np.float32)
    rng = np.random.default_rng(0x5E)
    rnd = rng.uniform(-0.1, 1.1, size=(8192, 3)).astype(np.float32)
    pts = np.concatenate([grid, rnd]).astype(np.float32)
    codes = np.array([L.refh_morton_encode(*map(float, p)) for p in pts], dtype=np.uint64)
    arrays["encode_in"] = pts
    arrays["encode_code"] = codes

    # --- Clamp / Min / Max ----------------------------------------------------------------------
    cl = []
    for a in e:
        for lo, hi in ((0.0, 2097151.0), (0.0, 1.0), (-1.0, 1.0)):
            r = L.refh_clamp(float(a), lo, hi)
            cl.append([f32bits(a), f32bits(lo), f32bits(hi), f32bits(r)])
    out["clamp"] = cl
    mm = []
    for a in e:
        for b in e:
            mm.append([f32bits(a), f32bits(b), f32bits(L.refh_min(float(a), float(b))),
                       f32bits(L.refh_max(float(a), float(b)))])
    out["minmax"] = mm

    # --- layouts --------------------------------------------------------------------------------
    lay = {}
    name, val = ctypes.c_char_p(), ctypes.c_longlong()
    i = 0
    while L.refh_layout(i, ctypes.byref(name), ctypes.byref(val)):
        lay[name.value.decode()] = int(val.value)
        i += 1
    out["layout"] = lay
    m = meshgen.cloth_grid(5)
    rows = m.nV
    sizes = np.zeros(rows, np.int32)
    offs = np.zeros(rows, np.int64)
    total = ctypes.c_int()
    nrows = L.refh_csr_probe(P(m.starts), rows, P(m.idx), P(sizes), P(offs), ctypes.byref(total))
    out["csr_probe"] = {"mesh": "cloth-5", "rows": int(nrows), "size": int(total.value),
                        "row_size": sizes.tolist(), "idxptr_offset": offs.tolist()}

    # --- meshes ---------------------------------------------------------------------------------
    meshes = {}
    for key, gen in MESHES.items():
        pos = gen()
        codes, box = mesh_codes(L, pos)
        order = np.argsort(codes, kind="stable").astype(np.int32)
        ties = int(np.count_nonzero(codes[order][1:] == codes[order][:-1]))
        rec = {"n": int(pos.shape[0]), "box": [f32bits(b) for b in box], "sha256": sha(codes.astype("<u8")),
               "ties": ties, "sample_stride": SAMPLE_STRIDE,
               "sample": ["0x%016x" % int(c) for c in codes[::SAMPLE_STRIDE]]}
        if ties == 0:
            rec["s2o_sha256"] = sha(order.astype("<i4"))
        if pos.shape[0] <= FULL_LIMIT:
            arrays[f"codes_{key}"] = codes
            if key == "jitter-3d":
                arrays["pos_jitter-3d"] = pos
        meshes[key] = rec
        print(f"{key}: n={pos.shape[0]} ties={ties} sha={rec['sha256'][:16]}", flush=True)
    out["meshes"] = meshes

    with open(os.path.join(HERE, "ref_headers.json"), "w") as f:
        json.dump(out, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "ref_morton.npz"), **arrays)
    print("wrote tests/golden/ref_headers.json, tests/golden/ref_morton.npz")


if __name__ == "__main__":
    main()
