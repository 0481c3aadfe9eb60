"""Synthetic inputs for the MAS preconditioner (SURVEY.md §8 "Config sizes").

Deterministic generators for the benchmark and parity configurations:

* ``cloth_grid(W)``  -- W x W flat cloth, positions (0.01 i, 0.01 j, 0),
  8-neighbour symmetric CSR (structural + shear), spring Hessian.
* ``tet_lattice(W)`` -- W^3 lattice, spacing 0.01, Freudenthal 6-tet split
  (neighbours +-(1,0,0) ... +-(1,1,1), valence <= 14), same spring Hessian.
* ``vf_contacts(...)`` -- VF contact records (48-byte ``VfSet``,
  SeCollisionElements.h:42-49) drawn with std::mt19937 semantics.

Hessian: ``K = 1000 d d^T`` with
``d = normalize(p_min - p_max + (0, 0, 0.003))`` where min/max are taken over
the vertex *index* of the pair, ``diag(v) = I + sum K``, ``off(v,u) = -K``.
3x3 blocks are returned as 9 floats in column-major order (``SeMatrix3f``,
SeMatrix.h:650-682); K is symmetric so the order only matters as a layout.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

STIFF = 1000.0
DZ = 0.003


@dataclass
class Mesh:
    pos: np.ndarray          # [nV, 4] float32 (SeVec3fSimd, w = 0)
    starts: np.ndarray       # [nV + 1] int32 CSR row starts (SeCsr::m_starts)
    idx: np.ndarray          # [nnz] int32 neighbour ids, ascending per row, no self
    diag: np.ndarray         # [nV, 9] float32 column-major 3x3
    off: np.ndarray          # [nnz, 9] float32 column-major 3x3, off[starts[v]+k] pairs with idx[starts[v]+k]
    faces: np.ndarray        # [nF, 4] int32 (Int4, 4th unused)
    edges: np.ndarray        # [nE, 4] int32 (Int4: two vertices, two opposite (unused -> -1))

    @property
    def nV(self) -> int:
        return int(self.pos.shape[0])

    @property
    def nnz(self) -> int:
        return int(self.idx.shape[0])


def _csr_from_pairs(n: int, a: np.ndarray, b: np.ndarray):
    """Symmetric CSR from undirected pairs (a, b); rows sorted ascending."""
    src = np.concatenate([a, b])
    dst = np.concatenate([b, a])
    order = np.lexsort((dst, src))
    src = src[order]
    dst = dst[order]
    counts = np.bincount(src, minlength=n)
    starts = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=starts[1:])
    return starts.astype(np.int32), dst.astype(np.int32), src


def _spring_hessian(pos64: np.ndarray, starts: np.ndarray, idx: np.ndarray, rows: np.ndarray):
    n = pos64.shape[0]
    lo = np.minimum(rows, idx)
    hi = np.maximum(rows, idx)
    d = pos64[lo] - pos64[hi]
    d[:, 2] += DZ
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    K = STIFF * d[:, :, None] * d[:, None, :]             # [nnz, 3, 3] symmetric
    diag = np.zeros((n, 3, 3), dtype=np.float64)
    diag[:, 0, 0] = diag[:, 1, 1] = diag[:, 2, 2] = 1.0
    np.add.at(diag, rows, K)
    off = -K
    # column-major: element (i, j) at j*3 + i  ->  transpose then flatten row-major
    diag9 = np.ascontiguousarray(diag.transpose(0, 2, 1).reshape(n, 9), dtype=np.float32)
    off9 = np.ascontiguousarray(off.transpose(0, 2, 1).reshape(-1, 9), dtype=np.float32)
    return diag9, off9


def cloth_grid(W: int) -> Mesh:
    ii, jj = np.meshgrid(np.arange(W), np.arange(W), indexing="ij")
    vid = (ii * W + jj).astype(np.int64)
    pos64 = np.zeros((W * W, 3), dtype=np.float64)
    pos64[vid.ravel(), 0] = 0.01 * ii.ravel()
    pos64[vid.ravel(), 1] = 0.01 * jj.ravel()
    pairs = []
    for di, dj in ((1, 0), (0, 1), (1, 1), (1, -1)):
        i0 = np.arange(max(0, -di), W - max(0, di))
        j0 = np.arange(max(0, -dj), W - max(0, dj))
        a_i, a_j = np.meshgrid(i0, j0, indexing="ij")
        a = (a_i * W + a_j).ravel()
        b = ((a_i + di) * W + (a_j + dj)).ravel()
        pairs.append((a, b))
    a = np.concatenate([p[0] for p in pairs])
    b = np.concatenate([p[1] for p in pairs])
    starts, idx, rows = _csr_from_pairs(W * W, a, b)
    pos32 = pos64.astype(np.float32)
    diag9, off9 = _spring_hessian(pos32.astype(np.float64), starts, idx, rows)
    pos4 = np.zeros((W * W, 4), dtype=np.float32)
    pos4[:, :3] = pos32
    # triangles: cell (i, j) -> (a, b, c), (a, c, d) with a=(i,j) b=(i+1,j) c=(i+1,j+1) d=(i,j+1)
    ci, cj = np.meshgrid(np.arange(W - 1), np.arange(W - 1), indexing="ij")
    va = (ci * W + cj).ravel()
    vb = ((ci + 1) * W + cj).ravel()
    vc = ((ci + 1) * W + cj + 1).ravel()
    vd = (ci * W + cj + 1).ravel()
    faces = np.zeros((2 * va.size, 4), dtype=np.int32)
    faces[0::2, 0], faces[0::2, 1], faces[0::2, 2] = va, vb, vc
    faces[1::2, 0], faces[1::2, 1], faces[1::2, 2] = va, vc, vd
    faces[:, 3] = -1
    edges = np.full((a.size, 4), -1, dtype=np.int32)
    edges[:, 0] = a
    edges[:, 1] = b
    return Mesh(pos4, starts, idx, diag9, off9, faces, edges)


def tet_lattice(W: int) -> Mesh:
    n = W ** 3
    g = np.arange(W)
    xi, yi, zi = np.meshgrid(g, g, g, indexing="ij")
    vid = (xi * W * W + yi * W + zi).ravel()
    pos64 = np.zeros((n, 3), dtype=np.float64)
    pos64[vid, 0] = 0.01 * xi.ravel()
    pos64[vid, 1] = 0.01 * yi.ravel()
    pos64[vid, 2] = 0.01 * zi.ravel()
    dirs = [(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (1, 0, 1), (0, 1, 1), (1, 1, 1)]
    A, B = [], []
    for dx, dy, dz in dirs:
        ax, ay, az = np.meshgrid(np.arange(W - dx), np.arange(W - dy), np.arange(W - dz), indexing="ij")
        a = (ax * W * W + ay * W + az).ravel()
        b = ((ax + dx) * W * W + (ay + dy) * W + (az + dz)).ravel()
        A.append(a)
        B.append(b)
    a = np.concatenate(A)
    b = np.concatenate(B)
    starts, idx, rows = _csr_from_pairs(n, a, b)
    pos32 = pos64.astype(np.float32)
    diag9, off9 = _spring_hessian(pos32.astype(np.float64), starts, idx, rows)
    pos4 = np.zeros((n, 4), dtype=np.float32)
    pos4[:, :3] = pos32
    faces = np.zeros((0, 4), dtype=np.int32)
    edges = np.full((a.size, 4), -1, dtype=np.int32)
    edges[:, 0] = a
    edges[:, 1] = b
    return Mesh(pos4, starts, idx, diag9, off9, faces, edges)


# ---------------------------------------------------------------------------
# contacts
# ---------------------------------------------------------------------------

def _mt_raw(seed: int, count: int) -> np.ndarray:
    """First ``count`` outputs of std::mt19937(seed).  numpy's legacy seeding is
    init_genrand(seed); checked against std::mt19937(3) in tests."""
    bg = np.random.MT19937(0)
    bg._legacy_seeding(seed)
    return bg.random_raw(count).astype(np.uint32)


VF_DTYPE = np.dtype({
    "names": ["vId", "fId", "stiff", "bary", "pad24", "normal"],
    "formats": ["<i4", "<i4", "<f4", ("<f4", 2), "<f4", ("<f4", 4)],
    "offsets": [0, 4, 8, 16, 24, 32],
    "itemsize": 48,
})
EF_DTYPE = np.dtype({
    "names": ["eId", "fId", "stiff", "bary", "normal"],
    "formats": ["<i4", "<i4", "<f4", ("<f4", 3), ("<f4", 4)],
    "offsets": [0, 4, 8, 12, 32],
    "itemsize": 48,
})
EE_DTYPE = np.dtype({
    "names": ["eId0", "eId1", "stiff", "bary", "pad24", "normal"],
    "formats": ["<i4", "<i4", "<f4", ("<f4", 2), "<f4", ("<f4", 4)],
    "offsets": [0, 4, 8, 16, 24, 32],
    "itemsize": 48,
})


def vf_contacts(mesh: Mesh, count: int, seed: int = 3, bary=(0.25, 0.25), stiff: float = 100.0):
    """v = rng() % N, f = rng() % nF, bary (0.25, 0.25),
    normal (0, 0, 1), stiff 100, zero-initialised records (B-2)."""
    raw = _mt_raw(seed, 2 * count).astype(np.uint64)
    vf = np.zeros(count, dtype=VF_DTYPE)
    vf["vId"] = (raw[0::2] % np.uint64(mesh.nV)).astype(np.int32)
    vf["fId"] = (raw[1::2] % np.uint64(mesh.faces.shape[0])).astype(np.int32)
    vf["stiff"] = stiff
    vf["bary"][:, 0] = bary[0]
    vf["bary"][:, 1] = bary[1]
    vf["normal"][:, 2] = 1.0
    counts = np.zeros(mesh.nV + 1, dtype=np.uint32)
    counts[mesh.nV] = count          # only the total at [nV] is read (.cpp:308)
    return vf, counts


def ef_contacts(mesh: Mesh, count: int, seed: int = 5, bary=(0.3, 0.2, 0.25), stiff: float = 50.0):
    """Edge-face contact records (EfSet, SeCollisionElements.h:33-41): e = rng() % nE,
    f = rng() % nF, fixed barycentrics, unit normal (0.6, 0, 0.8).  Counts [nE+1],
    total at [nE] (.cpp:306)."""
    raw = _mt_raw(seed, 2 * count).astype(np.uint64)
    ef = np.zeros(count, dtype=EF_DTYPE)
    ef["eId"] = (raw[0::2] % np.uint64(mesh.edges.shape[0])).astype(np.int32)
    ef["fId"] = (raw[1::2] % np.uint64(mesh.faces.shape[0])).astype(np.int32)
    ef["stiff"] = stiff
    for k in range(3):
        ef["bary"][:, k] = bary[k]
    ef["normal"][:, 0] = 0.6
    ef["normal"][:, 2] = 0.8
    counts = np.zeros(mesh.edges.shape[0] + 1, dtype=np.uint32)
    counts[-1] = count
    return ef, counts


def ee_contacts(mesh: Mesh, count: int, seed: int = 7, bary=(0.4, 0.7), stiff: float = 80.0):
    """Edge-edge contact records (EeSet, SeCollisionElements.h:43-50): two edges
    rng() % nE, fixed barycentrics, unit normal (0, 0.6, 0.8).  Counts [nE+1]."""
    raw = _mt_raw(seed, 2 * count).astype(np.uint64)
    ee = np.zeros(count, dtype=EE_DTYPE)
    ee["eId0"] = (raw[0::2] % np.uint64(mesh.edges.shape[0])).astype(np.int32)
    ee["eId1"] = (raw[1::2] % np.uint64(mesh.edges.shape[0])).astype(np.int32)
    ee["stiff"] = stiff
    ee["bary"][:, 0] = bary[0]
    ee["bary"][:, 1] = bary[1]
    ee["normal"][:, 1] = 0.6
    ee["normal"][:, 2] = 0.8
    counts = np.zeros(mesh.edges.shape[0] + 1, dtype=np.uint32)
    counts[-1] = count
    return ee, counts


def residual(nV: int, seed: int) -> np.ndarray:
    """r ~ U(-1, 1)^3, w = 0 (float32)."""
    rng = np.random.default_rng(seed)
    r = np.zeros((nV, 4), dtype=np.float32)
    r[:, :3] = rng.uniform(-1.0, 1.0, size=(nV, 3)).astype(np.float32)
    return r


# ---------------------------------------------------------------------------
# named configurations (BASELINE.json "configs")
# ---------------------------------------------------------------------------

CONFIGS = {
    "10k": dict(kind="cloth", W=100, levels=1, contacts=0),
    "256k": dict(kind="cloth", W=512, levels=3, contacts=0),
    "1M+contacts": dict(kind="cloth", W=1024, levels=4, contacts=100_000),
    "1M": dict(kind="cloth", W=1024, levels=4, contacts=0),
    "4M-tet": dict(kind="tet", W=160, levels=4, contacts=0),
}


def build_config(name: str) -> tuple[Mesh, dict]:
    cfg = CONFIGS[name]
    mesh = cloth_grid(cfg["W"]) if cfg["kind"] == "cloth" else tet_lattice(cfg["W"])
    return mesh, cfg
