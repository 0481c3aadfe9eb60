"""Loaders for the reference-pinned fixtures (tests/golden/ref_headers.json,
tests/golden/ref_morton.npz; made by tests/golden/make_ref_fixtures.py from the
reference's own headers).  Data only -- no reference code travels."""
from __future__ import annotations

import functools
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@functools.lru_cache(maxsize=None)
def ref_json() -> dict:
    with open(os.path.join(GOLDEN, "ref_headers.json")) as f:
        return json.load(f)


@functools.lru_cache(maxsize=None)
def ref_arrays() -> dict:
    with np.load(os.path.join(GOLDEN, "ref_morton.npz")) as z:   # allow_pickle=False (default)
        return {k: z[k] for k in z.files}


@functools.lru_cache(maxsize=None)
def ref_contact() -> dict:
    """tests/golden/ref_contact.npz: dir [N,3], stiff [N], w [N,5] and the
    reference headers' contact terms [N,234] (orc_contact_terms layout)."""
    with np.load(os.path.join(GOLDEN, "ref_contact.npz")) as z:   # allow_pickle=False (default)
        return {k: z[k] for k in z.files}


def bits_to_f32(h: str) -> np.float32:
    return np.array([int(h, 16)], np.uint32).view(np.float32)[0]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def mesh_positions(key: str) -> np.ndarray:
    """Positions of fixture mesh `key` (regenerated deterministically)."""
    from mas_amd import meshgen
    kind, _, size = key.partition("-")
    if kind == "cloth":
        return meshgen.cloth_grid(int(size)).pos
    if kind == "tet":
        return meshgen.tet_lattice(int(size)).pos
    if key == "jitter-3d":
        return ref_arrays()["pos_jitter-3d"]
    raise KeyError(key)


def check_codes(key: str, codes: np.ndarray, s2o: np.ndarray | None = None) -> None:
    """Assert Morton codes (and, when the reference's codes have no ties, the
    sorted-to-original permutation) equal the reference's, bit for bit."""
    rec = ref_json()["meshes"][key]
    codes = np.asarray(codes, np.uint64)
    assert codes.shape == (rec["n"],), (key, codes.shape)
    sample = np.array([int(h, 16) for h in rec["sample"]], np.uint64)
    bad = np.nonzero(codes[:: rec["sample_stride"]] != sample)[0]
    assert bad.size == 0, f"{key}: Morton code differs from the reference at vertex {bad[0] * rec['sample_stride']}"
    full = ref_arrays().get(f"codes_{key}")
    if full is not None:
        np.testing.assert_array_equal(codes, full)
    assert sha(codes.astype("<u8")) == rec["sha256"], f"{key}: Morton code array hash differs from the reference"
    if s2o is not None and "s2o_sha256" in rec:
        assert sha(np.asarray(s2o).astype("<i4")) == rec["s2o_sha256"], f"{key}: sort order differs"
