"""GPU Allocate pinned against the reference's OWN code.

The Morton codes (k_allocate.hip: AABB, SeMorton64::Encode with the ternary
NaN clamp) and the sort order that mas_allocate produces, read back through
mas_get_maps, against tests/golden/ref_headers.json / ref_morton.npz -- the
codes the reference's unmodified SeMorton.h / SeMath.h / SeAabb.h compute for
every BASELINE config mesh (10k / 256k / 1M cloth, 160^3 tet lattice), the
small parity meshes and a jittered 3-D cloud (tests/golden/make_ref_fixtures.py).
Bar: bit-exact (hash of the whole array, a strided sample, full arrays for the
small meshes); the reference's codes have no ties there, so the stable sort's
permutation is the only valid one and is checked by hash too.

The contact Hessian terms of the assembly kernels (k_assemble.hip
contact_outer / contact_self / contact_pair / contact_double, through
mas_dev_contact_terms) against tests/golden/ref_contact.npz -- what the
reference's own Float3 / SeMatrix3f / OuterProduct / Math::Square compute for
.cpp:1190,1208-1223.  Bar: bit-exact.
"""
import ctypes

import numpy as np
import pytest

from ref_fixtures import check_codes, mesh_positions, ref_contact, ref_json

pytestmark = pytest.mark.gpu


def _chain_csr(n):
    """v <-> v+1: Allocate needs a neighbour table; the codes do not depend on it."""
    a = np.arange(n - 1)
    starts = np.zeros(n + 1, np.int64)
    deg = np.zeros(n, np.int64)
    deg[:-1] += 1
    deg[1:] += 1
    np.cumsum(deg, out=starts[1:])
    idx = np.zeros(starts[-1], np.int32)
    fill = starts[:-1].copy()
    idx[fill[1:]] = a            # neighbour v-1 first (ascending)
    fill[1:] += 1
    idx[fill[:-1]] = a + 1
    return starts.astype(np.int32), idx


@pytest.mark.parametrize("key", list(ref_json()["meshes"]))
def test_gpu_morton_and_sort_match_reference(key):
    import mas_amd
    from mas_amd import _ptr
    pos = np.ascontiguousarray(mesh_positions(key), np.float32)
    n = pos.shape[0]
    starts, idx = _chain_csr(n)
    P = mas_amd.SeSchwarzPreconditioner(max_levels=1)
    P.m_positions = pos
    P.m_neighbours = (starts, idx)
    P.AllocatePrecoditioner(n, 0, 0)
    morton = np.zeros(n, np.uint64)
    s2o = np.zeros(n, np.int32)
    rc = P._L.mas_get_maps(P.h, _ptr(morton), _ptr(s2o), None, None, None, None, None)
    assert rc == 0, mas_amd.STATUS.get(rc, rc)
    check_codes(key, morton, s2o)


def test_gpu_contact_terms_match_reference():
    import mas_amd
    from mas_amd import _ptr
    c = ref_contact()
    n = c["dir"].shape[0]
    P = mas_amd.SeSchwarzPreconditioner()
    out = np.zeros((n, 234), np.float32)
    args = [np.ascontiguousarray(c[k], np.float32) for k in ("dir", "stiff", "w")]
    rc = P._L.mas_dev_contact_terms(P.h, *[_ptr(a) for a in args], _ptr(out), n)
    assert rc == 0, mas_amd.STATUS.get(rc, rc)
    bad = np.argwhere(out.view(np.uint32) != c["terms"].view(np.uint32))
    assert bad.size == 0, f"{len(bad)} terms differ, first stencil {bad[0][0]} entry {bad[0][1]}"
