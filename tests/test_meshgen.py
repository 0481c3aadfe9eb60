"""Synthetic input generators (SURVEY §8 'Config sizes')."""
import numpy as np

from conftest import cloth, tet


def test_cloth_csr_counts_and_symmetry():
    m = cloth(100)
    assert m.nV == 10_000 and m.nnz == 78_804            # 10k config
    rows = np.repeat(np.arange(m.nV), np.diff(m.starts))
    a = set(zip(rows.tolist(), m.idx.tolist()))
    assert all((j, i) in a for (i, j) in a)
    assert not np.any(rows == m.idx)
    assert np.diff(m.starts).max() == 8


def test_tet_csr_counts():
    m = tet(8)
    rows = np.repeat(np.arange(m.nV), np.diff(m.starts))
    assert np.diff(m.starts).max() == 14
    # 7 directions, undirected count prod(W - d_k)
    W = 8
    und = 3 * (W - 1) * W * W + 3 * (W - 1) ** 2 * W + (W - 1) ** 3
    assert m.nnz == 2 * und
    assert not np.any(rows == m.idx)


def test_hessian_symmetric_and_spd():
    m = cloth(12)
    n = m.nV
    D = m.diag.reshape(n, 3, 3).transpose(0, 2, 1)
    O = m.off.reshape(-1, 3, 3).transpose(0, 2, 1)
    rows = np.repeat(np.arange(n), np.diff(m.starts))
    H = np.zeros((3 * n, 3 * n))
    for v in range(n):
        H[3 * v:3 * v + 3, 3 * v:3 * v + 3] = D[v]
    for e, (i, j) in enumerate(zip(rows, m.idx)):
        H[3 * i:3 * i + 3, 3 * j:3 * j + 3] = O[e]
    assert np.allclose(H, H.T, atol=1e-3)
    assert np.linalg.eigvalsh((H + H.T) / 2).min() > 0.5   # I + springs


def test_mt19937_matches_std():
    from mas_amd import meshgen
    # first outputs of std::mt19937(3), checked with g++ in this container
    assert meshgen._mt_raw(3, 3).tolist() == [2365658986, 303761048, 3041471737]


def test_vf_contact_records_layout():
    from mas_amd import meshgen
    m = cloth(20)
    vf, counts = meshgen.vf_contacts(m, 50, seed=3)
    assert vf.dtype.itemsize == 48 and counts[m.nV] == 50
    raw = vf.view(np.uint8).reshape(50, 48)
    assert np.all(raw[:, 24:32] == 0)                       # zeroed padding (B-2)
    assert np.all(vf["vId"] < m.nV) and np.all(vf["fId"] < m.faces.shape[0])
