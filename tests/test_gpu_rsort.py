"""Prepare's look-back-free radix sort and scan (csrc/rsort.hip).

Every key/value sort and int exclusive scan of Prepare runs through these
kernels (radix.h, k_assemble.hip, k_levels.hip, k_coarse.hip), so their output
decides the summation orders the bitwise parity tests pin.  Here they are
checked directly, through the diagnostic entry points mas_dev_sort_pairs /
mas_dev_exclusive_scan, against
  * numpy's stable argsort / cumsum (the definition), bit-exact, and
  * the rocprim / hipcub kernels they replaced (impl 0), bit-exact,
over tile-boundary sizes (a tile is 4096 keys), key widths 1..32 with junk
above the sorted bits (only the low `bits` count, as in rocprim), heavy
duplicates (stability), and unaligned / in-place scans.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def handle():
    from mas_amd import SeSchwarzPreconditioner
    return SeSchwarzPreconditioner()


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()


def _sort(P, keys, vals, bits, impl):
    n = keys.size
    kin, vin = _dev(keys), _dev(vals)
    kout = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    vout = torch.empty_like(kout)
    torch.cuda.synchronize()  # the library runs on its own stream
    rc = P._L.mas_dev_sort_pairs(P.h, kin.data_ptr(), kout.data_ptr(), vin.data_ptr(), vout.data_ptr(), n, bits,
                                 impl)
    P._check(rc, "dev_sort_pairs")
    # the inputs stay untouched (callers sort from read-only arrays such as iota)
    assert np.array_equal(kin.cpu().numpy().view(np.uint32), keys)
    return kout[:n].cpu().numpy().view(np.uint32), vout[:n].cpu().numpy()


def _keys(rng, n, bits, dup):
    span = 1 << bits
    if dup:
        span = min(span, max(1, n // 50))  # ~50 copies per key: stability matters
    low = rng.integers(0, span, n, dtype=np.uint64).astype(np.uint32)
    if bits < 32:  # junk above the sorted bits must not count
        low |= (rng.integers(0, 1 << (32 - bits), n, dtype=np.uint64).astype(np.uint32) << np.uint32(bits))
    return low


SIZES = [1, 63, 4095, 4096, 4097, 100_003, (1 << 20) + 17]
BITS = [1, 5, 8, 9, 16, 20, 27, 32]


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("bits", BITS)
def test_sort_pairs_matches_stable_argsort_and_rocprim(handle, n, bits):
    rng = np.random.default_rng(n * 131 + bits)
    keys = _keys(rng, n, bits, dup=(n + bits) % 2 == 0)
    vals = rng.permutation(n).astype(np.int32)
    mask = np.uint32(0xFFFFFFFF if bits == 32 else (1 << bits) - 1)
    perm = np.argsort(keys & mask, kind="stable")
    k1, v1 = _sort(handle, keys, vals, bits, 1)
    assert np.array_equal(k1, keys[perm])
    assert np.array_equal(v1, vals[perm])
    k0, v0 = _sort(handle, keys, vals, bits, 0)
    assert np.array_equal(k0, k1) and np.array_equal(v0, v1)


def test_sort_pairs_presorted_and_constant(handle):
    """One digit everywhere: every lane of a wave in one peer group."""
    n = 300_000
    for keys in (np.full(n, 7, np.uint32), np.arange(n, dtype=np.uint32)):
        vals = np.arange(n, dtype=np.int32)[::-1].copy()
        k1, v1 = _sort(handle, keys, vals, 19, 1)
        perm = np.argsort(keys & np.uint32((1 << 19) - 1), kind="stable")
        assert np.array_equal(k1, keys[perm]) and np.array_equal(v1, vals[perm])


def test_sort_pairs_empty(handle):
    P = handle
    assert P._L.mas_dev_sort_pairs(P.h, None, None, None, None, 0, 8, 1) == 0


def _scan(P, x, impl, offset=0, inplace=False):
    n = x.size
    buf = torch.zeros(n + offset + 4, dtype=torch.int32, device="cuda")
    buf[offset:offset + n] = torch.from_numpy(x).cuda()
    if inplace:
        out = buf
    else:
        out = torch.zeros_like(buf)
    torch.cuda.synchronize()  # the library runs on its own stream
    rc = P._L.mas_dev_exclusive_scan(P.h, buf.data_ptr() + 4 * offset, out.data_ptr() + 4 * offset, n, impl)
    P._check(rc, "dev_exclusive_scan")
    return out[offset:offset + n].cpu().numpy()


@pytest.mark.parametrize("n", [1, 15, 4095, 4096, 4097, 65_537, (1 << 20) + 3, 5_000_011])
def test_exclusive_scan(handle, n):
    rng = np.random.default_rng(n)
    x = rng.integers(0, 100, n).astype(np.int32)
    want = np.concatenate([[0], np.cumsum(x, dtype=np.int64)[:-1]]).astype(np.int32)
    got = _scan(handle, x, 1)
    assert np.array_equal(got, want)
    assert np.array_equal(_scan(handle, x, 0), want)
    assert np.array_equal(_scan(handle, x, 1, offset=1), want)       # unaligned: scalar path
    assert np.array_equal(_scan(handle, x, 1, inplace=True), want)   # in == out
