"""The committed golden blob (tests/golden/cloth12_L0.masblob, written on an
MI355X by scripts/make_golden_blob.py) read by a host-only Python parser of
the format in csrc/blob.hip, and checked against the CPU oracle: header,
FNV-1a checksum, section table, and the GPU's Morton codes, permutations,
level sizes and packed inverses (decoded through the layout of csrc/layout.h)
against the oracle's for the same mesh."""
import os
import struct

import numpy as np

from conftest import REPO, cloth

BLOB = os.path.join(REPO, "tests", "golden", "cloth12_L0.masblob")
HDR = struct.Struct("<8sII" + "i" * 10 + "i" * 18 + "ii" + "QQ")
SEC = struct.Struct("<IIQQ")
IDS = {1: "morton", 2: "s2o", 3: "o2s", 4: "cst", 5: "going_next", 6: "coarse_tables", 7: "fine_mask", 8: "vmap",
       9: "members", 10: "l1_first", 11: "inv"}


def fnv1a(b: bytes) -> int:
    h = 1469598103934665603
    for x in b:
        h ^= x
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def parse(raw: bytes):
    f = HDR.unpack_from(raw, 0)
    magic, version, hdr_bytes = f[0], f[1], f[2]
    nV, nE, nF, L, natL, tc, nBlk, nFine, maxNbr, nSt = f[3:13]
    level_size = np.array(f[13:31], np.int32).reshape(9, 2)
    nsec, payload, checksum = f[31], f[33], f[34]
    secs = {}
    for i in range(nsec):
        sid, _, nbytes, off = SEC.unpack_from(raw, hdr_bytes + i * SEC.size)
        secs[IDS[sid]] = raw[off:off + nbytes]
    return dict(magic=magic, version=version, hdr_bytes=hdr_bytes, nV=nV, L=L, tc=tc, nBlk=nBlk, nFine=nFine,
                level_size=level_size, payload=payload, checksum=checksum, secs=secs)


def slot_ij(o):
    """csrc/layout.h slot_ij, restated."""
    if o < 4608:
        F, comp = o >> 2, o & 3
        q, Ln = F >> 6, F & 63
        h, n = Ln >> 5, Ln & 31
        f = 4 * q + comp
        if h == 1 or f < 63:
            k, e = divmod(f, 9)
            s = 8 + k if h else 1 + k
            m = (n + s) & 31
            r, c = 3 * n + e // 3, 3 * m + e % 3
        elif f < 66:
            b = f - 63
            r, c = (3 * n, 3 * (n + 16) + b) if n < 16 else (3 * (n - 16) + 1, 3 * n + b)
        else:
            d = f - 66
            a = 0 if d < 3 else (1 if d < 5 else 2)
            b = d if d < 3 else (d - 2 if d < 5 else 2)
            r, c = 3 * n + a, 3 * n + b
    else:
        t = o - 4608
        p, b = divmod(t, 3)
        r, c = 3 * p + 2, 3 * (p + 16) + b
    return min(r, c), max(r, c)


def test_golden_blob_header_and_checksum():
    raw = open(BLOB, "rb").read()
    b = parse(raw)
    assert b["magic"] == b"MASBLOB\x00" and b["version"] == 1
    assert b["hdr_bytes"] + b["payload"] == len(raw)
    assert fnv1a(raw[b["hdr_bytes"]:]) == b["checksum"]
    assert b["nV"] == 144 and b["nFine"] == 5 and b["tc"] == 32 * b["nBlk"]
    assert len(b["secs"]["inv"]) == b["nBlk"] * 4656 * 4
    assert all(len(v) % 4 == 0 for v in b["secs"].values())


def test_golden_blob_matches_oracle():
    from oracle import Oracle
    b = parse(open(BLOB, "rb").read())
    mesh = cloth(12)
    o = Oracle(mesh.nV, 0, 0, 0, 1)
    o.allocate(mesh)
    o.prepare(mesh)
    m = o.maps()
    assert b["L"] == o.num_levels
    np.testing.assert_array_equal(np.frombuffer(b["secs"]["morton"], np.uint64), m["morton"])
    np.testing.assert_array_equal(np.frombuffer(b["secs"]["s2o"], np.int32), m["s2o"])
    np.testing.assert_array_equal(np.frombuffer(b["secs"]["o2s"], np.int32), m["o2s"])
    np.testing.assert_array_equal(b["level_size"][: o.num_levels + 1], m["level_size"])
    np.testing.assert_array_equal(np.frombuffer(b["secs"]["going_next"], np.int32)[: mesh.nV],
                                  m["going_next"][: mesh.nV])
    inv = np.frombuffer(b["secs"]["inv"], np.float32).reshape(b["nBlk"], 4656)
    ij = [slot_ij(s) for s in range(4656)]
    for blk in range(b["nBlk"]):
        ref = o.block_inverse(blk)
        got = np.zeros((96, 96), np.float32)
        for s, (i, j) in enumerate(ij):
            got[i, j] = got[j, i] = inv[blk, s]
        np.testing.assert_array_equal(got, ref)  # GPU inverses bit-exact with the oracle's


def _fnv1a(buf):
    h = 1469598103934665603
    for b in buf.tobytes():
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def test_blob_validate_without_device():
    """mas_blob_validate (no GPU): the golden blob passes; a blob whose
    checksum is valid but whose maps leave the level table is refused."""
    import mas_amd
    blob = np.fromfile(BLOB, dtype=np.uint8)
    assert mas_amd.blob_validate(blob) == 0
    hb = int(blob[12:16].view(np.uint32)[0])
    ns = int(blob[128:132].view(np.int32)[0])
    tab = blob[hb:hb + 24 * ns].reshape(ns, 24)
    sec = {int(t[:4].view(np.uint32)[0]): (int(t[8:16].view(np.uint64)[0]), int(t[16:24].view(np.uint64)[0]))
           for t in tab}
    for sid, word, val in ((8, 1, 1 << 28), (2, 5, -3), (5, 3, 1 << 20), (9, 0, 1 << 20), (10, 2, -1)):
        bad = blob.copy()
        off = sec[sid][1]
        bad[off + 4 * word: off + 4 * word + 4] = np.array([val], np.int32).view(np.uint8)
        bad[144:152] = np.array([_fnv1a(bad[hb:])], np.uint64).view(np.uint8)
        assert mas_amd.blob_validate(bad) == -1, sid
    bad = blob.copy()
    bad[-1] ^= 1
    assert mas_amd.blob_validate(bad) == -1  # checksum
