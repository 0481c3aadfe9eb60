"""Multi-process sharding protocol on CPU (gloo, world size 2 and 3).

Each rank plans its Morton range with the library's host-only planner
(mas_shard_plan), restricts its own level-1 segment, allgathers the padded
segments over gloo, builds the coarse residual hierarchy in the reference's
order (level 1 from the gathered segments, levels 2-3 as left folds of R1 over
the level-1 ids, fp32) -- bitwise the oracle's m_mappedR -- solves the coarse
levels and its own fine blocks, and writes z for its own vertices.  The local
arithmetic is a numpy restatement of the GPU kernels driven by the oracle's
maps and block inverses; the assembled z must equal the oracle's
single-process apply.  This covers the N > 1 host logic; the kernels themselves are covered
by tests/test_gpu_shard.py (virtual shards on one GPU).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import REPO, PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, L, out_dir):
    import sys
    for p in (os.path.join(PKG, "python"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import mas_amd
    from mas_amd import meshgen
    from oracle import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mesh = meshgen.cloth_grid(W)
    o = Oracle(mesh.nV, 0, 0, L, 1)
    o.allocate(mesh)
    o.prepare(mesh)
    m = o.maps()
    nV, Lv = mesh.nV, o.num_levels
    ls = m["level_size"]
    begin1 = int(ls[1][1])
    gn = m["going_next"]
    nb = (nV + 31) // 32
    if Lv > 1:
        l1_first = np.array([gn[32 * b:min(32 * b + 32, nV)].min() - begin1 for b in range(nb)] + [int(ls[1][0])],
                            dtype=np.int32)
    else:  # single level: no coarse segment (the library plans empty segments)
        l1_first = np.zeros(nb + 1, np.int32)
    plan = mas_amd.shard_plan(nV, l1_first, rank, world)
    r = meshgen.residual(nV, 5)
    rs = r[m["s2o"]].astype(np.float32)                       # Morton order
    # own level-1 segment: ordered sums of the members (k_restrict_seg)
    seg = np.zeros((plan["seg_max"], 4), np.float32)
    anc1 = gn[:nV] - begin1
    for i in range(plan["l1_end"] - plan["l1_begin"]):
        P = plan["l1_begin"] + i
        acc = np.zeros(3, np.float32)
        for v in np.nonzero(anc1 == P)[0]:                   # ascending vertex (= lane) order
            acc = (acc + rs[v, :3]).astype(np.float32)
        seg[i, :3] = acc
    gathered = [torch.zeros(plan["seg_max"], 4) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(seg))
    # unpack (the gathered segments through every rank's plan)
    R = np.zeros((o.total_clusters, 3), np.float32)
    for g in range(world):
        pg = mas_amd.shard_plan(nV, l1_first, g, world)
        cnt = pg["l1_end"] - pg["l1_begin"]
        R[begin1 + pg["l1_begin"]: begin1 + pg["l1_end"]] = gathered[g].numpy()[:cnt, :3]
    # levels 2 .. min(L-1, 3) in the reference's order (BuildResidualHierarchy,
    # .cpp:1577-1590): walking the level-1 ids in order, each R1 is added into
    # every ancestor, in fp32 -- the order the library's coarse kernels keep
    # (redundant on every rank); level 4 is never prolonged (B-6) and skipped
    if Lv > 2:
        n1 = int(ls[1][0])
        for c in range(begin1, begin1 + n1):
            a = c
            for _ in range(2, min(Lv, 4)):
                a = int(gn[a])
                R[a] = (R[a] + R[c]).astype(np.float32)
    # the residual hierarchy is bitwise the oracle's (m_mappedR)
    o.apply(r)
    Ro = o.mapped_r()
    for l in range(1, min(Lv, 4)):
        b, n = int(ls[l][1]), int(ls[l][0])
        assert np.array_equal(R[b:b + n].view(np.uint32), Ro[b:b + n, :3].astype(np.float32).view(np.uint32)), l
    R = R.astype(np.float64)
    Z = np.zeros_like(R)
    for blk in range(o.total_clusters // 32):
        if blk < nb and not (plan["fine_block_begin"] <= blk < plan["fine_block_end"]):
            continue
        x = R[32 * blk:32 * blk + 32] if blk >= nb else rs[32 * blk:32 * blk + 32, :3].astype(np.float64)
        if blk < nb and x.shape[0] < 32:
            x = np.vstack([x, np.zeros((32 - x.shape[0], 3))])
        Z[32 * blk:32 * blk + 32] = (o.block_inverse(blk).astype(np.float64) @ x.ravel()).reshape(32, 3)
    own = np.arange(plan["vert_begin"], plan["vert_end"])
    zown = Z[own].copy()
    for l in range(1, min(Lv, 4)):
        zown += Z[m["coarse_tables"][own, l - 1]]
    zfull = np.zeros((nV, 3))
    zfull[m["s2o"][own]] = zown
    zt = torch.from_numpy(zfull)
    dist.all_reduce(zt)                                        # owner-computes: disjoint supports
    if rank == 0:
        z_ref = o.apply(r)[:, :3]
        err = float(np.linalg.norm(zt.numpy() - z_ref) / np.linalg.norm(z_ref))
        np.save(os.path.join(out_dir, "err.npy"), np.array([err]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,L", [(2, 40, 3), (3, 64, 0), (2, 100, 1)])
def test_sharded_protocol_gloo(tmp_path, world, W, L):
    mp.spawn(_worker, args=(world, _free_port(), W, L, str(tmp_path)), nprocs=world, join=True)
    err = float(np.load(tmp_path / "err.npy")[0])
    assert err <= 1e-5, err
