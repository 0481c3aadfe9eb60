"""Multi-process sharding protocol on CPU (gloo, world size 2 and 3).

What runs here is the host side of the sharded apply (include/mas_capi.h
mas_shard_*, python/mas_amd/distributed.py) over a real multi-process group:

  * every rank plans with the library's host-only planner (mas_shard_plan);
  * the plans partition the level-0 blocks, the Morton-sorted vertices and the
    level-1 nodes exactly once, in rank order, with every rank's level-1
    segment inside the padded seg_max the exchange sends;
  * each rank fills its padded segment with its own level-1 residuals, the
    segments are allgathered over gloo with the collective ShardedApply issues
    (all_gather_into_tensor of world * seg_max float4) and every rank unpacks
    the gathered buffer through every rank's plan: the result must be the
    whole level-1 residual, bitwise;
  * owner-computes z: the ranks' vertex ranges cover every vertex once.

The per-rank values (level-1 residuals, z) are the oracle's single-process
ones, read from the oracle (tests/ only): no kernel arithmetic is restated
here.  That the library's own restriction, unpack and finish kernels produce
exactly those values per rank is tested on the GPU: virtual shards bitwise
against the unsharded apply (tests/test_gpu_shard.py), the 2-process gloo
ShardedApply through the library (tests/test_gpu_shard.py, tests/shard_worker.py)
and the C++ two-thread hook test (tests/test_gpu_shard_cpp.py).
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


def _l1_first(m, nV, L):
    """l1_first for mas_shard_plan from the level maps (the same table the
    library derives on the device in mas_shard_setup)."""
    ls, gn = m["level_size"], m["going_next"]
    nb = (nV + 31) // 32
    if L <= 1:
        return np.zeros(nb + 1, np.int32)
    begin1 = int(ls[1][1])
    return np.array([gn[32 * b:min(32 * b + 32, nV)].min() - begin1 for b in range(nb)] + [int(ls[1][0])],
                    dtype=np.int32)


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
    nb = (nV + 31) // 32
    l1_first = _l1_first(m, nV, Lv)
    n1 = int(l1_first[-1])
    plans = [mas_amd.shard_plan(nV, l1_first, g, world) for g in range(world)]
    plan = plans[rank]

    # the plans partition blocks, vertices and level-1 nodes in rank order
    assert plans[0]["fine_block_begin"] == 0 and plans[-1]["fine_block_end"] == nb
    assert plans[0]["vert_begin"] == 0 and plans[-1]["vert_end"] == nV
    assert plans[0]["l1_begin"] == 0 and plans[-1]["l1_end"] == n1
    for a, b in zip(plans, plans[1:]):
        assert a["fine_block_end"] == b["fine_block_begin"]
        assert a["vert_end"] == b["vert_begin"] and a["l1_end"] == b["l1_begin"]
    for p in plans:
        assert p["vert_begin"] == 32 * p["fine_block_begin"] and p["vert_end"] == min(32 * p["fine_block_end"], nV)
        assert p["l1_begin"] == l1_first[p["fine_block_begin"]] and p["l1_end"] == l1_first[p["fine_block_end"]]
        assert p["l1_end"] - p["l1_begin"] <= p["seg_max"] and p["seg_max"] == plan["seg_max"]

    r = meshgen.residual(nV, 5)
    o.apply(r)
    Ro = o.mapped_r()
    begin1 = int(m["level_size"][1][1]) if Lv > 1 else 0

    # own padded segment, the exchange ShardedApply issues, unpack by every plan
    seg = torch.zeros(plan["seg_max"], 4)
    cnt = plan["l1_end"] - plan["l1_begin"]
    if cnt:
        seg[:cnt, :3] = torch.from_numpy(Ro[begin1 + plan["l1_begin"]:begin1 + plan["l1_end"], :3].astype(np.float32))
    gathered = torch.empty(world * plan["seg_max"], 4)
    dist.all_gather_into_tensor(gathered, seg)
    R1 = np.full((n1, 3), np.nan, np.float32)
    for g, pg in enumerate(plans):
        c = pg["l1_end"] - pg["l1_begin"]
        R1[pg["l1_begin"]:pg["l1_end"]] = gathered[g * pg["seg_max"]:g * pg["seg_max"] + c, :3].numpy()
        assert not gathered[g * pg["seg_max"] + c:(g + 1) * pg["seg_max"]].any()   # padding stays zero
    assert np.array_equal(R1.view(np.uint32), Ro[begin1:begin1 + n1, :3].astype(np.float32).view(np.uint32))

    # owner-computes z: disjoint vertex ranges that cover every vertex
    z = o.apply(r)[:, :3]
    own = np.arange(plan["vert_begin"], plan["vert_end"])
    zfull = np.zeros((nV, 3))
    owners = np.zeros(nV)
    zfull[m["s2o"][own]] = z[m["s2o"][own]]
    owners[m["s2o"][own]] = 1
    zt, ot = torch.from_numpy(zfull), torch.from_numpy(owners)
    dist.all_reduce(zt)
    dist.all_reduce(ot)
    if rank == 0:
        assert np.all(ot.numpy() == 1)
        np.save(os.path.join(out_dir, "z.npy"), zt.numpy())
        np.save(os.path.join(out_dir, "zref.npy"), z)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,L", [(2, 40, 3), (3, 64, 0), (2, 100, 1)])
def test_sharded_protocol_gloo(tmp_path, world, W, L):
    mp.spawn(_worker, args=(world, _free_port(), W, L, str(tmp_path)), nprocs=world, join=True)
    np.testing.assert_array_equal(np.load(tmp_path / "z.npy"), np.load(tmp_path / "zref.npy"))
