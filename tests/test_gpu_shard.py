"""Sharded apply on one GPU with virtual ranks: every rank's restrict, an
in-process 'allgather' (concatenation), every rank's finish into one z.  The
union must be bitwise equal to the unsharded apply (same kernels, same
arithmetic)."""
import numpy as np
import pytest

from conftest import cloth, tet

pytestmark = pytest.mark.gpu


def _virtual_sharded(P, r, world, overlap=False):
    import torch
    plans = [P.shard_setup(g, world) for g in range(world)]
    seg = plans[0]["seg_max"]
    assert all(p["seg_max"] == seg for p in plans)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):  # torch ops and the library kernels on one stream
        segs = [torch.zeros((seg, 4), dtype=torch.float32, device="cuda") for _ in range(world)]
        for g in range(world):
            P.shard_restrict(g, world, r, segs[g], s.cuda_stream)
        gathered = torch.cat(segs, 0).contiguous()
        z = torch.full_like(r, float("nan"))
        for g in range(world):
            if overlap:  # level-0 blocks first (z = Z0), then coarse + prolongation
                P.shard_fine(g, world, r, z, s.cuda_stream)
                P.shard_complete(g, world, gathered, z, s.cuda_stream)
            else:
                P.shard_finish(g, world, gathered, r, z, s.cuda_stream)
    s.synchronize()
    # ranges tile the vertices exactly
    assert plans[0]["vert_begin"] == 0 and plans[-1]["vert_end"] == r.shape[0]
    for a, b in zip(plans, plans[1:]):
        assert a["vert_end"] == b["vert_begin"] and a["l1_end"] == b["l1_begin"]
    return z


def _unsharded(P, r):
    import torch
    z = torch.zeros_like(r)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    P.PreconditioningDevice(z, r, s.cuda_stream)
    s.synchronize()
    return z


@pytest.mark.parametrize("kind,W,L,worlds,nc", [("cloth", 64, 0, (1, 2, 3, 8), 0), ("cloth", 100, 1, (2, 5), 0),
                                                ("tet", 16, 3, (2, 4), 0), ("cloth", 1024, 4, (2, 8), 0),
                                                ("cloth", 1024, 4, (8,), 100_000), ("tet", 160, 4, (8,), 0)])
@pytest.mark.parametrize("grouped", [True, False])
def test_virtual_shards_bitwise(kind, W, L, worlds, nc, grouped):
    """Includes BASELINE configs[3] (1M + 100k VF contacts, 8 ranks) and
    configs[4] (4M tet lattice, 8 ranks: ~26k level-1 nodes per rank); both
    level-3 forms (grouped: R3 from the children's R2 recomputed in the
    level-3 workgroups; reference: the fold over every gathered R1)."""
    import torch
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(W) if kind == "cloth" else tet(W)
    contacts = meshgen.vf_contacts(mesh, nc, seed=3) if nc else None
    P = mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts, reference_restriction=not grouped)
    r = torch.from_numpy(meshgen.residual(mesh.nV, 3)).cuda()
    z_ref = torch.zeros_like(r)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    P.PreconditioningDevice(z_ref, r, s.cuda_stream)
    s.synchronize()
    for world in worlds:
        for overlap in (False, True):
            z = _virtual_sharded(P, r, world, overlap)
            assert torch.equal(z, z_ref), (world, overlap, float((z - z_ref).abs().max()))


@pytest.mark.parametrize("kind,W,L,world,nc", [("cloth", 100, 3, 3, 0), ("tet", 16, 3, 2, 0),
                                               ("cloth", 1024, 4, 8, 100_000), ("tet", 160, 4, 8, 0)])
def test_shard_prepared_handles_bitwise(kind, W, L, world, nc):
    """Sharded Prepare (mas_set_prepare_shard): rank g's handle
    assembles and factors only its own level-0 blocks (plus the replicated
    coarse levels); its restrict and finish reproduce the unsharded apply's z
    on its vertices bit for bit, and its level-0 assemble + factor time
    (prepare_fine_ms) shrinks with the world.
    Such a handle refuses the single-GPU apply, other shards and other ranks'
    level-0 blocks.  Includes BASELINE configs[3] (1M + 100k VF contacts) and
    configs[4] (4M tet lattice) at 8 ranks."""
    import torch
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(W) if kind == "cloth" else tet(W)
    contacts = meshgen.vf_contacts(mesh, nc, seed=3) if nc else None
    Pf = mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts)
    r = torch.from_numpy(meshgen.residual(mesh.nV, 6)).cuda()
    z_ref = _unsharded(Pf, r)
    t_full = Pf.stats()["prepare_fine_ms"]
    ranks = [mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts, shard=(g, world)) for g in range(world)]
    mas_amd.exchange_coarse_rows(ranks)
    s = torch.cuda.Stream()
    plans = [Pg.shard_setup(g, world) for g, Pg in enumerate(ranks)]
    seg = plans[0]["seg_max"]
    # the coarse blocks a rank's sharded apply reads -- its level-1 blocks
    # and every level >= 2 block -- bitwise the unsharded Prepare's, from
    # the rows it assembled itself plus the exchanged ones (coarse_split.hip)
    info = Pf.info()
    ls, nblk, nl = info["level_size"], info["num_blocks"], info["num_levels"]
    b1 = int(ls[1][1]) // 32
    # cloth-100 / 3 ranks: the equal split cuts level-2 subtrees (every rank
    # assembles every row, mode 2); the others are clean (own rows, mode 1)
    want_mode = 2 if (kind, W, world) == ("cloth", 100, 3) else 1
    for g, Pg in enumerate(ranks):
        assert Pg.stats()["coarse_split"] == want_mode, (g, Pg.stats()["coarse_split"])
        pl = plans[g]
        ranges = [(b1 + pl["l1_begin"] // 32, b1 + (pl["l1_end"] + 31) // 32)]
        if nl > 2:
            ranges.append((int(ls[2][1]) // 32, nblk))
        for a, b in ranges:
            got, want = Pg.packed_inverses(a, b - a), Pf.packed_inverses(a, b - a)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (g, a, b)
        for blk in sorted({ranges[0][0], ranges[0][1] - 1} | (set(range(*ranges[1])) if nl > 2 else set())):
            assert np.array_equal(Pg.block_matrix(blk).view(np.uint32), Pf.block_matrix(blk).view(np.uint32)), (g, blk)
    if want_mode == 1 and b1 + 1 < ranges[0][0]:  # another rank's level-1 block is not this one's
        with pytest.raises(mas_amd.MasError, match="STATE"):
            ranks[-1].packed_inverses(b1, 1)
    with torch.cuda.stream(s):
        segs = [torch.zeros((seg, 4), dtype=torch.float32, device="cuda") for _ in range(world)]
        for g, Pg in enumerate(ranks):
            Pg.shard_restrict(g, world, r, segs[g], s.cuda_stream)
        gathered = torch.cat(segs, 0).contiguous()
        z = torch.full_like(r, float("nan"))
        for g, Pg in enumerate(ranks):
            Pg.shard_finish(g, world, gathered, r, z, s.cuda_stream)
    s.synchronize()
    assert torch.equal(z, z_ref), float((z - z_ref).abs().max())
    # a loose bound only (a shared box makes a tight one a flake source; at
    # world 8 the rank's level-0 kernel measures ~0.16x the unsharded one):
    # scripts/dev/prep_shard.py measures the per-rank Prepare
    t_rank = max(Pg.stats()["prepare_fine_ms"] for Pg in ranks)
    print(f"level-0 assemble + factor: unsharded {t_full:.3f} ms, slowest of {world} ranks {t_rank:.3f} ms")
    if mesh.nV >= 1 << 20:  # small meshes' kernels are one block's latency either way
        assert t_rank < 0.5 * t_full, (t_rank, t_full)
    P1 = ranks[1]
    with pytest.raises(mas_amd.MasError, match="STATE"):
        P1.PreconditioningDevice(torch.zeros_like(r), r, s.cuda_stream)
    with pytest.raises(mas_amd.MasError, match="STATE"):
        P1.shard_finish(0, world, gathered, r, z, s.cuda_stream)
    with pytest.raises(mas_amd.MasError, match="STATE"):
        P1.block_inverse(0)
    P1.block_inverse(plans[1]["fine_block_begin"])


def test_sharded_apply_helper_world1():
    import torch
    import mas_amd
    from mas_amd import meshgen
    from mas_amd.distributed import ShardedApply
    mesh = cloth(64)
    P = mas_amd.from_mesh(mesh, max_levels=0)
    r = torch.from_numpy(meshgen.residual(mesh.nV, 4)).cuda()
    z = torch.zeros_like(r)
    torch.cuda.synchronize()
    S = ShardedApply(P, 0, 1)
    s = torch.cuda.Stream()
    S(z, r, s)
    s.synchronize()
    assert np.array_equal(z.cpu().numpy(), P.Preconditioning(None, r.cpu().numpy()))


def test_sharded_apply_helper_overlap_world1():
    """The overlapped helper path (fine, then complete) on a one-rank world."""
    import torch
    import mas_amd
    from mas_amd import meshgen
    from mas_amd.distributed import ShardedApply
    mesh = cloth(100)
    P = mas_amd.from_mesh(mesh, max_levels=3)
    r = torch.from_numpy(meshgen.residual(mesh.nV, 9)).cuda()
    z = torch.zeros_like(r)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    for overlap in (True, False):
        S = ShardedApply(P, 0, 1, overlap=overlap)
        S(z, r, s)
        s.synchronize()
        assert np.array_equal(z.cpu().numpy(), P.Preconditioning(None, r.cpu().numpy())), overlap


@pytest.mark.parametrize("kind,W,L,worlds,nc,refr,mode", [("cloth", 100, 3, (1, 2, 3), 0, False, 0),
                                                          ("tet", 16, 3, (2, 8), 0, False, 0),
                                                          ("cloth", 100, 3, (2, 3), 0, False, 1),
                                                          ("cloth", 1024, 4, (8,), 100_000, False, 0),
                                                          ("cloth", 1024, 4, (8,), 100_000, False, 1),
                                                          ("cloth", 1024, 4, (8,), 100_000, False, 2),
                                                          ("cloth", 1024, 4, (8,), 100_000, True, 0),
                                                          ("tet", 160, 4, (8,), 0, False, 0)])
def test_one_call_shard_apply_bitwise(kind, W, L, worlds, nc, refr, mode, monkeypatch):
    """mas_shard_apply_device (the collective inside the library): with an
    in-process allgather hook -- it writes every rank's segment into `recv`
    through the step-wise restrict, so all ranks' calls run in one process --
    the union of the ranks' own z entries equals the unsharded apply bitwise,
    with the grouped level 3 and the reference's (refr), in every stream form
    (MAS_SHARD_MODE: 0 everything on the apply stream, the default; 1 / 2 the
    collective on the communication stream with the coarse levels behind it
    or after the level-0 solves).  World 1 through the loopback stand-in."""
    import torch
    import mas_amd
    from mas_amd import meshgen
    from mas_amd.distributed import device_view
    monkeypatch.setenv("MAS_SHARD_MODE", str(mode))
    mesh = cloth(W) if kind == "cloth" else tet(W)
    contacts = meshgen.vf_contacts(mesh, nc, seed=3) if nc else None
    P = mas_amd.from_mesh(mesh, max_levels=L, contacts=contacts, reference_restriction=refr)
    r = torch.from_numpy(meshgen.residual(mesh.nV, 8)).cuda()
    z_ref = _unsharded(P, r)
    s = torch.cuda.Stream()
    for world in worlds:
        calls = []

        def hook(send, recv, nbytes, strm):
            n = nbytes // 16
            calls.append(nbytes)
            dst = device_view(recv, 4 * n * world, r.device).view(world, n, 4)
            for g in range(world):  # every rank's segment, as an allgather would deliver it
                P.shard_restrict(g, world, r, dst[g], strm)

        z = torch.full_like(r, float("nan"))
        for g in range(world):
            P.shard_apply(g, world, z, r, allgather=hook if world > 1 else None, stream=s.cuda_stream)
        s.synchronize()
        assert torch.equal(z, z_ref), (world, float((z - z_ref).abs().max()))
        assert len(calls) == (world if world > 1 else 0)
    z1 = torch.full_like(r, float("nan"))
    for _ in range(2):  # the second call reuses the comm stream and tables
        P.shard_apply_loopback(0, 1, z1, r, stream=s.cuda_stream)
    s.synchronize()
    assert torch.equal(z1, z_ref)


def test_one_call_shard_apply_errors():
    import torch
    import mas_amd
    from mas_amd import meshgen
    mesh = cloth(40)
    P = mas_amd.from_mesh(mesh)
    r = torch.from_numpy(meshgen.residual(mesh.nV, 1)).cuda()
    z = torch.zeros_like(r)
    with pytest.raises(mas_amd.MasError, match="ARG"):
        P.shard_apply(0, 2, z, r)  # no allgather for world 2

    def broken(*a):
        raise RuntimeError("link down")

    with pytest.raises(mas_amd.MasError, match="link down"):
        P.shard_apply(1, 2, z, r, allgather=broken)
    with pytest.raises(mas_amd.MasError, match="STATE"):
        P.shard_apply_rccl(z, r)  # no communicator yet


def test_rccl_transport_world1():
    """The library's own RCCL communicator (dlopen'd librccl, mas_rccl_init)
    on a one-rank world: same z as the unsharded apply."""
    import torch
    import mas_amd
    from mas_amd import meshgen
    from mas_amd.distributed import ShardedApply
    mesh = cloth(100)
    P = mas_amd.from_mesh(mesh, max_levels=3)
    r = torch.from_numpy(meshgen.residual(mesh.nV, 12)).cuda()
    z_ref = _unsharded(P, r)
    S = ShardedApply(P, 0, 1, transport="rccl")
    z = torch.zeros_like(r)
    s = torch.cuda.Stream()
    for _ in range(3):
        S(z, r, s)
    s.synchronize()
    assert torch.equal(z, z_ref)
    # and an allgather over a one-rank RCCL communicator through mas_shard_apply_device's hook path
    z2 = torch.zeros_like(r)
    P.shard_apply_rccl(z2, r, s.cuda_stream)
    s.synchronize()
    assert torch.equal(z2, z_ref)
    # the one-call apply captured as a HIP graph (comm stream forked and joined inside) and replayed
    z3 = torch.zeros_like(r)
    S(z3, r, s)
    S.capture(z3, r, s)
    z3.zero_()
    torch.cuda.synchronize()
    for _ in range(2):
        S(z3, r, s)
    s.synchronize()
    assert torch.equal(z3, z_ref)


def test_two_processes_gloo_drive_library():
    """Two ranks as two processes on this GPU, gloo: each rank prepares its
    own shard (own level-0 blocks, own coarse rows), exchanges the coarse rows
    with the other process (mas_prepare_shard_rows / _complete through
    torch.distributed), runs the library's one-call sharded apply with a gloo
    allgather hook, and checks its own z entries bitwise against an unsharded
    handle's apply."""
    import os
    import subprocess
    import sys
    from conftest import REPO
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29611", WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "shard_worker.py")],
                              env=dict(env, RANK=str(g), LOCAL_RANK="0"), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for g in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
        assert "SHARD_OK" in out, out[-3000:]


def test_prepare_exchange_inside_prepare():
    """The coarse-row exchange run inside mas_prepare through a registered
    allgather hook (mas_set_prepare_allgather): rank 0 of a world of 2 whose
    hook delivers both ranks' segments (taken from two-phase rank handles)
    ends its Prepare with nothing pending, and its coarse inverses equal the
    unsharded handle's bitwise; a failing hook fails the Prepare with
    MAS_ERR_COMM."""
    import torch
    import mas_amd
    from mas_amd import meshgen
    from mas_amd.distributed import device_view
    mesh = cloth(128)
    contacts = meshgen.vf_contacts(mesh, 500, seed=3)
    Pf = mas_amd.from_mesh(mesh, max_levels=4, contacts=contacts)
    two = [mas_amd.from_mesh(mesh, max_levels=4, contacts=contacts, shard=(g, 2)) for g in range(2)]
    segs = [Pg.prepare_shard_rows() for Pg in two]
    nbytes = segs[0][1]
    dev = torch.device("cuda", torch.cuda.current_device())
    gathered = torch.cat([device_view(ptr, nbytes // 4, dev).clone() for ptr, _ in segs])
    calls = []

    def hook(send, recv, nb, strm):
        calls.append(nb)
        with torch.cuda.stream(torch.cuda.ExternalStream(strm, device=dev)):
            device_view(recv, 2 * nb // 4, dev).copy_(gathered)

    P0 = mas_amd.SeSchwarzPreconditioner(max_levels=4)
    P0.set_prepare_shard(0, 2)
    P0.set_prepare_allgather(hook)
    P0.m_positions, P0.m_neighbours, P0.m_edges, P0.m_faces = mesh.pos, (mesh.starts, mesh.idx), mesh.edges, mesh.faces
    P0.AllocatePrecoditioner(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0])
    vf, vfC = contacts
    P0.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, vf, None, None, vfC)
    assert calls == [nbytes] and not P0.rows_pending and P0.stats()["coarse_split"] in (1, 2)
    info = Pf.info()
    ls, nblk = info["level_size"], info["num_blocks"]
    plan = P0.shard_setup(0, 2)
    b1 = int(ls[1][1]) // 32
    for a, b in ((b1 + plan["l1_begin"] // 32, b1 + (plan["l1_end"] + 31) // 32), (int(ls[2][1]) // 32, nblk)):
        assert np.array_equal(P0.packed_inverses(a, b - a).view(np.uint32), Pf.packed_inverses(a, b - a).view(np.uint32))

    def broken(*a):
        raise RuntimeError("link down")

    P0.set_prepare_allgather(broken)
    with pytest.raises(mas_amd.MasError, match="COMM"):
        P0.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, vf, None, None, vfC)
