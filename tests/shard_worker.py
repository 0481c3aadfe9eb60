"""One rank of tests/test_gpu_shard.py::test_two_processes_gloo_drive_library
(RANK / WORLD_SIZE / MASTER_* from the environment; every rank on cuda:0)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mas_amd  # noqa: E402
from mas_amd import meshgen  # noqa: E402
from mas_amd.distributed import ShardedApply  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    mesh = meshgen.cloth_grid(128)
    contacts = meshgen.vf_contacts(mesh, 500, seed=3)
    # the reference: an unsharded handle; the rank's own: a sharded Prepare
    # (own level-0 blocks and own coarse rows), whose coarse-row exchange
    # ShardedApply runs over gloo before its first apply
    P_full = mas_amd.from_mesh(mesh, max_levels=4, contacts=contacts, device=0)
    P = mas_amd.from_mesh(mesh, max_levels=4, contacts=contacts, device=0, shard=(rank, world))
    assert P.rows_pending, "a sharded Prepare leaves its coarse rows to exchange"
    r = torch.from_numpy(meshgen.residual(mesh.nV, 77)).cuda()
    s = torch.cuda.Stream()
    z_ref = torch.zeros_like(r)
    torch.cuda.synchronize()
    P_full.PreconditioningDevice(z_ref, r, s.cuda_stream)
    S = ShardedApply(P, rank, world)
    z = torch.full_like(r, float("nan"))
    for _ in range(3):
        S(z, r, s)
    s.synchronize()
    plan = S.plan
    own = torch.from_numpy(P.maps()["s2o"][plan["vert_begin"]:plan["vert_end"]].astype(np.int64)).cuda()
    ok = torch.equal(z[own], z_ref[own]) and not P.rows_pending and P.stats()["coarse_split"] in (1, 2)
    flag = torch.tensor([1 if ok else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    dist.destroy_process_group()
    if not ok or int(flag) != 1:
        print(f"rank {rank}: own slice differs", flush=True)
        return 1
    print(f"SHARD_OK rank {rank} verts [{plan['vert_begin']}, {plan['vert_end']})", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
