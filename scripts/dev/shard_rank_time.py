"""Per-rank compute of the Morton-range sharded apply, measured on ONE GPU:
rank g of a world of W runs restrict -> (allgather replaced by a device copy
of its own segment; the communication is NOT in these numbers) -> finish;
mode one_call: mas_shard_apply_device with the loopback stand-in
(mas_allgather_loopback), in the stream form MAS_SHARD_MODE selects.
Prints ms per apply for every (W, g) so the critical path of an N-GPU apply
can be read as max_g(compute) + allgather.  Dev tool; GPU only."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "preconditioner-for-cloth-and-deformable-body-simulation_amd", "python"))
import torch  # noqa: E402
import mas_amd  # noqa: E402
from mas_amd import meshgen  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "1M+contacts"
worlds = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4,8").split(",")]
mesh, cfg = meshgen.build_config(cfg_name)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts)
r = torch.from_numpy(meshgen.residual(mesh.nV, 5)).cuda()
z = torch.zeros_like(r)
s = torch.cuda.Stream()
out = {}
steps = 200
modes = (sys.argv[3] if len(sys.argv) > 3 else "finish,fine_then_complete,one_call").split(",")
for W, mode in [(w, m) for w in worlds for m in modes]:
    for g in sorted({0, W - 1}):
        plan = P.shard_setup(g, W)
        seg = torch.zeros((plan["seg_max"], 4), dtype=torch.float32, device="cuda")
        gathered = torch.zeros((W * plan["seg_max"], 4), dtype=torch.float32, device="cuda")
        dst = gathered[g * plan["seg_max"]:(g + 1) * plan["seg_max"]]

        def step():
            if mode == "one_call":  # mas_shard_apply_device (MAS_SHARD_MODE)
                P.shard_apply_loopback(g, W, z, r, s.cuda_stream)
                return
            P.shard_restrict(g, W, r, seg, s.cuda_stream)
            with torch.cuda.stream(s):
                dst.copy_(seg)
            if mode == "fine_then_complete":
                P.shard_fine(g, W, r, z, s.cuda_stream)
                P.shard_complete(g, W, gathered, z, s.cuda_stream)
            else:
                P.shard_finish(g, W, gathered, r, z, s.cuda_stream)

        for _ in range(20):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(steps):
            step()
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
        P.set_profiling(True)
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        st = P.stats()
        P.set_profiling(False)
        key = f"W{W}/rank{g}/{mode}"
        out[key] = {"ms_per_apply": round(ms, 5), "pre_fine_ms": round(st["pre_fine_ms_avg"], 5),
                                "fine_ms": round(st["fine_ms_avg"], 5), "post_fine_ms": round(st["post_fine_ms_avg"], 5),
                                "fine_blocks": plan["fine_block_end"] - plan["fine_block_begin"]}
        print(key, out[key], flush=True)
print(json.dumps({"config": cfg_name, "note": "per-rank compute only; allgather replaced by a local copy", **out}))
