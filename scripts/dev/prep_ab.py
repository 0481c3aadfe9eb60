"""Interleaved A/B of a creation-time env knob on steady-state Prepare:
python scripts/dev/prep_ab.py <config> <VAR> <a,b,...> [reps]
One handle per value (the knob is read by mas_create), Prepares alternated so
box noise hits every value alike; prints the median and min per value.
Each handle owns up to three HIP streams: with more streams in the process
than GPU_MAX_HW_QUEUES (4) some share a hardware queue, so a knob whose value
is stream overlap cannot be compared this way."""
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "../../preconditioner-for-cloth-and-deformable-body-simulation_amd/python"))

import mas_amd
from mas_amd import meshgen

cfg_name, var, vals = sys.argv[1], sys.argv[2], sys.argv[3].split(",")
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 8
mesh, cfg = meshgen.build_config(cfg_name)
contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
handles = []
for v in vals:
    os.environ[var] = v
    handles.append(mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts))
times = {v: [] for v in vals}
for r in range(reps + 1):
    for v, P in zip(vals, handles):
        if contacts is None:
            P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
        else:
            P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, contacts[0], None, None, contacts[1])
        if r:  # the first round warms up
            times[v].append(P.stats()["prepare_ms"])
for v in vals:
    t = times[v]
    print(f"{cfg_name} {var}={v}: median {statistics.median(t):.3f} ms, min {min(t):.3f} ms ({len(t)} reps)", flush=True)
