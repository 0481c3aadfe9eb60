#!/usr/bin/env python3
"""bench.py -- MAS preconditioner apply throughput on MI355X.

One "step" = one Preconditioning apply (SeSchwarzPreconditioner.cpp:100-110)
of the benchmark workload on device-resident r / z (float4 [nV], the
SeVec3fSimd layout), after Allocate + Prepare.  Default workload: BASELINE.json
configs[2], the 1M-vertex cloth Hessian (1024 x 1024 grid) + 100k VF contact
stencils, 4 levels, 32-node subdomains, fp32 -- the configuration the north
star's 1-GPU roofline target is quoted on.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME]

N > 1 (one rank per GPU): the same 1M problem is sharded by Morton range
(strong scaling): rank g solves its own level-0 blocks, one RCCL allgather of
the level-1 residual segments per apply, coarse levels >= 2 redundant
(DESIGN.md §7).  value = applies of the whole problem per second (max time
over ranks).  Rank 0 prints ONE JSON line.  Run under torch.distributed.run
(WORLD_SIZE set: --gpus must equal it), or plainly as `python bench.py --gpus
N`: then this process starts `python -m torch.distributed.run --nproc-per-node
N bench.py ...` as a child before anything touches the GPU, forwards rank 0's
JSON line and exits with the child's status.  With the nccl backend every rank
needs its own device (LOCAL_RANK < device count, else a loud failure); the gloo
backend may put several ranks on one GPU (a one-GPU rehearsal of N > 1).

roofline: the dominant kernel is the fused fine-level kernel (gather r through
the Morton map, 32-node block solves, prolongation, scatter z).  Its
algorithmic bytes per launch = nFineBlocks * 18 624 B (packed fp32 inverse,
SURVEY §8(d)) + nV * (16 r + 16 z + 4 perm + 4 * (min(L,4)-1) ancestor ids);
its average duration comes from HIP events on the apply stream around `steps`
back-to-back launches of that kernel (mas_profile_fine, after the timed
region): a timing marker between the coarse launch and the fine kernel of
every apply holds the fine kernel back several microseconds, so the per-apply
events (apply_breakdown_ms, also reported) overstate it; the back-to-back
average agrees with the rocprofv3 kernel trace (profiles/round5/).
apply_breakdown_ms.coarse_back_to_back times an apply's coarse launch the
same way (mas_profile_coarse): pre_fine, from the per-apply events, carries
the marker delay.

cpu_baseline: the CPU restatement of the reference (oracle/, OpenMP, the
reference's packed layout and loop structure) on this host, bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "preconditioner-for-cloth-and-deformable-body-simulation_amd")
sys.path.insert(0, os.path.join(PKG, "python"))

METRIC = "preconditioner applies/sec + ms/apply, N-vertex 3×3-block cloth Hessian"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
CONFIG_ORDER = ["10k", "256k", "1M+contacts", "1M", "4M-tet"]   # BASELINE.json configs order
BLOCK_BYTES = 4656 * 4


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(info):
    nV, L = info["num_verts"], info["num_levels"]
    per_vertex = 16 + 16 + 4 + 4 * (min(L, 4) - 1)
    fine = info["num_fine_blocks"] * BLOCK_BYTES + nV * per_vertex
    apply = info["num_blocks"] * BLOCK_BYTES + nV * per_vertex
    return fine, apply


def _pmc_summary():
    """The newest committed PMC summary (profiles/round*/pmc_traffic.json)."""
    rounds = sorted((d for d in os.listdir(os.path.join(REPO, "profiles")) if d.startswith("round")),
                    key=lambda d: int("".join(c for c in d if c.isdigit()) or 0))
    for d in reversed(rounds):
        path = os.path.join(REPO, "profiles", d, "pmc_traffic.json")
        if os.path.exists(path):
            return path
    return None


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary (the
    counters need their own rocprofv3 passes, so they cannot be read live),
    with the commit and workload that pass measured."""
    path = _pmc_summary()
    try:
        with open(path) as f:
            d = json.load(f)
        meta = d.get("__meta__", {})
        for name, v in d.items():
            if name != "__meta__" and kernel in name:
                return int(v["corrected_bytes"]), os.path.relpath(path, REPO), meta
    except (OSError, TypeError, ValueError, KeyError):
        pass
    return None, None, {}


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": avail,
            "OMP_PROC_BIND": os.environ.get("OMP_PROC_BIND"), "OMP_PLACES": os.environ.get("OMP_PLACES")}


def cgroup_cpus():
    """CPUs the cgroup quota allows this process (None: no quota)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:          # cgroup v2: "<quota> <period>" or "max <period>"
            q, per = f.read().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(per)))
        return None
    except (OSError, ValueError):
        pass
    try:                                                   # cgroup v1
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return max(1, -(-q // per)) if q > 0 else None
    except (OSError, ValueError):
        return None


def cpu_baseline(mesh, cfg, contacts, r_np, steps):
    """OMP_NUM_THREADS = CPU_THREAD_NUM = nproc - 1 (the reference's
    WIN32 rule, SeOmp.cpp:29-33), threads pinned close, where nproc is the number
    of CPUs this process may run on: its affinity set, capped by the cgroup CPU
    quota when there is one (the GPU box shows the whole host's 256 CPUs but
    grants a share of them; 255 threads on that share measured ~40x slower).
    The raw nproc - 1 and the box's OMP_NUM_THREADS are timed beside it (shorter
    samples) when they differ."""
    os.environ["OMP_PROC_BIND"] = "close"   # before the OpenMP runtime loads
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from oracle import Oracle  # test infrastructure: the timed CPU baseline only
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 2
    quota = cgroup_cpus()
    avail = min(affinity, quota) if quota else affinity
    threads = max(1, avail - 1)
    env_threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    o = Oracle(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0], cfg["levels"], threads)
    o.allocate(mesh)
    if contacts is None:
        o.prepare(mesh)
    else:
        o.prepare(mesh, vf=contacts[0], vfC=contacts[1])

    def timed(n, k):
        o.set_threads(n)
        for _ in range(3):
            o.apply(r_np)
        ts = []
        for _ in range(k):
            t = time.perf_counter()
            z = o.apply(r_np)
            ts.append(time.perf_counter() - t)
        return statistics.median(ts), z

    med, z = timed(threads, steps)
    out = {"value": round(1.0 / med, 3), "unit": "applies/s", "cores": threads, "kind": "port", **cpu_info(),
           "cgroup_quota_cpus": quota, "OMP_NUM_THREADS_env": env_threads or None,
           "sample": f"{cfg['name']} workload, oracle/ CPU restatement (OpenMP, {threads} threads = nproc - 1 "
                     f"with nproc = {avail} CPUs available to the process, OMP_PROC_BIND=close, reference "
                     f"packed layout), median of {steps} applies after 3 warm-up; ms/apply {med * 1e3:.2f}"}
    others = {}
    if env_threads and env_threads != threads:
        others["at_OMP_NUM_THREADS_env"] = env_threads
    raw = max(1, (os.cpu_count() or 2) - 1)
    if raw != threads:
        others["at_raw_nproc_minus_1"] = raw
    for key, n in others.items():
        m2, _ = timed(n, max(3, steps // 4))
        out[key] = {"threads": n, "value": round(1.0 / m2, 3), "ms_per_apply": round(m2 * 1e3, 3)}
    return out, z


def page_aligned(a):
    """A copy of `a` starting on a page boundary, its buffer covering the last
    page whole (what mas_config.host_register asks of the caller)."""
    import numpy as np
    n = a.nbytes
    buf = np.empty(n + (-n) % 4096 + 4096, np.uint8)
    off = (-buf.ctypes.data) % 4096
    v = buf[off:off + n].view(a.dtype).reshape(a.shape)
    v[...] = a
    return v


def host_path(P, mesh, contacts, r_np, make_handle, reps=5, applies=20):
    """The drop-in host-pointer path (SeSchwarzPreconditioner.h:59-63): a PCG
    loop that already calls the reference passes host arrays, so Prepare
    copies the CSR Hessian H2D and every apply copies r in and z out.  Wall
    time of the synchronous calls, median of `reps` Prepares / `applies`
    applies after the first, on the default handle (the runtime's pageable
    staging) and on a second handle with mas_config.host_register = 1 and
    page-aligned arrays (registered at their second call, mas_capi.hip
    pin_host)."""
    import numpy as np

    def measure(h, diag, off, starts, r, cts):
        z_np = page_aligned(np.zeros_like(r))

        def prep():
            if cts is None:
                h.PreparePreconditioner(diag, off, starts)
            else:
                h.PreparePreconditioner(diag, off, starts, None, None, cts[0], None, None, cts[1])

        t = time.perf_counter()
        prep()
        first = time.perf_counter() - t
        tp, ta = [], []
        for _ in range(reps):
            t = time.perf_counter()
            prep()
            tp.append(time.perf_counter() - t)
        dev_ms = h.stats()["prepare_ms"]
        h.Preconditioning(z_np, r)
        for _ in range(applies):
            t = time.perf_counter()
            h.Preconditioning(z_np, r)
            ta.append(time.perf_counter() - t)
        return {"prepare_ms_incl_h2d": round(statistics.median(tp) * 1e3, 3),
                "prepare_first_call_ms_incl_h2d": round(first * 1e3, 3),
                "prepare_ms_device": round(dev_ms, 3),
                "apply_ms_incl_pcie": round(statistics.median(ta) * 1e3, 4)}, z_np

    nV, nnz = mesh.nV, int(mesh.starts[-1])
    pageable, z1 = measure(P, mesh.diag, mesh.off, mesh.starts, r_np, contacts)
    P2 = make_handle(host_register=True)
    registered, z2 = measure(P2, page_aligned(mesh.diag), page_aligned(mesh.off), page_aligned(mesh.starts),
                             page_aligned(r_np), contacts)
    del P2
    return {**pageable, "registered": registered,
            "z_bitwise_registered_vs_pageable": bool(np.array_equal(z1.view(np.uint32), z2.view(np.uint32))),
            "h2d_bytes_prepare": nV * 36 + nnz * 36 + (nV + 1) * 4, "pcie_bytes_apply": 2 * 16 * nV,
            "note": "host arrays through mas_prepare / mas_apply (synchronous), wall clock; top level: the default "
                    "handle (pageable staging by the runtime); registered: mas_config.host_register = 1 with "
                    "page-aligned arrays (page-locked at their second call); value and roofline use "
                    "device-resident vectors"}


PREP_KEYS = ("prepare_ms", "prepare_levels_ms", "prepare_assemble_ms", "prepare_factor_ms", "prepare_fine_ms",
             "prepare_complete_ms", "prepare_wall_ms")


class LaunchError(SystemExit):
    """A rank/device layout that cannot run: exit status 2 with the reason."""

    def __init__(self, msg):
        log(f"bench.py: {msg}")
        super().__init__(2)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(argv, gpus, env):
    """The torch.distributed.run command a plain `bench.py --gpus N` (N > 1)
    starts as its child, or None when this process is a rank already
    (WORLD_SIZE set by a launcher) or N == 1."""
    if "WORLD_SIZE" in env or gpus <= 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={free_port()}",
            os.path.abspath(__file__), *argv]


def run_launcher(cmd):
    """Run the ranks as ONE child process tree (never an exec: nothing in this
    process has touched the GPU, and nothing will); rank 0's JSON line goes to
    stdout, every other line of the children's stdout to stderr."""
    import signal
    import subprocess
    log("bench.py: launching " + " ".join(cmd[1:]))

    def die_with_parent():
        # the launcher (and through it every rank) gets SIGTERM if this
        # process dies first, e.g. killed by a driver's time limit: no rank is
        # left holding a GPU
        try:
            import ctypes
            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except OSError:
            pass

    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1, preexec_fn=die_with_parent)

    def forward(signum, _frame):  # SIGTERM / SIGINT to this process: pass it on, then wait for the ranks
        p.send_signal(signum)

    old = {sig: signal.signal(sig, forward) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        for line in p.stdout:
            s = line.strip()
            if s.startswith("{") and '"metric"' in s:
                print(s, flush=True)
            else:
                sys.stderr.write(line)
                sys.stderr.flush()
        return p.wait()
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)


def check_rank_layout(gpus, world, local, ndev, backend):
    """Under a launcher: --gpus must equal WORLD_SIZE; with nccl (RCCL) every
    rank needs a device of its own.  Returns the device index for this rank."""
    if gpus != world:
        raise LaunchError(f"--gpus {gpus} but WORLD_SIZE={world}: launch one rank per GPU "
                          f"(torch.distributed.run --nproc-per-node {gpus})")
    if ndev <= 0:
        raise LaunchError("no GPU visible (torch.cuda.device_count() == 0)")
    if local < ndev:
        return local
    if backend == "nccl":
        raise LaunchError(f"LOCAL_RANK {local} needs GPU {local}, but only {ndev} GPU(s) are visible: "
                          f"the nccl (RCCL) backend runs one rank per GPU; use --dist-backend gloo to "
                          f"rehearse {world} ranks on fewer GPUs")
    return local % ndev  # gloo rehearsal: ranks share the visible GPUs


def launch_check(args, rank, world, local):
    """--launch-check: each rank reports its layout and exits before any GPU
    work (the CPU test of the launcher)."""
    import torch
    out = {"rank": rank, "world": world, "local_rank": local, "gpus": args.gpus,
           "device_count": torch.cuda.device_count()}
    if rank == 0:
        print(json.dumps({"metric": "launch-check", **out}), flush=True)
    else:
        print(json.dumps(out), flush=True)
    # tests/test_bench_launch.py: ranks that stay up until the parent is stopped
    time.sleep(float(os.environ.get("BENCH_LAUNCH_CHECK_SLEEP", "0")))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="1M+contacts", choices=CONFIG_ORDER)
    ap.add_argument("--cpu-steps", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcg", action="store_true", help="skip the end-to-end PCG solve report")
    ap.add_argument("--no-host-path", action="store_true", help="skip the host-pointer (PCIe-inclusive) report")
    ap.add_argument("--sharded", action="store_true",
                    help="use the Morton-range sharded apply even on one GPU (overhead measurement)")
    ap.add_argument("--graph", action="store_true",
                    help="sharded path: replay one captured HIP graph per step (measured slower than eager "
                         "launches on one GPU at 1M and 256k: profiles/round1/ab/shard_overhead.json)")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "torch"],
                    help="sharded path: the handle's own RCCL communicator (mas_shard_apply_rccl, one library "
                         "call per apply) or an allgather hook through torch.distributed")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) for real runs; gloo only to exercise N>1 on one GPU")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher test: every rank reports its layout and exits before any GPU work")
    args = ap.parse_args()
    if args.gpus < 1:
        raise LaunchError(f"--gpus {args.gpus}: need at least 1")

    # N > 1 without a launcher: start the ranks as a child process before
    # anything here loads HIP (no torch.cuda call, no library load).
    cmd = launcher_command(sys.argv[1:], args.gpus, os.environ)
    if cmd is not None:
        if args.dist_backend == "nccl" and not args.launch_check:
            import torch  # device_count() does not initialise the GPU
            ndev = torch.cuda.device_count()
            if ndev < args.gpus:
                raise LaunchError(f"--gpus {args.gpus} with the nccl (RCCL) backend needs {args.gpus} GPUs, "
                                  f"{ndev} visible; use --dist-backend gloo to rehearse {args.gpus} ranks on "
                                  f"fewer GPUs")
        sys.exit(run_launcher(cmd))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        check_rank_layout(args.gpus, world, local, max(world, 1), args.dist_backend)
        launch_check(args, rank, world, local)
        return

    import numpy as np
    import torch
    import mas_amd
    from mas_amd import meshgen

    local = check_rank_layout(args.gpus, world, local, torch.cuda.device_count(), args.dist_backend)
    torch.cuda.set_device(local)
    dist = None
    sharded_path = world > 1 or args.sharded
    if sharded_path:
        import torch.distributed as dist
        if world == 1:  # a one-rank group for --sharded
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    mesh, cfg = meshgen.build_config(args.config)
    cfg = dict(cfg, name=args.config)
    contacts = meshgen.vf_contacts(mesh, cfg["contacts"], seed=3) if cfg["contacts"] else None
    t0 = time.perf_counter()
    # sharded path: each rank's Prepare assembles and factors only its own
    # level-0 blocks (mas_set_prepare_shard); the coarse levels are replicated
    P = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts, device=local,
                          shard=(rank, world) if sharded_path else None)
    setup_s = time.perf_counter() - t0
    info = P.info()
    st_first = P.stats()
    # steady-state Prepare (the per-solve call in a simulator): buffers exist,
    # repeat it and keep the median; the first call also allocates
    # A sharded Prepare (ABI 5) is mas_prepare (own coarse rows) + one
    # allgather of the coarse-row segments + mas_prepare_shard_complete; its
    # prepare_ms here is the two device parts, prepare_wall_ms the host wall
    # clock of all three (the collective included)
    from mas_amd.distributed import exchange_coarse_rows
    reps = []
    for _ in range(9):
        if dist is not None:
            dist.barrier()
        t = time.perf_counter()
        if contacts is None:
            P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
        else:
            P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, contacts[0], None, None,
                                    contacts[1])
        exchanged = sharded_path and exchange_coarse_rows(P, None, torch.device("cuda", local))
        wall_ms = (time.perf_counter() - t) * 1e3
        stp = P.stats()
        stp["prepare_wall_ms"] = wall_ms
        stp["prepare_device_only_ms"] = stp["prepare_ms"]
        if exchanged:
            stp["prepare_ms"] = stp["prepare_ms"] + stp["prepare_complete_ms"]
        reps.append(stp)
    st0 = sorted(reps, key=lambda d: d["prepare_ms"])[len(reps) // 2]  # the median of 9
    seed = 0x5EED + CONFIG_ORDER.index(args.config)
    r_np = meshgen.residual(mesh.nV, seed)
    r = torch.from_numpy(r_np).cuda()
    z = torch.zeros_like(r)
    # an explicit stream: torch's default stream handle is 0, which the C ABI
    # maps to the handle's own stream
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    def barrier():
        if dist is not None:
            dist.barrier()

    use_graph = False
    if sharded_path:  # Morton-range shards + one RCCL allgather per apply
        from mas_amd.distributed import ShardedApply
        transport = args.transport if args.dist_backend == "nccl" else "torch"
        try:
            sharded = ShardedApply(P, rank, world, device=torch.device("cuda", local), transport=transport)
        except Exception as e:  # the library's RCCL could not start: the torch hook still shards
            log(f"rccl transport unavailable ({e!r}); using the torch.distributed allgather hook")
            transport = "torch"
            sharded = ShardedApply(P, rank, world, device=torch.device("cuda", local), transport=transport)
        plan = sharded.plan
        use_graph = args.graph and args.dist_backend == "nccl"

        def step():
            sharded(z, r, stream)
    else:
        plan = None
        transport = None

        def step():
            P.PreconditioningDevice(z, r, sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if use_graph:
        sharded.capture(z, r, stream)
        for _ in range(3):
            step()
        torch.cuda.synchronize()

    # timed region: K applies, bracketed by barrier + synchronize (no
    # instrumentation inside: per-kernel events cost ~10 us per apply).
    barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier()
    wall = time.perf_counter() - w0
    elapsed = ev0.elapsed_time(ev1) / 1e3

    # kernel-duration pass: the same K applies with the library's HIP events
    # recorded on the apply stream around each kernel group (roofline source).
    if use_graph:
        sharded.graph = None  # the kernel-duration pass runs eagerly (events are recorded by the library)
    P.set_profiling(True)
    torch.cuda.synchronize()
    ev2, ev3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev2.record(stream)
    for _ in range(args.steps):
        step()
    ev3.record(stream)
    torch.cuda.synchronize()
    elapsed_ev = ev2.elapsed_time(ev3) / 1e3
    st = P.stats()
    P.set_profiling(False)
    # the roofline kernel's duration: `steps` back-to-back launches between two events
    fine_b2b_ms = P.profile_fine(z, r, args.steps, sptr) if not sharded_path else None
    # the coarse launch(es) the same way (their per-apply events carry the marker delay too)
    coarse_b2b_ms = (P.profile_coarse(r, args.steps, sptr)
                     if not sharded_path and info["num_levels"] >= 2 else None)

    t_max = elapsed
    shard_check = None
    if dist is not None:
        tt = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
        # correctness of the sharded path on this run: every rank's own z
        # entries must equal the unsharded apply's bitwise (no communication
        # needed: each rank checks its own slice, then one MIN over ranks)
        # (the reference is an unsharded handle: this rank's own one factored
        # only its shard's level-0 blocks and refuses the single-GPU apply)
        P_full = mas_amd.from_mesh(mesh, max_levels=cfg["levels"], contacts=contacts, device=local)
        z_ref = torch.zeros_like(r)
        P_full.PreconditioningDevice(z_ref, r, sptr)
        torch.cuda.synchronize()
        own = torch.from_numpy(P.maps()["s2o"][plan["vert_begin"]:plan["vert_end"]].astype(np.int64)).cuda()
        ok = torch.tensor([1.0 if torch.equal(z[own], z_ref[own]) else 0.0], device="cuda", dtype=torch.float64)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        del P_full
        # Prepare: the slowest rank's steady-state phases
        pt = torch.tensor([st0[k] for k in PREP_KEYS], device="cuda", dtype=torch.float64)
        dist.all_reduce(pt, op=dist.ReduceOp.MAX)
        st0 = dict(st0, **dict(zip(PREP_KEYS, pt.tolist())))
        props = torch.cuda.get_device_properties(local)
        me = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "handle_device": local,
              "current_device": torch.cuda.current_device(), "z_device": z.device.index,
              "gpu_uuid": str(getattr(props, "uuid", "")) or None}
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
        shard_check = {"own_slices_bitwise_equal_unsharded": bool(ok.item() == 1.0),
                       "form": "overlapped (fine during allgather)" if sharded.overlap else "serial",
                       "backend": args.dist_backend, "ranks": ranks,
                       "distinct_gpus": len({r["gpu_uuid"] or r["handle_device"] for r in ranks})}

    fine_bytes, apply_bytes = algorithmic_bytes(info)
    if plan is not None:  # the rank's own level-0 blocks and vertices
        L4 = min(info["num_levels"], 4)
        fine_bytes = ((plan["fine_block_end"] - plan["fine_block_begin"]) * BLOCK_BYTES +
                      (plan["vert_end"] - plan["vert_begin"]) * (36 + 4 * (L4 - 1)))
    # the committed PMC figure is one whole-problem launch: a sharded rank's
    # launch moves only its own slice, so N > 1 lines carry no traffic figure
    traffic = pmc_traffic("k_solve_fine") if plan is None else (None, None, {})
    fine_s = (fine_b2b_ms if fine_b2b_ms is not None else st["fine_ms_avg"]) / 1e3
    achieved = fine_bytes / fine_s / 1e9 if fine_s > 0 else None
    value = args.steps / t_max          # applies of the whole problem per second
    ms_per_step = t_max / args.steps * 1e3

    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "applies/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": {
                "10k": "10k-vertex cloth (100x100 grid), 1 level",
                "256k": "256k-vertex cloth (512x512 grid), 3 levels",
                "1M+contacts": "1M-vertex cloth (1024x1024 grid) + 100k VF contact stencils, 4 levels",
                "1M": "1M-vertex cloth (1024x1024 grid), 4 levels",
                "4M-tet": "4M-vertex tet lattice (160^3, valence 14), 4 levels",
            }[args.config],
            "name": args.config,
            "num_verts": info["num_verts"],
            "levels": info["num_levels"],
            "subdomain": 32,
            "blocks": info["num_blocks"],
            "fine_blocks": info["num_fine_blocks"],
            "contact_stencils": info["num_stencils"],
            "parallelism": (f"{world} Morton-range shards, allgather of level-1 segments via "
                            + ("the library's RCCL communicator (mas_shard_apply_rccl)" if transport == "rccl"
                               else f"a torch.distributed {args.dist_backend} hook (mas_shard_apply_device)")
                            + (", HIP-graph replay" if use_graph else ", eager launches")
                            if sharded_path else "single-gpu"),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_solve_fine (fused gather + level-0 block solves + prolongation)",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": traffic[0],
            "traffic_source": (f"{traffic[1]}: separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                               "passes of this bench command, FETCH_SIZE x2 (gfx950 wide-read correction) + "
                               "WRITE_SIZE, KB = 1024 B, per launch") if traffic[1] else
                              ("not measured per rank (the committed PMC pass is the whole single-GPU launch)"
                               if plan is not None else None),
            "traffic_measured_at": traffic[2] or None,
            "bytes_per_launch": fine_bytes,
            "avg_launch_ms": round(fine_s * 1e3, 5),
            "avg_launch_source": ("HIP events around back-to-back launches of the kernel (mas_profile_fine)"
                                  if fine_b2b_ms is not None else
                                  "HIP events the library records around the kernel in every apply"),
            "avg_launch_ms_per_apply_events": round(st["fine_ms_avg"], 5),
        },
        "apply_breakdown_ms": {
            "pre_fine": round(st["pre_fine_ms_avg"], 5),
            "coarse_back_to_back": round(coarse_b2b_ms, 5) if coarse_b2b_ms is not None else None,
            "fine_solve": round(st["fine_ms_avg"], 5),
            "post_fine": round(st["post_fine_ms_avg"], 5),
            "events_total": round(st["apply_ms_avg"], 5),
            "coarse_launches": ("none (one level)" if info["num_levels"] <= 1 else
                                "one per level" if info["num_levels"] == 2 else
                                {0: "one per level", 2: "two (k_restrict12, k_solve123)",
                                 3: "one (k_coarse1, tagged hand-offs)"}[st["apply_mode"]]),
            "ms_per_step_with_kernel_events": round(elapsed_ev / args.steps * 1e3, 5),
        },
        "apply_algorithmic_GBps": round(apply_bytes / (t_max / args.steps) / 1e9, 1),
        "apply_bytes": apply_bytes,
        "prepare_ms": round(st0["prepare_ms"], 3),
        "prepare_scope": (f"sharded Prepare, slowest of {world} ranks: own level-0 blocks and own coarse rows "
                          f"(coarse_split {st0.get('coarse_split')}), + mas_prepare_shard_complete; the coarse-row "
                          f"allgather is in prepare_wall_ms only" if sharded_path else "whole problem"),
        "prepare_wall_ms": round(st0["prepare_wall_ms"], 3),
        "prepare_first_call_ms": round(st_first["prepare_ms"], 3),
        "prepare_breakdown_ms": {"levels": round(st0["prepare_levels_ms"], 3),
                                 "assemble": round(st0["prepare_assemble_ms"], 3),
                                 "factor": round(st0["prepare_factor_ms"], 3),
                                 "level0_fused_overlapped": round(st0["prepare_fine_ms"], 3)},
        "factor_formation": ("level-0 and coarse inverses Inv = L^-T D^-1 L^-1 on the matrix cores (v_mfma_f32_32x32x2_f32)"
                             if st0.get("factor_formation") == 1 else
                             "level-0 and coarse inverses in the reference's operation order on the vector ALUs"),
        # the handle's mas_config switches (include/mas_capi.h): 0 = the tolerance-mode defaults (z within
        # 1e-5 of the reference arithmetic), 1 = the reference's own operation order, bitwise
        "mas_config": {"reference_formation": 0, "reference_restriction": 0},
        "allocate_ms": round(st0["allocate_ms"], 3),
        "host_setup_s": round(setup_s, 2),
        "wall_s_timed": round(wall, 4),
        "cpu_baseline": None,
    }
    if shard_check is not None:
        out["shard_check"] = shard_check

    if rank == 0 and world == 1 and not args.no_pcg:
        # end-to-end context (not the metric): one GPU-resident PCG solve of
        # A x = r with this preconditioner, and the unpreconditioned CG
        try:
            dd = torch.from_numpy(np.ascontiguousarray(mesh.diag, np.float32)).cuda()
            do = torch.from_numpy(np.ascontiguousarray(mesh.off, np.float32)).cuda()
            dr = torch.from_numpy(np.ascontiguousarray(mesh.starts, np.int32)).cuda()
            torch.cuda.synchronize()
            pcg = {}
            # one untimed solve first: a process's first solve also pays first-use
            # costs (0.244 vs 0.234 ms/iteration at 1M + contacts, profiles/round5/ab/)
            xw = torch.zeros_like(r)
            P.pcg_solve_device(dd, do, dr, xw, r, max_iters=5000, tol=1e-5, precondition=True, stream=sptr)
            torch.cuda.synchronize()
            for name, pre in (("mas", True), ("none", False)):
                x = torch.zeros_like(r)
                res = P.pcg_solve_device(dd, do, dr, x, r, max_iters=5000, tol=1e-5, precondition=pre,
                                         stream=sptr)
                torch.cuda.synchronize()
                pcg[name] = {k: (float(f"{v:.4g}") if isinstance(v, float) else v) for k, v in res.items()}
                pcg[name]["ms_per_iter"] = round(res["solve_ms"] / max(res["iterations"], 1), 4)
            pcg["tol"] = 1e-5
            pcg["note"] = ("Prepare excluded; the contact stencils are in the preconditioner only (A = CSR Hessian); "
                           "the second MAS solve of the process (one untimed solve first)")
            out["pcg_solve"] = pcg
        except Exception as e:  # context only
            log(f"pcg report failed: {e!r}")

    if rank == 0 and world == 1 and not args.no_host_path:
        try:
            out["host_path"] = host_path(P, mesh, contacts, r_np, lambda **kw: mas_amd.from_mesh(
                mesh, max_levels=cfg["levels"], contacts=contacts, device=local, **kw))
        except Exception as e:  # context only
            log(f"host path report failed: {e!r}")

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cb, z_cpu = cpu_baseline(mesh, cfg, contacts, r_np, args.cpu_steps)
            z_gpu = z.cpu().numpy()
            cb["z_rel_err_vs_gpu"] = float(np.linalg.norm(z_gpu[:, :3] - z_cpu[:, :3]) /
                                           np.linalg.norm(z_cpu[:, :3]))
            out["cpu_baseline"] = cb
        except Exception as e:  # the baseline is reported, never required
            log(f"cpu_baseline failed: {e!r}")

    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
