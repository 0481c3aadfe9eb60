"""bench.py's rank launch (CPU): `python bench.py --gpus N` must run N ranks by
itself, a launcher's WORLD_SIZE must match --gpus, and the nccl backend must
refuse ranks without a GPU of their own instead of sharing one."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_launcher_command_only_without_a_launcher():
    assert bench.launcher_command(["--gpus", "1"], 1, {}) is None
    assert bench.launcher_command(["--gpus", "4"], 4, {"WORLD_SIZE": "4"}) is None
    cmd = bench.launcher_command(["--gpus", "4", "--steps", "7"], 4, {})
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "7"]
    assert os.path.samefile(cmd[-5], os.path.join(REPO, "bench.py"))


def test_rank_layout_checks():
    assert bench.check_rank_layout(8, 8, 5, 8, "nccl") == 5
    with pytest.raises(SystemExit) as e:  # --gpus disagrees with the launcher
        bench.check_rank_layout(8, 2, 0, 8, "nccl")
    assert e.value.code == 2
    with pytest.raises(SystemExit):       # nccl: rank 1 has no GPU of its own
        bench.check_rank_layout(2, 2, 1, 1, "nccl")
    with pytest.raises(SystemExit):       # no GPU at all
        bench.check_rank_layout(1, 1, 0, 0, "gloo")
    assert bench.check_rank_layout(2, 2, 1, 1, "gloo") == 0  # gloo rehearsal shares the GPU


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=REPO)


@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_plain_bench_launches_n_ranks(backend):
    p = _run(["--gpus", "2", "--launch-check", "--dist-backend", backend])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout  # rank 0's line only; the other rank's output goes to stderr
    d = json.loads(lines[0])
    assert d["metric"] == "launch-check" and d["rank"] == 0 and d["world"] == 2 and d["gpus"] == 2
    assert '"rank": 1' in p.stderr  # rank 1 ran too


def test_launcher_world_mismatch_fails():
    p = _run(["--gpus", "3", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr


def test_launcher_ranks_end_with_the_parent():
    """A parent bench.py that is terminated takes its launcher and every rank
    with it (signal forwarding + PR_SET_PDEATHSIG): nothing is left holding a
    GPU after a driver's time limit."""
    import signal
    import threading
    import time
    import psutil
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", BENCH_LAUNCH_CHECK_SLEEP="120")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.Popen([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--launch-check",
                          "--dist-backend", "gloo"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         env=env, cwd=REPO, start_new_session=True)
    err = []
    threading.Thread(target=lambda: err.extend(p.stderr), daemon=True).start()
    try:
        deadline = time.time() + 150
        while time.time() < deadline and not any('"rank": 1' in l for l in err):
            time.sleep(0.5)
        assert any('"rank": 1' in l for l in err), "".join(err)[-2000:]
        tree = psutil.Process(p.pid).children(recursive=True)  # the launcher and its ranks (own sessions)
        assert len(tree) >= 3, tree
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) != 0
        gone, alive = psutil.wait_procs(tree, timeout=30)
        assert not alive, [q.pid for q in alive]
    finally:
        for q in locals().get("tree", []):
            try:
                q.kill()
            except psutil.Error:
                pass
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
