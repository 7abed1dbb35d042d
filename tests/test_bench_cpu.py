"""bench.py's host-side decisions (no GPU): which data-parallel minibatch
mode a run uses and which BASELINE.json configuration its JSON line names
(DESIGN.md §5-6).  The driver runs `bench.py --gpus N` with the defaults for
N = 1, 2, 4, 8; configs[3] is 8192 envs per GPU on 8 GPUs."""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _args(bench, *argv):
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


@pytest.mark.parametrize("world,num_envs,mode", [(1, 16384, "global"), (2, 16384, "per_gpu"),
                                                 (4, 16384, "per_gpu"), (8, 16384, "per_gpu"),
                                                 (8, 8192, "global")])
def test_auto_dp_minibatch(bench, world, num_envs, mode):
    a = _args(bench, "--num-envs", str(num_envs))
    assert a.dp_minibatch == "auto"
    assert bench.dp_mode(a, world) == mode


def test_explicit_dp_minibatch_wins(bench):
    a = _args(bench, "--dp-minibatch", "global")
    assert bench.dp_mode(a, 8) == "global"
    a = _args(bench, "--dp-minibatch", "per_gpu")
    assert bench.dp_mode(a, 1) == "per_gpu"


def test_workload_labels(bench):
    a = _args(bench)
    a.dp_minibatch = bench.dp_mode(a, 1)
    assert bench.workload_name(a, 1).startswith("BASELINE.json configs[2]:")
    for world in (2, 4, 8):
        a = _args(bench)
        a.dp_minibatch = bench.dp_mode(a, world)
        name = bench.workload_name(a, world)
        assert name.startswith("weak-scaling series of BASELINE.json configs[2]")
        assert f"global minibatch={4096 * world} (4096 rows per GPU" in name
    a = _args(bench, "--num-envs", "8192")
    a.dp_minibatch = bench.dp_mode(a, 8)
    name = bench.workload_name(a, 8)
    assert name.startswith("BASELINE.json configs[3]:") and "global minibatch=4096 (512 rows per GPU" in name
    # a per-GPU minibatch of 4096 on 8 x 8192 envs is not configs[3] (global minibatch 32768)
    a = _args(bench, "--num-envs", "8192", "--dp-minibatch", "per_gpu")
    assert not bench.workload_name(a, 8).startswith("BASELINE.json configs[3]")
    a = _args(bench, "--num-envs", "4096", "--hidden", "64")
    a.dp_minibatch = bench.dp_mode(a, 1)
    assert bench.workload_name(a, 1).startswith("BASELINE.json configs[1]:")
    a = _args(bench, "--surrogate")
    a.dp_minibatch = bench.dp_mode(a, 1)
    assert bench.workload_name(a, 1).startswith("BASELINE.json configs[4]:")


def _run_bench(*argv, env=None, timeout=180):
    import subprocess
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.pop("RANK", None)
    e.pop("LOCAL_RANK", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=e, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 4])
def test_gpus_n_launches_n_ranks_and_rank0_reports_once(n):
    """`bench.py --gpus N` (no launcher) starts N ranks itself; the process
    group has N ranks, the max-over-ranks timing and the report run, and
    exactly one JSON line comes out (rank 0's), with n_gpus from the group."""
    import json
    r = _run_bench("--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks_seen"] == n and out["steps"] == 3 and out["dry_run"]
    assert out["config"]["parallelism"] == f"dp{n}"


def test_gpus_1_stays_one_process():
    import json
    r = _run_bench("--dry-run", "--steps", "2", "--warmup", "0")
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 1 and out["ranks_seen"] == 1


def test_world_size_must_match_gpus():
    r = _run_bench("--gpus", "2", "--dry-run", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "--gpus 2 but WORLD_SIZE=1" in r.stderr


def test_lost_rank_ends_the_run_nonzero():
    """A rank that dies mid-run (exit 7 before the closing barrier): the other
    rank's collective fails, satrl.dist.run_or_exit aborts and exits non-zero
    (3), the launcher stops and reports a failure -- within the deadline, no
    hang."""
    import time
    t0 = time.time()
    r = _run_bench("--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1",
                   env={"SATRL_DRY_RUN_FAIL_RANK": "1", "SATRL_DP_TIMEOUT_S": "30"}, timeout=120)
    assert r.returncode != 0
    assert time.time() - t0 < 90
    assert not [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]


def test_surviving_rank_exits_nonzero_on_its_own():
    """Under an external launcher (torchrun-style env, no bench.py parent to
    stop it), the surviving rank itself detects the lost peer at its next
    collective and exits with satrl.dist.EXIT_PEER_FAILURE within the
    deadline."""
    import socket
    import subprocess
    import time
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
    procs = []
    for r in range(2):
        e = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                 MASTER_PORT=port, SATRL_DRY_RUN_FAIL_RANK="1", SATRL_DP_TIMEOUT_S="30")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                                       "--steps", "2", "--warmup", "1"], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    t0 = time.time()
    out0, err0 = procs[0].communicate(timeout=120)
    procs[1].communicate(timeout=60)
    assert procs[1].returncode == 7
    assert procs[0].returncode == 3, err0[-2000:]
    assert "data-parallel failure, aborting" in err0
    assert time.time() - t0 < 90
