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
