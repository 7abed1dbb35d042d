"""bench.py's N-rank path on a 1-GPU box: `--gpus 2 --one-device` runs two
ranks (gloo, both on cuda:0; RCCL refuses two ranks on one GPU) through the
whole bench -- launch, rollout + GAE + update per rank, barrier + max-over-
ranks timing, the data-parallel measurements and the configs[3]-semantics
slice -- and rank 0 alone prints the JSON line (the driver's 8-GPU run uses
the same code path with RCCL)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("allreduce", ["rccl", "peer"])
def test_bench_two_ranks_one_device(allreduce):
    """... and with --allreduce peer the whole update runs through the peer
    all-reduce kernel (IPC within the device); either way the line carries
    the peer kernel's all-reduce time beside the c10d path.  Both at the
    product's hidden width (256).

    Both ranks share ONE device here, so rank 0's peer all-reduce waves spin
    on CUs while rank 1's next kernel must still be placed: the peer grid is
    at most one 256-thread workgroup per CU (satrl_peer_blocks), i.e. one
    spinning wave per SIMD, which leaves every CU room for a 16-wave rowpass
    workgroup (a 641-block grid, up to three spinning waves per SIMD, starved
    it in round 4).  The peer waits are bounded by SATRL_DP_TIMEOUT_S (30 s
    here, so a stall fails the test instead of the box's hang check)."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env["SATRL_DP_TIMEOUT_S"] = "30"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--one-device",
                        "--num-envs", "512", "--horizon", "32", "--epochs", "1", "--minibatch", "4096",
                        "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--kernel-iters", "10",
                        "--global-slice", "8", "--allreduce", allreduce], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["cpu_baseline"] is None
    dp = out["data_parallel"]
    assert dp["world"] == 2 and dp["backend"] == "gloo"
    sl = dp["configs3_semantics_slice"]
    assert sl["rows_per_rank"] == 2048 and sl["us_per_global_minibatch_step"] > 0
    assert dp["allreduce"] == allreduce and dp["peer_allreduce_error"] is False and dp["peer_allreduce_us"] > 0


def test_bench_one_gpu_line_keeps_the_contract():
    """The N = 1 line the driver records: one JSON line with the contract's
    keys, the rowpass roofline (achieved = FLOP per launch / launch time,
    frac = achieved / peak) and a bounded CPU baseline of the same workload."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--num-envs", "1024", "--horizon", "64",
                        "--epochs", "1", "--minibatch", "4096", "--steps", "1", "--warmup", "1",
                        "--kernel-iters", "10", "--cpu-baseline-seconds", "1"],
                       env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert out["metric"] == base["metric"] and out["unit"] == "env-steps/s"
    assert out["n_gpus"] == 1 and out["steps"] == 1 and out["warmup"] == 1
    assert out["higher_is_better"] is True and out["scaling"] == "weak" and out["vs_baseline"] is None
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert abs(out["value"] - 1024 * 64 / (out["ms_per_step"] / 1e3)) <= 1e-6 * out["value"]
    assert "workload" in out["config"] and out["config"]["parallelism"] == "dp1"
    rf = out["roofline"]
    assert rf["bound"] == "mfma" and rf["unit"] == "TFLOP/s" and rf["peak"] == 157.3
    assert rf["achieved"] > 0 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert abs(rf["achieved"] - rf["flop_per_launch"] / rf["avg_launch_us"] / 1e6) <= 1e-6 * rf["achieved"]
    cb = out["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference") and cb["sample"]
