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


def test_bench_two_ranks_one_device():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--one-device",
                        "--num-envs", "512", "--horizon", "32", "--epochs", "1", "--minibatch", "4096",
                        "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--kernel-iters", "10",
                        "--global-slice", "8"], env=env, capture_output=True, text=True, timeout=240)
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
