#!/bin/bash
# GPU box (round 4): the bf16x3 fc2 products at H 256 -- parity tests, the
# in-graph minibatch step and the rollout's policy launch, then one bench
# line.  The first failure ends it.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_ppo_gpu.py -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/r4_bf3_tests.log 2>&1
PROBE_H=256 timeout -k 10 120 python3 tools/minibatch_time.py 4096 512 > gpurun_out/r4_bf3_time.log 2>&1
timeout -k 10 120 python3 tools/policy_time.py >> gpurun_out/r4_bf3_time.log 2>&1
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/r4_bf3_bench.json 2> gpurun_out/r4_bf3_bench.err
grep -E "passed|failed" gpurun_out/r4_bf3_tests.log | tail -1
grep -v amdgpu.ids gpurun_out/r4_bf3_time.log
python3 -c "import json; d=json.load(open('gpurun_out/r4_bf3_bench.json')); print({k: d[k] for k in ('value','rollout_ms','update_ms','gae_ms')}); print(d['roofline']['live_marginal_avg_launch_us'])"
