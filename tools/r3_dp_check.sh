#!/bin/bash
# GPU box: pin the dW2 table, run the dW2/DP GPU tests, rehearse `bench.py --gpus 2`
# on one device (gloo) and a short 1-GPU bench.  Each GPU step has its own limit.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/dw2_pin.py gpurun_out/dw2_plans.json > gpurun_out/dw2_pin.log 2>&1
cp gpurun_out/dw2_plans.json ppo-rl-satellite_amd/satrl/dw2_plans.json
timeout -k 10 600 python3 -u -m pytest tests/test_dw2_plans_gpu.py tests/test_dp_gpu.py -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/dp_tests.log 2>&1
timeout -k 10 300 python3 -u bench.py --gpus 2 --one-device --num-envs 1024 --horizon 64 --epochs 2 --steps 2 \
    --warmup 1 --no-cpu-baseline --kernel-iters 20 --global-slice 16 > gpurun_out/bench_rehearsal.json \
    2> gpurun_out/bench_rehearsal.err
timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_n1.json \
    2> gpurun_out/bench_n1.err
tail -c 600 gpurun_out/bench_n1.json
