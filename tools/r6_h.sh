#!/bin/bash
# GPU box (round 6, pass H): the whole -m gpu suite on the round's kernels,
# then the default and configs[1] bench lines (live spans).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
rc=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/r6h_gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc" | tee gpurun_out/r6h_gpu_tests.rc
[ "$rc" -ge 124 ] && exit "$rc"
timeout -k 10 400 python3 bench.py --profile-tag r5 > gpurun_out/r6h_bench.json 2> gpurun_out/r6h_bench.err || exit 1
timeout -k 10 300 python3 bench.py --num-envs 4096 --hidden 64 --no-cpu-baseline --profile-tag r5 \
    > gpurun_out/r6h_bench_configs1.json 2> gpurun_out/r6h_bench_configs1.err
tail -c 300 gpurun_out/r6h_bench.json
