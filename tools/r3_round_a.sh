#!/bin/bash
# GPU box: the whole -m gpu suite, then the r3 profile round (counter passes, env
# traces, bench under kernel stats) and an unprofiled bench reading the fresh profiles.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/r3_gpu_tests.log 2>&1
fi
timeout -k 10 1500 bash tools/profile_round.sh r3 > gpurun_out/r3_profile.log 2>&1
timeout -k 10 400 python3 bench.py --profile-tag r3 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err
tail -c 400 gpurun_out/r3_bench.json
