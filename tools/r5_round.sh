#!/bin/bash
# GPU box (round 5): the whole -m gpu suite, then the r5 profile round (counter passes, env
# traces, bench under kernel stats) and an unprofiled bench reading the fresh profiles.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  # test failures are recorded and the profile round still runs; a time limit,
  # abort or crash (rc >= 124) ends the script before any further GPU step
  rc=0
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      > gpurun_out/r5_gpu_tests.log 2>&1 || rc=$?
  echo "gpu tests rc=$rc" | tee gpurun_out/r5_gpu_tests.rc
  [ "$rc" -ge 124 ] && exit "$rc"
fi
timeout -k 10 1500 bash tools/profile_round.sh r5 > gpurun_out/r5_profile.log 2>&1
timeout -k 10 400 python3 bench.py --profile-tag r5 > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err
timeout -k 10 300 python3 bench.py --num-envs 4096 --hidden 64 --no-cpu-baseline --profile-tag r5 \
    > gpurun_out/r5_bench_configs1.json 2> gpurun_out/r5_bench_configs1.err
tail -c 400 gpurun_out/r5_bench.json
