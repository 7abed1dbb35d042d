#!/bin/bash
# One GPU-box pass (gpurun): the GPU test suite, the rocprof profile round
# (PMC passes + bench under kernel stats, tools/profile_round.sh) and an
# unprofiled bench that reads the fresh profiles.  Every step has its own
# time limit; the first failure ends the script.  A heartbeat file under
# gpurun_out/ shows progress.
set -euo pipefail
TAG=${1:-r2}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
{ cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max"; nproc; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}";
  python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))'; } > gpurun_out/host_info.txt 2>&1
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_gpu_tests.log 2>&1
fi
if [ "${SKIP_PROFILE:-0}" != "1" ]; then
  timeout -k 10 1000 bash tools/profile_round.sh "$TAG" > gpurun_out/${TAG}_profile.log 2>&1
fi
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
tail -1 gpurun_out/${TAG}_bench.json
