#!/bin/bash
# GPU box (round 4, session 3): the GPU test suite, the default and configs[1]
# bench lines, then the in-graph step A/B (tools/ab_round4.sh run) of the
# variants named in AB.  Each step has its own limit; the first failure ends it.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
TAG=${TAG:-r4s3}
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
if [ "${TESTS:-all}" != "none" ]; then
  SEL=${TESTS:-tests}
  [ "$SEL" = all ] && SEL=tests
  timeout -k 10 600 python3 -u -m pytest $SEL -m gpu -x -v --timeout 200 --timeout-method thread \
      > gpurun_out/${TAG}_tests.log 2>&1
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  timeout -k 10 200 python3 bench.py --num-envs 4096 --hidden 64 --no-cpu-baseline \
      > gpurun_out/${TAG}_bench_c1.json 2> gpurun_out/${TAG}_bench_c1.err
fi
if [ -n "${AB:-}" ]; then
  timeout -k 10 400 bash tools/ab_round4.sh run $AB > gpurun_out/${TAG}_ab.log 2>&1
fi
echo done
