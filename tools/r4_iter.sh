#!/bin/bash
# GPU box (round 4 iterations): selected GPU tests, the probe round
# (tools/r4_probe.sh) and the two bench shapes (configs[2] default, configs[1]).
# Each step has its own limit; the first failure ends the script.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
TAG=${TAG:-r4i}
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
fi
if [ "${PROBE:-1}" = 1 ]; then
  timeout -k 10 500 bash tools/r4_probe.sh > gpurun_out/${TAG}_probe.log 2>&1
  cp -r gpurun_out/r4_probe gpurun_out/${TAG}_probe
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  timeout -k 10 200 python3 bench.py --num-envs 4096 --hidden 64 --no-cpu-baseline > gpurun_out/${TAG}_bench_c1.json 2> gpurun_out/${TAG}_bench_c1.err
fi
echo done
