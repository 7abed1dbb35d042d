#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
TAG=r6c VARIANTS="kxwt" bash tools/ab_spans.sh || exit 1
timeout -k 10 400 python3 bench.py --profile-tag r5 > gpurun_out/r6c_bench.json 2> gpurun_out/r6c_bench.err
tail -c 200 gpurun_out/r6c_bench.json
