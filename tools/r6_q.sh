#!/bin/bash
# GPU box (round 6, final pass): the whole -m gpu suite on the round's last
# kernels, then the unprofiled bench lines that read profiles/r6_*: the
# default (configs[2]), configs[1], configs[4] (--surrogate) and ten timed
# iterations.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
rc=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/r6q_gpu_tests.log 2>&1 || rc=$?
echo "gpu tests rc=$rc" | tee gpurun_out/r6q_gpu_tests.rc
tail -3 gpurun_out/r6q_gpu_tests.log
[ "$rc" -ne 0 ] && exit "$rc"
timeout -k 10 400 python3 bench.py > gpurun_out/r6q_bench.json 2> gpurun_out/r6q_bench.err || exit 1
timeout -k 10 300 python3 bench.py --num-envs 4096 --hidden 64 --no-cpu-baseline \
    > gpurun_out/r6q_bench_configs1.json 2> gpurun_out/r6q_bench_configs1.err || exit 1
timeout -k 10 400 python3 bench.py --surrogate --no-cpu-baseline > gpurun_out/r6q_bench_configs4.json \
    2> gpurun_out/r6q_bench_configs4.err || exit 1
timeout -k 10 600 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r6q_bench_10steps.json \
    2> gpurun_out/r6q_bench_10steps.err || exit 1
for f in r6q_bench r6q_bench_configs1 r6q_bench_configs4 r6q_bench_10steps; do
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('rocprof_avg_launch_us'))"
done
