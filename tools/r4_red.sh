#!/bin/bash
# GPU box (round 4): the reduce / norm-fold load rounds.  PPO / DP / C-host /
# bench GPU tests on the product library, the in-graph minibatch step of the
# product against the previous source (tools/_probe/libsatrl_redold.so, built
# here by `make variant VNAME=redold`), product first and last, then the
# product's kernel stats (r4_kprof.sh) and bench lines.  Each step has its own
# limit; a failing step ends the script.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_ppo_gpu.py tests/test_dp_gpu.py tests/test_c_host_gpu.py \
      tests/test_bench_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/red_tests.log 2>&1
fi
OLD=$ROOT/tools/_probe/libsatrl_${AB_OLD:-redold}.so
ab() {   # ab <tag> <env...>
  local tag=$1; shift
  for lib in product old product; do
    if [ "$lib" = old ]; then L=(SATRL_LIB_PATH="$OLD"); else L=(); fi
    env "${L[@]}" "$@" timeout -k 10 200 python3 tools/minibatch_time.py ${MBS:-4096 512} \
        >> gpurun_out/red_ab_$tag.log 2>&1
    echo "^ $lib" >> gpurun_out/red_ab_$tag.log
  done
}
ab h256 PROBE_H=256
MBS=4096 ab h64 PROBE_H=64
timeout -k 10 700 bash tools/r4_kprof.sh > gpurun_out/red_kprof.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/red_bench.json 2> gpurun_out/red_bench.err
timeout -k 10 300 python3 bench.py --num-envs 4096 --hidden 64 --no-cpu-baseline \
    > gpurun_out/red_bench_configs1.json 2> gpurun_out/red_bench_configs1.err
tail -c 300 gpurun_out/red_bench.json
