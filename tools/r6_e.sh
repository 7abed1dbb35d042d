#!/bin/bash
# GPU box (round 6, pass E): the env kernel's phase-IV solve queue -- the
# bitwise step-kernel test, then the mid-episode sweep (4k / 16k / 64k) of
# the product at each queue width against the committed env kernel
# (envhead) and a 128-VGPR build (wps4), alternating.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
L=gpurun_out/r6e_env.log
timeout -k 10 300 python3 -u -m pytest tests/test_env_gpu.py -k "agree_bitwise or autoreset_full_size or step_kernel_per_step" -v --timeout 240 --timeout-method thread > gpurun_out/r6e_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $L
[ "$rc" -ge 124 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python3 -u tools/env_sweep.py 2:64:0 2:64:1 2:64:2 2:64:4 >> $L 2>&1 || exit 1
  SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_envhead.so timeout -k 10 200 python3 -u tools/env_sweep.py 2:64 >> $L 2>&1 || exit 1
  SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_wps4.so timeout -k 10 200 python3 -u tools/env_sweep.py 2:64:0 2:64:1 >> $L 2>&1 || exit 1
done
grep -v amdgpu.ids $L
