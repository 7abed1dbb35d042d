#!/bin/bash
# round 5: fc1 on the split-bf16 MFMA (product) vs the f32 16x16x4 chain
# (tools/_probe/libsatrl_head.so): in-graph step A/B, then the update / rollout parity tests
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_head.so
for r in 1 2; do
  timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 >> gpurun_out/r5i_time.log 2>&1 &&
  SATRL_LIB_PATH=$V timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 | sed 's/$/ [head]/' >> gpurun_out/r5i_time.log 2>&1 &&
  timeout -k 10 120 python -u tools/policy_time.py >> gpurun_out/r5i_time.log 2>&1 &&
  SATRL_LIB_PATH=$V timeout -k 10 120 python -u tools/policy_time.py | sed 's/$/ [head]/' >> gpurun_out/r5i_time.log 2>&1 || exit 1
done
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_ppo_gpu.py tests/test_rd_gpu.py tests/test_dropin_gpu.py tests/test_c_host_gpu.py > gpurun_out/r5i_tests.log 2>&1
