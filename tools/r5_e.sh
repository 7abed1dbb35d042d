#!/bin/bash
# round 5: H 64 reduce with 16 chunks in the W2 region (product) against the
# previous build (tools/_probe/libsatrl_head.so), in-graph step, alternating;
# the H 64 parity tests on the product
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_ppo_gpu.py -k "fused_dw2_rowpass or update_matches_reference or fused_step or epoch_with_ragged" \
    tests/test_dp_gpu.py > gpurun_out/r5e_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5e_tests.log
for r in 1 2; do
  PROBE_H=64 timeout -k 10 200 python -u tools/minibatch_time.py 4096 >> gpurun_out/r5e_step.log 2>&1 &&
  SATRL_LIB_PATH=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_head.so PROBE_H=64 timeout -k 10 200 python -u tools/minibatch_time.py 4096 | sed 's/$/ [head]/' >> gpurun_out/r5e_step.log 2>&1 || exit 1
done
