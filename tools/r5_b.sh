#!/bin/bash
# round 5: the reference-pinned H 256 update tests and the hand-written mb <= 1024
# path (k-packed planes from the 16-row rowpass; no hipBLASLt), the C host, the
# peer all-reduce (capped grid, deadline, reset); then the in-graph step, round-4
# tree (tools/_probe/r4tree: hipBLASLt at mb 512) against this tree
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_ppo_gpu.py -k "update_matches_reference or kx_rowpass or fused_step or epoch_with_ragged or logp_equals or fused_dw2_reduce" \
    tests/test_c_host_gpu.py tests/test_dp_gpu.py -s > gpurun_out/r5b_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5b_tests.log
timeout -k 10 200 python -u tools/_probe/r4tree/tools/minibatch_time.py 512 4096 > gpurun_out/r5b_step.log 2>&1 &&
timeout -k 10 200 python -u tools/minibatch_time.py 512 4096 >> gpurun_out/r5b_step.log 2>&1 &&
timeout -k 10 200 python -u tools/_probe/r4tree/tools/minibatch_time.py 512 >> gpurun_out/r5b_step.log 2>&1 &&
timeout -k 10 200 python -u tools/minibatch_time.py 512 777 >> gpurun_out/r5b_step.log 2>&1 &&
timeout -k 10 300 python -u tools/step_ab.py 256 4096 product,fuse_reduce=0 2 >> gpurun_out/r5b_step.log 2>&1 &&
PROBE_H=64 timeout -k 10 200 python -u tools/minibatch_time.py 4096 >> gpurun_out/r5b_step.log 2>&1 &&
PROBE_H=64 timeout -k 10 200 python -u tools/_probe/r4tree/tools/minibatch_time.py 4096 >> gpurun_out/r5b_step.log 2>&1
