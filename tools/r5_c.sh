#!/bin/bash
# round 5: parity of the H 256 update vs the reference fixtures and of the fused
# dW2 + reduce; then the in-graph step A/B: fused (write-through slabs / release
# fence) vs two launches vs the round-4 tree, at mb 4096 and 512, and rocprof
# kernel stats of the mb-512 step (this tree two-launch, round-4 tree)
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_ppo_gpu.py -k "update_matches_reference or fused_dw2_reduce or kx_rowpass" -s \
    > gpurun_out/r5c_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5c_tests.log
timeout -k 10 300 python -u tools/step_ab.py 256 4096 product,fuse_reduce=2,fuse_reduce=0 2 > gpurun_out/r5c_step.log 2>&1 &&
timeout -k 10 300 python -u tools/step_ab.py 256 512 product,fuse_reduce=2,fuse_reduce=0 2 >> gpurun_out/r5c_step.log 2>&1 &&
timeout -k 10 200 python -u tools/_probe/r4tree/tools/minibatch_time.py 512 4096 >> gpurun_out/r5c_step.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5c_p512 -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/step_ab.py 256 512 fuse_reduce=0 1 > /dev/null 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5c_r4_512 -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/_probe/r4tree/tools/minibatch_time.py 512 > /dev/null 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5c_p4096 -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/step_ab.py 256 4096 product 1 > /dev/null 2>&1
rm -f $GRAFT_REPO_ROOT/gpurun_out/r5c_*/run_kernel_trace.csv
