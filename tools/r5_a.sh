#!/bin/bash
# round 5, first GPU call: the reference-pinned H 256 update tests, then the
# in-graph minibatch step at the product shapes (baseline for this round)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ppo_gpu.py \
    -k "update_matches_reference" -s > gpurun_out/r5a_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/minibatch_time.py 4096 512 > gpurun_out/r5a_step.log 2>&1 &&
PROBE_H=64 timeout -k 10 300 python -u tools/minibatch_time.py 4096 >> gpurun_out/r5a_step.log 2>&1
