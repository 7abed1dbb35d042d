#!/bin/bash
# round 5: the whole -m gpu suite on this tree, then the dW2 split count at mb 512 / 1024
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5d_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5d_tests.log
timeout -k 10 300 python -u tools/step_ab.py 256 512 product,S=4,S=2 2 > gpurun_out/r5d_step.log 2>&1 &&
timeout -k 10 300 python -u tools/step_ab.py 256 1024 product,S=4 2 >> gpurun_out/r5d_step.log 2>&1
