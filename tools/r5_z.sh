#!/bin/bash
# round 5: the next group's rows staged on a forked branch of each graph
# (two graphs, two stage buffers): graph-vs-eager and update tests, then the
# in-graph step and a bench line
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_ppo_gpu.py -k "graph_groups or folded or update_matches_reference or full_size or ragged_tail" > gpurun_out/r5z_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/minibatch_time.py 512 4096 > gpurun_out/r5z_time.log 2>&1 &&
PROBE_H=64 timeout -k 10 300 python -u tools/minibatch_time.py 4096 >> gpurun_out/r5z_time.log 2>&1 &&
timeout -k 10 420 python3 bench.py --profile-tag r5 > gpurun_out/r5z_bench.json 2> gpurun_out/r5z_bench.err
