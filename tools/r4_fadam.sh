#!/bin/bash
# GPU box (round 4): the deferred-Adam H 64 step -- its parity tests, then the
# in-graph minibatch step with and without it.  The first failure ends the script.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = "1" ] || timeout -k 10 300 python3 -u -m pytest tests/test_ppo_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "deferred or fused_dw2 or ragged_tail or graph_groups or fused_step or logp_equals" > gpurun_out/r4_fadam_tests.log 2>&1
for FA in 1 0; do
  SATRL_FUSED_ADAM=$FA PROBE_H=64 timeout -k 10 120 python3 tools/minibatch_time.py 4096 512 4096 \
      >> gpurun_out/r4_fadam_time.log 2>&1
done
cat gpurun_out/r4_fadam_time.log
