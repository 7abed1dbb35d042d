#!/bin/bash
# GPU box (round 4): the split-bf16 dW2 kernel at H 256 -- its parity test,
# then the in-graph step against the library GEMM (SATRL_DW2_LIB=1)
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_ppo_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "dw2_kernel_vs_torch or fused_step or ragged_tail or graph_groups or logp_equals" > gpurun_out/r4_dw2_tests.log 2>&1
for E in SATRL_DW2_LIB=0 SATRL_DW2_LIB=1 SATRL_DW2_LIB=0; do
  env $E PROBE_H=256 timeout -k 10 120 python3 tools/minibatch_time.py 4096 512 2>&1 | grep -v amdgpu.ids | sed "s/^/$E /" >> gpurun_out/r4_dw2_time.log
done
grep -E "passed|failed" gpurun_out/r4_dw2_tests.log | tail -1
cat gpurun_out/r4_dw2_time.log
