#!/bin/bash
# round 5: the env step kernels per env count (wide at 64 / 32 / 16 envs per
# workgroup, the split kernel), and the policy launch with the split-ahead
# forward (tools/_probe/libsatrl_polsa.so) against the product
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/env_sweep.py 2:64 2:32 2:16 1:64 > gpurun_out/r5g_env.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 120 python -u tools/policy_time.py >> gpurun_out/r5g_pol.log 2>&1 &&
  SATRL_LIB_PATH=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_polsa.so timeout -k 10 120 python -u tools/policy_time.py | sed 's/$/ [polsa]/' >> gpurun_out/r5g_pol.log 2>&1 || exit 1
done
