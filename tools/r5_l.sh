#!/bin/bash
# round 5: 16-row, 8-wave rowpass workgroups (two per CU) at every mb
# (tools/_probe/libsatrl_nw8.so) against the product: in-graph step, twice
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 python -u tools/minibatch_time.py 512 1024 2048 4096 >> gpurun_out/r5l_time.log 2>&1 &&
  SATRL_LIB_PATH=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_nw8.so timeout -k 10 120 python -u tools/minibatch_time.py 512 1024 2048 4096 | sed 's/$/ [nw8]/' >> gpurun_out/r5l_time.log 2>&1 || exit 1
done
