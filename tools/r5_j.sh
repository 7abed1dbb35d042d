#!/bin/bash
# round 5: what bounds the split-bf16 fc2 phases now -- timing-only builds
# without weight loads (fakeb), without the split VALU (nosplit), neither (both)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 >> gpurun_out/r5j_time.log 2>&1 || exit 1
  for v in fakeb nosplit both; do
    SATRL_LIB_PATH=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_$v.so timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 | sed "s/\$/ [$v]/" >> gpurun_out/r5j_time.log 2>&1 || exit 1
  done
done
