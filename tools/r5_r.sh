#!/bin/bash
# round 5: dw2_kx upper bounds -- timing-only builds without the slab stores
# (dnost) or without the MFMA loop body (dnomf), in-graph step at mb 4096 / 512
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 >> gpurun_out/r5r.log 2>&1 || exit 1
  for v in dnost dnomf; do
    SATRL_LIB_PATH=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_$v.so timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 | sed "s/\$/ [$v]/" >> gpurun_out/r5r.log 2>&1 || exit 1
  done
done
