#!/bin/bash
# round 5: dw2_kx slab stores widened through LDS (product: plain 16-B stores;
# dsc1: the same write-through) against the 4-B accumulator-layout stores
# (head): bitwise identity, then the in-graph step, twice
set -o pipefail
mkdir -p gpurun_out
TAG=r5s BITS=1 VNAME=head bash tools/ab_head.sh || exit 1
for r in 1 2; do
  SATRL_LIB_PATH=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_dsc1.so timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 | sed 's/$/ [dsc1]/' >> gpurun_out/r5s_ab.log 2>&1 || exit 1
done
