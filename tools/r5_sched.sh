#!/bin/bash
# round 5: the whole library built with the AMDGPU scheduler strategies
# max-ilp (schilp) and max-memory-clause (schmem) against the product
# (default strategy): bitwise, then the in-graph step and the policy launch
set -o pipefail
mkdir -p gpurun_out
TAG=r5sa BITS=1 VNAME=schilp bash tools/ab_head.sh && TAG=r5sb BITS=1 VNAME=schmem bash tools/ab_head.sh
