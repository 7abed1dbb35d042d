#!/bin/bash
# GPU box (round 4): dw2_kx on 128x128 output tiles (variant kxt128) against
# the product's 64x64: the k-packed parity test on both builds, then the
# in-graph step (product / variant / product).  Each step has its own limit.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
V=$ROOT/tools/_probe/libsatrl_kxt128.so
timeout -k 10 200 python3 -u -m pytest tests/test_ppo_gpu.py -m gpu -q -x --timeout 100 --timeout-method thread \
    -k "kx_rowpass or fused_step_vs_torch" > gpurun_out/kxt_tests_product.log 2>&1
SATRL_LIB_PATH=$V timeout -k 10 200 python3 -u -m pytest tests/test_ppo_gpu.py -m gpu -q -x --timeout 100 \
    --timeout-method thread -k "kx_rowpass or fused_step_vs_torch" > gpurun_out/kxt_tests_variant.log 2>&1
AB_H64=0 timeout -k 10 400 bash tools/ab_round4.sh run kxt128 > /dev/null 2>&1
grep -v amdgpu.ids gpurun_out/ab_round4.log | grep "==\|us per"
