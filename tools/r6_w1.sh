#!/bin/bash
# GPU box (round 6, pass W1): the reduce's W1 / tail regions inside the dW2
# launch (satrl_ppo_dw2_kx_w1): its GPU tests, whole updates + rollouts
# bitwise against the previous commit's build (tools/_probe/libsatrl_head.so,
# which falls back to dw2_kx + the full reduce), then span A/B.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
L=gpurun_out/r6w1_tests.log
timeout -k 10 400 python -u -m pytest tests/test_ppo_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "dw2_kx_w1 or kx_rowpass or update_matches_reference_h256 or exchange" > $L 2>&1 || { tail -40 $L; exit 1; }
tail -3 $L
L=gpurun_out/r6w1_bitwise.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6w1_prod.npz > $L 2>&1 &&
SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_head.so timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6w1_v.npz >> $L 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r6w1_prod.npz'), np.load('gpurun_out/r6w1_v.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('w1-fused vs head bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
rm -f gpurun_out/r6w1_*.npz
grep bitwise $L
TAG=r6w1 VARIANTS="head" REPS=3 MBS=4096,512 bash tools/ab_spans.sh
