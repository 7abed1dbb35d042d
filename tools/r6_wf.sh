#!/bin/bash
# GPU box (round 6, pass WF): (w1first) the fused dW2 + W1 / tail launch with
# its reduce blocks dealt first (padded to a multiple of 8): bitwise against
# the product, then span A/B at mb 4096 / 512.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
L=gpurun_out/r6wf_bitwise.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6wf_prod.npz > $L 2>&1 &&
SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_w1first.so timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6wf_v.npz >> $L 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r6wf_prod.npz'), np.load('gpurun_out/r6wf_v.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('w1first bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
rm -f gpurun_out/r6wf_*.npz
grep bitwise $L
TAG=r6wf VARIANTS="w1first" REPS=3 MBS=4096,512 bash tools/ab_spans.sh
