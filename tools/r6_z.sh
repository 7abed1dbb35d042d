#!/bin/bash
# GPU box (round 6, pass Z): (hsplit64) the H 64 actor's loss-head chain split
# over waves 0-2 (one output dimension each, one wave per SIMD there):
# bitwise against the product at H 64, then span A/B at configs[1]'s mb 4096.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
L=gpurun_out/r6z_bitwise.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6z_prod.npz 64 > $L 2>&1 &&
SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_hsplit64.so timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6z_v.npz 64 >> $L 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r6z_prod.npz'), np.load('gpurun_out/r6z_v.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('hsplit64 bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
rm -f gpurun_out/r6z_*.npz
grep bitwise $L
TAG=r6z H=64 VARIANTS="hsplit64" REPS=4 MBS=4096 bash tools/ab_spans.sh
