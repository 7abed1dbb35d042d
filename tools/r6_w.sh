#!/bin/bash
# GPU box (round 6, pass W): (hsplit) the actor's loss-head chain split over
# waves 0-2, one output dimension each; (cs1024) the column-split rowpass up
# to 1024 rows: bitwise against the product, then span A/B (hsplit at mb
# 4096, cs1024 at mb 1024 / 768).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
L=gpurun_out/r6w_bitwise.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6w_prod.npz 256 > $L 2>&1 || exit 1
for v in hsplit cs1024; do
  SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_$v.so timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6w_$v.npz 256 >> $L 2>&1 &&
  python -c "
import numpy as np
a, b = np.load('gpurun_out/r6w_prod.npz'), np.load('gpurun_out/r6w_$v.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('$v bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
done
rm -f gpurun_out/r6w_*.npz
grep bitwise $L
TAG=r6w VARIANTS="hsplit" REPS=4 MBS=4096 bash tools/ab_spans.sh || exit 1
TAG=r6w2 VARIANTS="cs1024" REPS=3 MBS=1024,768 bash tools/ab_spans.sh
