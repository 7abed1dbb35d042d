#!/bin/bash
# GPU box (round 6): rows-first gather (the staged rows' loads before the
# weight loads, an LDS-only barrier after the gather): bitwise against the
# product at H 256 and H 64, then span A/B at mb 4096 at both widths.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
L=gpurun_out/r6rf_bitwise.log
: > $L
for h in 256 64; do
  timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6rf_prod.npz $h >> $L 2>&1 &&
  SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_rf.so timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6rf_v.npz $h >> $L 2>&1 &&
  python -c "
import numpy as np
a, b = np.load('gpurun_out/r6rf_prod.npz'), np.load('gpurun_out/r6rf_v.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('rf H $h bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
done
rm -f gpurun_out/r6rf_*.npz
grep bitwise $L
TAG=r6rf VARIANTS="rf" REPS=4 MBS=4096 bash tools/ab_spans.sh || exit 1
TAG=r6rf64 H=64 VARIANTS="rf" REPS=4 MBS=4096 bash tools/ab_spans.sh
