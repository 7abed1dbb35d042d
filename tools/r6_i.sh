#!/bin/bash
# GPU box (round 6, pass I): osum [row][output][tile] layout (loss head reads
# partials as b128) bitwise vs the pre-change build at H 256 and H 64, then the
# in-graph step / live spans A/B against it and the dW2 depth/width variants.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
V=$ROOT/tools/_probe/libsatrl_preosum.so
L=gpurun_out/r6i_bitwise.log
for h in 256 64; do
  timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6i_new.npz $h >> $L 2>&1 &&
  SATRL_LIB_PATH=$V timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6i_old.npz $h >> $L 2>&1 &&
  python -c "
import numpy as np
a, b = np.load('gpurun_out/r6i_new.npz'), np.load('gpurun_out/r6i_old.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('H $h bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || exit 1
done
rm -f gpurun_out/r6i_*.npz
cat $L
TAG=r6i VARIANTS="preosum kxd4 kxd5 kxs16" REPS=3 bash tools/ab_spans.sh
