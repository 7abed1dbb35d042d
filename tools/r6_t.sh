#!/bin/bash
# GPU box (round 6, pass T): wave 0's k-packed H1 stores of the 32-row
# rowpass after the post-head barrier (w0late) or an LDS-only post-head
# barrier (ldsbar): bitwise against the product, then in-graph A/B.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
L=gpurun_out/r6t_bitwise.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6t_prod.npz 256 > $L 2>&1 || exit 1
for v in ${VARIANTS:-w0late ldsbar}; do
  SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_$v.so timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6t_$v.npz 256 >> $L 2>&1 &&
  python -c "
import numpy as np
a, b = np.load('gpurun_out/r6t_prod.npz'), np.load('gpurun_out/r6t_$v.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('$v bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
done
rm -f gpurun_out/r6t_*.npz
grep bitwise $L
TAG=r6t VARIANTS="${VARIANTS:-w0late ldsbar}" REPS=4 MBS=4096 bash tools/ab_spans.sh
