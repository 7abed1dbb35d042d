#!/bin/bash
# GPU box (round 6): dw2_kx on 64 x 32 output tiles (two workgroups per CU):
# bitwise against the product, then span A/B at mb 4096 / 512.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
L=gpurun_out/r6n32_bitwise.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6n32_prod.npz 256 > $L 2>&1 || exit 1
for v in n32; do
  SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_$v.so timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6n32_$v.npz 256 >> $L 2>&1 &&
  python -c "
import numpy as np
a, b = np.load('gpurun_out/r6n32_prod.npz'), np.load('gpurun_out/r6n32_$v.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('$v bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
done
rm -f gpurun_out/r6n32_*.npz
grep bitwise $L
TAG=r6n32 VARIANTS="n32" REPS=4 MBS=4096,512 bash tools/ab_spans.sh
