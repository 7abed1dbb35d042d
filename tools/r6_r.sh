#!/bin/bash
# GPU box (round 6, pass R): net-per-XCD placement of the 32-row rowpass and
# dw2_kx (tools/_probe/libsatrl_nx.so: XCD x holds net x & 1 and splits
# 2(x>>1), 2(x>>1)+1) bitwise and in-graph A/B against the product.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
V=$ROOT/tools/_probe/libsatrl_nx.so
L=gpurun_out/r6r_bitwise.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6r_new.npz 256 > $L 2>&1 &&
SATRL_LIB_PATH=$V timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6r_old.npz 256 >> $L 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r6r_new.npz'), np.load('gpurun_out/r6r_old.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('H 256 bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
rm -f gpurun_out/r6r_*.npz
grep bitwise $L
TAG=r6r VARIANTS="nx" REPS=4 MBS=4096 bash tools/ab_spans.sh
