#!/bin/bash
# GPU box (round 6, pass G): the XCD-matched rowpass block mapping (xmap):
# bitwise against the product, then the in-graph step / spans / gaps A/B
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
L=gpurun_out/r6g_bits.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6g_new.npz > $L 2>&1 &&
SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_xmap.so timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6g_x.npz >> $L 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r6g_new.npz'), np.load('gpurun_out/r6g_x.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || exit 1
rm -f gpurun_out/r6g_*.npz
grep differing $L
TAG=r6g VARIANTS="xmap" REPS=3 bash tools/ab_spans.sh
