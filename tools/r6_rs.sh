#!/bin/bash
# GPU box (round 6, pass RS): (dw2rs) dw2_kx with register-staged chunk loads
# (global_load_dwordx4 + ds_write_b128, two VGPR sets) instead of LDS-DMA:
# bitwise against the product, then span A/B at mb 4096 / 512.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
L=gpurun_out/r6rs_bitwise.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6rs_prod.npz > $L 2>&1 &&
SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_dw2rs.so timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6rs_v.npz >> $L 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r6rs_prod.npz'), np.load('gpurun_out/r6rs_v.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('dw2rs bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
rm -f gpurun_out/r6rs_*.npz
grep bitwise $L
TAG=r6rs VARIANTS="dw2rs" REPS=3 MBS=4096,512 bash tools/ab_spans.sh
