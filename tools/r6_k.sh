#!/bin/bash
# GPU box (round 6, pass K): the column-split short rowpass (rowpass_cs_kernel)
# bitwise against the committed build (tools/_probe/libsatrl_precs.so: mb 512
# and a 134-row ragged tail run it), the H 256 update / C-host GPU tests, then
# the in-graph step and live spans A/B at mb 512 and 4096.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
V=$ROOT/tools/_probe/libsatrl_precs.so
L=gpurun_out/r6k_bitwise.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6k_new.npz 256 > $L 2>&1 &&
SATRL_LIB_PATH=$V timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6k_old.npz 256 >> $L 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r6k_new.npz'), np.load('gpurun_out/r6k_old.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('H 256 bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
rm -f gpurun_out/r6k_*.npz
cat $L | grep -v amdgpu.ids
timeout -k 10 400 python3 -u -m pytest tests/test_ppo_gpu.py tests/test_c_host_gpu.py -m gpu -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/r6k_tests.log 2>&1 || { tail -40 gpurun_out/r6k_tests.log; exit 1; }
tail -3 gpurun_out/r6k_tests.log
TAG=r6k VARIANTS="precs" REPS=3 MBS=512,4096 bash tools/ab_spans.sh
