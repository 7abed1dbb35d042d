#!/bin/bash
# GPU box (round 6, pass RO): reduce_kernel dealing its W1 / tail blocks the
# lowest workgroup ids (logical block order unchanged): bitwise against the
# previous commit's build at H 256 and H 64, the update GPU tests, then span
# A/B at configs[1] (H 64, mb 4096) and H 256.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
L=gpurun_out/r6ro_bitwise.log
: > $L
for H in 256 64; do
  timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6ro_prod.npz $H >> $L 2>&1 &&
  SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_head.so timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6ro_v.npz $H >> $L 2>&1 &&
  python -c "
import numpy as np
a, b = np.load('gpurun_out/r6ro_prod.npz'), np.load('gpurun_out/r6ro_v.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('H $H reduce order bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
done
rm -f gpurun_out/r6ro_*.npz
grep bitwise $L
timeout -k 10 400 python -u -m pytest tests/test_ppo_gpu.py tests/test_dp_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r6ro_tests.log 2>&1 || { tail -30 gpurun_out/r6ro_tests.log; exit 1; }
tail -2 gpurun_out/r6ro_tests.log
TAG=r6ro H=64 VARIANTS="head" REPS=3 MBS=4096,512 bash tools/ab_spans.sh
