#!/bin/bash
# GPU box (round 6, pass B): Step-1 rowpass change (split-once plane stores)
# bitwise vs the committed build (tools/_probe/libsatrl_head.so), in-graph
# step + live kernel spans A/B (alternating), the launch-floor microbenchmark.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
V=$ROOT/tools/_probe/libsatrl_head.so
L=gpurun_out/r6b_ab.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6b_new.npz > $L 2>&1 &&
SATRL_LIB_PATH=$V timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6b_head.npz >> $L 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r6b_new.npz'), np.load('gpurun_out/r6b_head.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || exit 1
rm -f gpurun_out/r6b_*.npz
for r in 1 2; do
  timeout -k 10 200 python -u tools/span_time.py 256 4096,512 >> $L 2>&1 &&
  SATRL_LIB_PATH=$V timeout -k 10 200 python -u tools/span_time.py 256 4096,512 >> $L 2>&1 || exit 1
done
timeout -k 10 120 ./tools/_probe/launch_floor > gpurun_out/r6b_launch_floor.json 2> gpurun_out/r6b_launch_floor.err || exit 1
timeout -k 10 200 python -u tools/span_time.py 64 4096 1 rollout >> $L 2>&1
cat $L
