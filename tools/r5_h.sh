#!/bin/bash
# round 5: fc2 B-operand split with v_dot2c_f32_bf16 residuals (product) vs the
# widen + packed-subtract split (tools/_probe/libsatrl_head.so): bitwise identity
# of whole updates + rollout passes, then in-graph step A/B at H 256 and H 64
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_head.so
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r5h_new.npz > gpurun_out/r5h_bits.log 2>&1 &&
SATRL_LIB_PATH=$V timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r5h_head.npz >> gpurun_out/r5h_bits.log 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r5h_new.npz'), np.load('gpurun_out/r5h_head.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('bitwise differing arrays:', bad, 'of', len(a.files))
" >> gpurun_out/r5h_bits.log 2>&1 || exit 1
rm -f gpurun_out/r5h_*.npz
for r in 1 2; do
  timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 >> gpurun_out/r5h_time.log 2>&1 &&
  SATRL_LIB_PATH=$V timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 | sed 's/$/ [head]/' >> gpurun_out/r5h_time.log 2>&1 &&
  PROBE_H=64 timeout -k 10 120 python -u tools/minibatch_time.py 4096 | sed 's/$/ [h64]/' >> gpurun_out/r5h_time.log 2>&1 &&
  PROBE_H=64 SATRL_LIB_PATH=$V timeout -k 10 120 python -u tools/minibatch_time.py 4096 | sed 's/$/ [h64 head]/' >> gpurun_out/r5h_time.log 2>&1 || exit 1
done
