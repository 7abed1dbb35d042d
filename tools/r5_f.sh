#!/bin/bash
# round 5: split-ahead fc2 phases (product) vs without (tools/_probe/libsatrl_nosa.so):
# bitwise identity of whole updates + rollout passes, parity tests, in-graph step A/B
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_nosa.so
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r5f_sa.npz > gpurun_out/r5f_bits.log 2>&1 &&
SATRL_LIB_PATH=$V timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r5f_nosa.npz >> gpurun_out/r5f_bits.log 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r5f_sa.npz'), np.load('gpurun_out/r5f_nosa.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('bitwise differing arrays:', bad, 'of', len(a.files))
" >> gpurun_out/r5f_bits.log 2>&1
rm -f gpurun_out/r5f_*.npz
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_ppo_gpu.py -k "update_matches_reference or kx_rowpass or fused_step or logp_equals or short_rowpass or contiguous" \
    > gpurun_out/r5f_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5f_tests.log
for r in 1 2; do
  timeout -k 10 200 python -u tools/minibatch_time.py 4096 512 >> gpurun_out/r5f_step.log 2>&1 &&
  SATRL_LIB_PATH=$V timeout -k 10 200 python -u tools/minibatch_time.py 4096 512 | sed 's/$/ [nosa]/' >> gpurun_out/r5f_step.log 2>&1 || exit 1
done
