#!/bin/bash
# development A/B of the product build against tools/_probe/libsatrl_head.so
# (the last commit's ppo_kernels.hip: make variant VNAME=head VSRC=...):
# bitwise identity of whole updates + rollout passes (when BITS=1), then the
# in-graph minibatch step at H 256 (mb 512, 4096) and the policy launch, twice
# usage: TAG=name BITS=1 [VNAME=head] bash tools/ab_head.sh  (VNAME: another tools/_probe/libsatrl_<VNAME>.so)
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_${VNAME:-head}.so
L=gpurun_out/${TAG}_ab.log
if [ "${BITS:-0}" = 1 ]; then
  timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/${TAG}_new.npz > $L 2>&1 &&
  SATRL_LIB_PATH=$V timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/${TAG}_head.npz >> $L 2>&1 &&
  python -c "
import numpy as np
a, b = np.load('gpurun_out/${TAG}_new.npz'), np.load('gpurun_out/${TAG}_head.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || exit 1
  rm -f gpurun_out/${TAG}_*.npz
fi
for r in 1 2; do
  timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 >> $L 2>&1 &&
  SATRL_LIB_PATH=$V timeout -k 10 120 python -u tools/minibatch_time.py 512 4096 | sed 's/$/ [head]/' >> $L 2>&1 &&
  timeout -k 10 120 python -u tools/policy_time.py >> $L 2>&1 &&
  SATRL_LIB_PATH=$V timeout -k 10 120 python -u tools/policy_time.py | sed 's/$/ [head]/' >> $L 2>&1 || exit 1
done
