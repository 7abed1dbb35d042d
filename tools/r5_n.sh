#!/bin/bash
# round 5: H = 64's folded Adam steps (satrl_ppo_rowpass_dw2_adam).
# 1. the new bitwise test + the update tests; 2. whole updates + rollout
# passes at H 256 and H 64 against the last commit's tree (tools/_probe/headtree:
# its own Python host and library) bit for bit; 3. in-graph step, folded vs not
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_ppo_gpu.py -k "folded_adam or update_graph_groups or fused_dw2 or epoch_with_ragged or update_matches_reference or logp_equals" > gpurun_out/r5n_tests.log 2>&1 || exit 1
for H in 256 64; do
  timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r5n_new_$H.npz $H > gpurun_out/r5n_bits.log 2>&1 &&
  timeout -k 10 300 python -u tools/_probe/headtree/tools/bitwise_dump.py gpurun_out/r5n_head_$H.npz $H >> gpurun_out/r5n_bits.log 2>&1 || exit 1
done
python -c "
import numpy as np
for H in (256, 64):
    a, b = np.load(f'gpurun_out/r5n_new_{H}.npz'), np.load(f'gpurun_out/r5n_head_{H}.npz')
    bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
    print('H', H, 'bitwise differing arrays:', bad, 'of', len(a.files))
" >> gpurun_out/r5n_bits.log 2>&1 || exit 1
rm -f gpurun_out/r5n_*.npz
timeout -k 10 300 python -u tools/step_ab.py 64 4096 product,fold_adam=0 2 > gpurun_out/r5n_step.log 2>&1 &&
timeout -k 10 300 python -u tools/step_ab.py 64 512 product,fold_adam=0 2 >> gpurun_out/r5n_step.log 2>&1
