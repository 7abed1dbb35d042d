#!/bin/bash
# GPU box (round 6, pass M): column-split rowpass with the head reading X1 and
# phase D reading the other quarters' dZ2 planes straight from X2: bitwise
# against the pre-split build, in-graph A/B against the first split build
# (cs1), its phase stamps; the dot2 special-value probe.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
V=$ROOT/tools/_probe/libsatrl_precs.so
L=gpurun_out/r6m_bitwise.log
timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6m_new.npz 256 > $L 2>&1 &&
SATRL_LIB_PATH=$V timeout -k 10 300 python -u tools/bitwise_dump.py gpurun_out/r6m_old.npz 256 >> $L 2>&1 &&
python -c "
import numpy as np
a, b = np.load('gpurun_out/r6m_new.npz'), np.load('gpurun_out/r6m_old.npz')
bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
print('H 256 bitwise differing arrays:', bad, 'of', len(a.files))
" >> $L 2>&1 || { tail -30 $L; exit 1; }
rm -f gpurun_out/r6m_*.npz
grep bitwise $L
timeout -k 10 60 ./tools/_probe/dot2_exact > gpurun_out/r6m_dot2.txt 2>&1 || exit 1
cat gpurun_out/r6m_dot2.txt
TAG=r6m VARIANTS="cs1" REPS=3 MBS=512 bash tools/ab_spans.sh || exit 1
PROBE_MB=512 PROBE_CHAIN=1 timeout -k 10 200 python -u tools/phase_probe.py probe > gpurun_out/r6m_phase_cs.txt 2>&1
grep -A16 "actor quarter 3" gpurun_out/r6m_phase_cs.txt; tail -8 gpurun_out/r6m_phase_cs.txt
