#!/bin/bash
# GPU box: kernel timeline of graph-replayed H 64 steps, deferred Adam on / off
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r4_fadam_tl
mkdir -p "$OUT"
for FA in 1 0; do
  ( cd /tmp && export TMPDIR=/tmp && SATRL_FUSED_ADAM=$FA PROBE_H=64 REPS=10 timeout -k 10 180 rocprofv3 --kernel-trace \
      --output-format csv -d "$OUT/tl_fa$FA" -o run -- python3 "$ROOT/tools/step_timeline.py" run > "$OUT/tl_fa$FA.log" 2>&1 )
  CSV=$(find "$OUT/tl_fa$FA" -name '*kernel_trace.csv')
  python3 tools/step_timeline.py parse $CSV > "$OUT/timeline_fa$FA.txt" 2>&1
  find "$OUT/tl_fa$FA" -name '*kernel_trace.csv' -delete
done
cat "$OUT"/timeline_fa*.txt
