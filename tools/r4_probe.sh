#!/bin/bash
# GPU box (round 4): where the minibatch step's time goes at H 64 and H 256.
#   1. per-wave phase stamps of the rowpass (probe build) + eager launch timings
#   2. the kernel timeline of graph-replayed steps under rocprofv3 --kernel-trace
# Every step has its own time limit; the first failure ends the script.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r4_probe
mkdir -p "$OUT"
for H in ${PROBE_HS:-64 256}; do
  PROBE_H=$H timeout -k 10 120 python3 tools/phase_probe.py probe > "$OUT/phase_h$H.txt" 2>&1
  PROBE_H=$H PROBE_CHAIN=1 timeout -k 10 120 python3 tools/phase_probe.py probe > "$OUT/phase_chain_h$H.txt" 2>&1
  ( cd /tmp && export TMPDIR=/tmp && PROBE_H=$H REPS=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv \
      -d "$OUT/tl_h$H" -o run -- python3 "$ROOT/tools/step_timeline.py" run > "$OUT/tl_h$H.log" 2>&1 )
  CSV=$(find "$OUT/tl_h$H" -name '*kernel_trace.csv')
  python3 tools/step_timeline.py parse $CSV > "$OUT/timeline_h$H.txt" 2>&1
  find "$OUT/tl_h$H" -name '*kernel_trace.csv' -delete
done
tail -n 30 "$OUT"/timeline_h*.txt
