#!/bin/bash
# GPU box (round 4): kernel durations of graph-replayed minibatch steps
# (tools/minibatch_time.py, H 256 mb 4096 and H 64) under rocprofv3 kernel
# stats, for the product library and the environment settings in KP (e.g.
# "SATRL_DW2_KX=0").  One step per profile, each under its own limit.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/kprof
mkdir -p "$OUT"
i=0
for e in base ${KP:-}; do
  E=(); [ "$e" != base ] && E=("$e")
  env "${E[@]}" PROBE_H=256 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/h256_$i" -o run -- \
      python3 "$ROOT/tools/minibatch_time.py" 4096 > "$OUT/h256_$i.log" 2>&1
  rm -f "$OUT"/h256_$i/run_kernel_trace.csv
  i=$((i+1))
done
PROBE_H=64 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/h64" -o run -- \
    python3 "$ROOT/tools/minibatch_time.py" 4096 > "$OUT/h64.log" 2>&1
rm -f "$OUT"/h64/run_kernel_trace.csv
echo done
