#!/bin/bash
# round 5: per-wave phase stamps of the product rowpass (probe build), H 256 and H 64,
# back to back and as the last rowpass of graph-replayed steps
set -o pipefail
OUT=gpurun_out/r5_probe
mkdir -p $OUT
for H in 256 64; do
  PROBE_H=$H timeout -k 10 120 python3 tools/phase_probe.py probe > $OUT/phase_h$H.txt 2>&1 &&
  PROBE_H=$H PROBE_CHAIN=1 timeout -k 10 120 python3 tools/phase_probe.py probe > $OUT/phase_chain_h$H.txt 2>&1 || exit 1
done
