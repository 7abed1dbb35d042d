#!/bin/bash
# round 5: phase stamps of the H 256 rowpass with all / half / none of the
# split-bf16 MFMAs of phases B and D (timing-only probe builds)
set -o pipefail
OUT=gpurun_out/r5_o
mkdir -p $OUT
for v in probe phalf pnomf; do
  PROBE_H=256 PROBE_CHAIN=1 timeout -k 10 120 python3 tools/phase_probe.py probe:tools/_probe/libsatrl_$v.so > $OUT/chain_$v.txt 2>&1 || exit 1
done
