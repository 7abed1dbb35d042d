#!/bin/bash
# GPU box (round 6, pass F): write-through hand-off A/B (H 256 mb 4096 / 512;
# H 64: the fused dW2 slabs), then the env kernel's solve queue (r6_e.sh).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
bash tools/r6_e.sh || exit 1
TAG=r6f VARIANTS="kxwth1 dwwt h1dw kxwt" REPS=2 bash tools/ab_spans.sh || exit 1
TAG=r6f64 H=64 MBS=4096 VARIANTS="fwt" REPS=3 bash tools/ab_spans.sh || exit 1
