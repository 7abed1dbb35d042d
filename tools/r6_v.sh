#!/bin/bash
# GPU box (round 6, pass V): timing-only variant (tools/_probe/libsatrl_pf.so):
# adam_kernel loads the next minibatch's staged rows into the L2 of the XCD
# whose rowpass blocks read them (tools/l2_persist.hip: an L2 line a kernel
# loaded hits in the next kernel on that XCD, 89 against 222-353 ns).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
TAG=r6v VARIANTS="pf" REPS=4 MBS=4096 bash tools/ab_spans.sh || exit 1
TAG=r6v64 H=64 VARIANTS="pf" REPS=4 MBS=4096 bash tools/ab_spans.sh
