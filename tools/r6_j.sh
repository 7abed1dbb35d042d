#!/bin/bash
# GPU box (round 6, final profile pass): every counter pass and kernel trace of
# tools/profile_round.sh r6 (the bench under rocprofv3 reads them), then the
# rowpass issue / stall counters (tools/stall_pmc.sh).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
bash tools/profile_round.sh r6 > gpurun_out/r6j_profile.log 2>&1 || { echo "profile_round rc=$?"; exit 1; }
cd "$ROOT" && bash tools/stall_pmc.sh > gpurun_out/r6j_stall.json 2> gpurun_out/r6j_stall.err || exit 1
tail -c 400 gpurun_out/prof_r6/bench.json
