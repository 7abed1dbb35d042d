#!/bin/bash
# Run on the GPU box (gpurun): the FETCH_SIZE and WRITE_SIZE passes (separate
# runs, no tracing domains beside --pmc) on the rowpass workload, then
# bench.py under rocprofv3 kernel stats (it reads the traffic figure the PMC
# passes just wrote into profiles/).  Scratch goes to gpurun_out/prof_<tag>;
# the summaries land in gpurun_out/prof_<tag>/profiles (copied into the
# committed profiles/ afterwards).
set -euo pipefail
TAG=${1:-r1}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$ROOT/tools/rowpass_workload.py" 40 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 "$ROOT/tools/rowpass_workload.py" 40 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_env_fetch" -o run -- \
    python3 "$ROOT/tools/env_workload.py" 40 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_env_write" -o run -- \
    python3 "$ROOT/tools/env_workload.py" 40 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d "$OUT/pmc_mfma" -o run -- python3 "$ROOT/tools/rowpass_workload.py" 40 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d "$OUT/pmc_policy_mfma" -o run -- python3 "$ROOT/tools/policy_workload.py" 40 > /dev/null 2>&1
python3 "$ROOT/tools/summarize_profiles.py" "$OUT" "$TAG" "$ROOT/profiles"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o run -- \
    python3 "$ROOT/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"
rm -f "$OUT/bench/run_kernel_trace.csv"
python3 "$ROOT/tools/summarize_profiles.py" "$OUT" "$TAG" "$OUT/profiles"
cp "$ROOT/profiles/${TAG}_rowpass_pmc.json" "$ROOT/profiles/${TAG}_env_pmc.json" "$ROOT/profiles/${TAG}_rowpass_mfma_pmc.json" \
    "$ROOT/profiles/${TAG}_policy_mfma_pmc.json" \
    "$OUT/profiles/" 2>/dev/null || true
cp "$OUT/profiles/${TAG}_bench_kernel_stats.csv" "$ROOT/profiles/"
tail -1 "$OUT/bench.json"
