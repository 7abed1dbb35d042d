#!/bin/bash
# Run on the GPU box (gpurun): every counter pass in a run of its own (no
# tracing domains beside --pmc), the env kernel's in-rollout and per-size
# kernel traces, then bench.py under rocprofv3 kernel stats (it reads the
# PMC summaries just written into profiles/).  Scratch goes to
# gpurun_out/prof_<tag>; the summaries land in gpurun_out/prof_<tag>/profiles
# (copied into the committed profiles/ afterwards).
set -euo pipefail
TAG=${1:-r3}
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
W="$ROOT/tools"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
pmc() {   # pmc <dir> <counters...> -- <workload args>
  local d=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  timeout -s KILL 180 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d "$OUT/$d" -o run -- python3 "$@" > /dev/null 2>&1
}
pmc pmc_fetch FETCH_SIZE -- "$W/rowpass_workload.py" 40
pmc pmc_write WRITE_SIZE -- "$W/rowpass_workload.py" 40
pmc pmc_env_fetch FETCH_SIZE -- "$W/env_workload.py" 40
pmc pmc_env_write WRITE_SIZE -- "$W/env_workload.py" 40
pmc pmc_mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- "$W/rowpass_workload.py" 40
pmc pmc_policy_mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- "$W/policy_workload.py" 40
# BASELINE configs[1] (H 64, 4096 envs): its rowpass (dW2 fused) and policy kernel
pmc pmc_fetch_h64 FETCH_SIZE -- "$W/rowpass_workload.py" 40 64 4096
pmc pmc_write_h64 WRITE_SIZE -- "$W/rowpass_workload.py" 40 64 4096
pmc pmc_mfma_h64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- "$W/rowpass_workload.py" 40 64 4096
pmc pmc_policy_mfma_h64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- "$W/policy_workload.py" 40 64 4096
# the post-rowpass chain (dw2_kx, reduce, Adam) of eager minibatch steps
pmc pmc_step_fetch FETCH_SIZE -- "$W/step_workload.py" 40
pmc pmc_step_write WRITE_SIZE -- "$W/step_workload.py" 40
pmc pmc_step_mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- "$W/step_workload.py" 40
# FP64 VALU work of the env step: the F64 instruction counters this rocprofv3 lists (<= 7 SQ + GRBM)
F64=$(grep -o 'SQ_INSTS_VALU_[A-Z0-9_]*F64' "$OUT/avail.txt" | sort -u | head -7 | tr '\n' ' ')
if [ -n "$F64" ]; then
  # shellcheck disable=SC2086
  pmc pmc_env_fp64 $F64 GRBM_GUI_ACTIVE -- "$W/env_workload.py" 40
fi
# env kernel durations: the training rollout alone, and mid-episode per env count
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/env_rollout" -o run -- \
    python3 "$W/env_workload.py" rollout 1 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/env_sweep" -o run -- \
    python3 "$W/env_workload.py" sweep 200 > /dev/null 2>&1
python3 "$W/summarize_profiles.py" "$OUT" "$TAG" "$ROOT/profiles"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o run -- \
    python3 "$ROOT/bench.py" --profile-tag "$TAG" > "$OUT/bench.json" 2> "$OUT/bench.err"
# BASELINE configs[1] (4096 envs, H 64): its own kernel stats for its roofline line
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench_configs1" -o run -- \
    python3 "$ROOT/bench.py" --num-envs 4096 --hidden 64 --no-cpu-baseline --profile-tag "$TAG" \
    > "$OUT/bench_configs1.json" 2> "$OUT/bench_configs1.err"
rm -f "$OUT/bench/run_kernel_trace.csv" "$OUT/bench_configs1/run_kernel_trace.csv" "$OUT/env_rollout/run_kernel_trace.csv"
# the committed summaries first, then this run's (the fresh bench stats must win)
mkdir -p "$OUT/profiles"
cp "$ROOT"/profiles/"${TAG}"_*.json "$OUT/profiles/" 2>/dev/null || true
cp "$ROOT"/profiles/"${TAG}"_*.csv "$OUT/profiles/" 2>/dev/null || true
python3 "$W/summarize_profiles.py" "$OUT" "$TAG" "$OUT/profiles"
cp "$OUT/profiles/${TAG}_bench_kernel_stats.csv" "$ROOT/profiles/"
cp "$OUT/profiles/${TAG}_bench_configs1_kernel_stats.csv" "$ROOT/profiles/" 2>/dev/null || true
tail -1 "$OUT/bench.json"
