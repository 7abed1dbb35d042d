#!/bin/bash
# Round-3 A/B measurements of the rowpass / update chain, in
# two halves: `build` here (hipcc cross-compiles the dev variants into
# tools/_probe/, they travel with the tree), `run` on the GPU box (gpurun).
# Every variant is a dev build of round 3's ppo_kernels.hip (git ca3c6c3, where
# the timing-only knobs below still live; the product source dropped them in
# round 4) with extra defines; none is the product.  Timing tools: rowpass_ab.py (rowpass alone, back to back),
# minibatch_time.py (in-graph step), phase_probe.py (per-wave stamps).
#
#   bash tools/ab_round3.sh build
#   gpurun --timeout 900 -- 'bash tools/ab_round3.sh run'
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
# name:defines
VARIANTS=(
  "fakeb:-DSATRL_RP_FAKE_LDS_B"                       # B operand from LDS (feed from on-chip)
  "fakega:-DSATRL_RP_FAKE_GATHER"                     # no row gather / W1 loads
  "fakeboth:-DSATRL_RP_FAKE_LDS_B -DSATRL_RP_FAKE_GATHER"
  "csync1:-DSATRL_RP_CHUNK_SYNC=1"                    # waves meet every chunk
  "csync2:-DSATRL_RP_CHUNK_SYNC=2"
  "ff3:-DSATRL_RP_FAKE_FEED=3"                        # no operand loads at all in B / D
  "lb1:-DSATRL_RP_LDSBAR=1"                           # LDS-only phase barriers
  "wt1:-DSATRL_WT=1"                                  # write-through H1 / dZ2
  "wt15:-DSATRL_WT=15"                                # ... and slabs, G, P/M/V/W2T
  "prio3:-DSATRL_RP_PRIO=3"                           # s_setprio in phases B and D
)
case "${1:-}" in
  build)
    mkdir -p tools/_probe/r3
    git show ca3c6c3:ppo-rl-satellite_amd/csrc/ppo_kernels.hip > tools/_probe/r3/ppo_kernels.hip
    for v in "${VARIANTS[@]}"; do
      make -s -C ppo-rl-satellite_amd/csrc variant VNAME="${v%%:*}" VSRC=../../tools/_probe/r3/ppo_kernels.hip \
          VDEFS="${v#*:}"
    done
    make -s -C ppo-rl-satellite_amd/csrc probe
    ;;
  run)
    mkdir -p gpurun_out
    LOG=gpurun_out/ab_round3.log
    : > "$LOG"
    for v in base "${VARIANTS[@]%%:*}" base; do
      if [ "$v" = base ]; then L=ppo-rl-satellite_amd/satrl/libsatrl.so; else L=tools/_probe/libsatrl_$v.so; fi
      echo "== $v" >> "$LOG"
      timeout -k 10 120 python3 tools/rowpass_ab.py "$L" >> "$LOG" 2>&1
      SATRL_LIB_PATH=$L timeout -k 10 120 python3 tools/minibatch_time.py 4096 512 >> "$LOG" 2>&1
    done
    echo "== two streams: rowpass beside dW2" >> "$LOG"
    timeout -k 10 200 python3 tools/overlap_probe.py >> "$LOG" 2>&1
    echo "== per-net chains out of phase" >> "$LOG"
    timeout -k 10 300 python3 tools/split_offset.py 4096 64 >> "$LOG" 2>&1
    echo "== phase probe" >> "$LOG"
    timeout -k 10 120 python3 tools/phase_probe.py probe >> "$LOG" 2>&1
    grep -v amdgpu.ids "$LOG"
    ;;
  *)
    echo "usage: $0 build|run" >&2
    exit 2
    ;;
esac
