#!/bin/bash
# Round-4 A/B of the update step: `build` here (variants of the product
# ppo_kernels.hip written by tools/ab_variants.py, compiled into
# tools/_probe/), `run` on the GPU box: the in-graph minibatch step
# (tools/minibatch_time.py) at H 256 mb 4096 / 512 and H 64 mb 4096 for the
# product library and every variant, the product first and last.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
case "${1:-}" in
  build)
    shift
    for v in $(python3 tools/ab_variants.py "$@"); do
      make -s -C ppo-rl-satellite_amd/csrc variant VNAME="$v" VSRC="../../tools/_probe/ab4/$v.hip"
    done
    ;;
  run)
    shift
    mkdir -p gpurun_out
    LOG=gpurun_out/ab_round4.log
    : > "$LOG"
    # a variant NAME is tools/_probe/libsatrl_NAME.so; env:VAR=VAL runs the
    # product library with that environment setting
    for v in base "$@" base; do
      E=()
      if [ "$v" = base ]; then L=ppo-rl-satellite_amd/satrl/libsatrl.so
      elif [ "${v#env:}" != "$v" ]; then L=ppo-rl-satellite_amd/satrl/libsatrl.so; E=("${v#env:}")
      else L=tools/_probe/libsatrl_$v.so; fi
      echo "== $v" >> "$LOG"
      env "${E[@]}" SATRL_LIB_PATH=$L PROBE_H=256 timeout -k 10 120 python3 tools/minibatch_time.py 4096 512 >> "$LOG" 2>&1
      if [ "${AB_H64:-1}" = "1" ]; then
        env "${E[@]}" SATRL_LIB_PATH=$L PROBE_H=64 timeout -k 10 120 python3 tools/minibatch_time.py 4096 >> "$LOG" 2>&1
      fi
      if [ "${AB_POLICY:-0}" = "1" ]; then
        env "${E[@]}" SATRL_LIB_PATH=$L timeout -k 10 120 python3 tools/policy_time.py >> "$LOG" 2>&1
      fi
    done
    grep -v amdgpu.ids "$LOG"
    ;;
  *)
    echo "usage: $0 build [variants] | run variants..." >&2
    exit 2
    ;;
esac
