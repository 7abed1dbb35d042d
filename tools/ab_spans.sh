#!/bin/bash
# development A/B (GPU box): the product build against tools/_probe/libsatrl_<V>.so
# for each V in VARIANTS, alternating REPS times: in-graph minibatch step and the
# live kernel spans (tools/span_time.py) at H $H, minibatch sizes $MBS.
# usage: TAG=name VARIANTS="kxwt other" [H=256] [MBS=4096,512] [REPS=3] bash tools/ab_spans.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd "$ROOT"
mkdir -p gpurun_out
L=gpurun_out/${TAG}_ab.log
for r in $(seq 1 ${REPS:-3}); do
  timeout -k 10 200 python -u tools/span_time.py ${H:-256} ${MBS:-4096,512} >> $L 2>&1 || exit 1
  for v in $VARIANTS; do
    SATRL_LIB_PATH=$ROOT/tools/_probe/libsatrl_$v.so timeout -k 10 200 python -u tools/span_time.py ${H:-256} ${MBS:-4096,512} >> $L 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $L
