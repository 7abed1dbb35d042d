#!/bin/bash
# Development: the two-rank one-device peer bench with and without the k-packed dW2
set -uo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for kx in 0 1; do
  echo "== SATRL_DW2_KX=$kx" >> gpurun_out/peerdiag.log
  SATRL_DW2_KX=$kx timeout -k 10 200 python3 bench.py --gpus 2 --one-device --num-envs 512 --horizon 32 --epochs 1 \
      --minibatch 4096 --steps 1 --warmup 1 --no-cpu-baseline --kernel-iters 10 --global-slice 8 --allreduce peer \
      > gpurun_out/peerdiag_$kx.out 2> gpurun_out/peerdiag_$kx.err
  rc=$?
  echo "rc=$rc" >> gpurun_out/peerdiag.log
  case $rc in 0|1|3) ;; *) exit $rc ;; esac
done
