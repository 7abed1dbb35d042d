set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
: > gpurun_out/wt.log
for v in base wt1 wt3 wt15 base wt1 wt3 wt15; do
  echo "== $v" >> gpurun_out/wt.log
  if [ $v = base ]; then L=ppo-rl-satellite_amd/satrl/libsatrl.so; else L=tools/_probe/libsatrl_$v.so; fi
  SATRL_LIB_PATH=$L timeout -k 10 120 python3 tools/minibatch_time.py 4096 512 >> gpurun_out/wt.log 2>&1
done
SATRL_LIB_PATH=tools/_probe/libsatrl_wt15.so timeout -k 10 400 python3 -u -m pytest tests/test_ppo_gpu.py -x -q --timeout 200 --timeout-method thread >> gpurun_out/wt.log 2>&1
grep -v amdgpu.ids gpurun_out/wt.log
