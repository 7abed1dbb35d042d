set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
: > gpurun_out/lb.log
timeout -k 10 400 python3 -u -m pytest tests/test_ppo_gpu.py -x -q --timeout 200 --timeout-method thread >> gpurun_out/lb.log 2>&1
for v in base eb0 lb0 lb0eb1 base; do
  echo "== $v" >> gpurun_out/lb.log
  if [ $v = base ]; then L=ppo-rl-satellite_amd/satrl/libsatrl.so; else L=tools/_probe/libsatrl_$v.so; fi
  timeout -k 10 120 python3 tools/rowpass_ab.py $L >> gpurun_out/lb.log 2>&1
  SATRL_LIB_PATH=$L timeout -k 10 120 python3 tools/minibatch_time.py 4096 512 >> gpurun_out/lb.log 2>&1
done
echo "== phase probe" >> gpurun_out/lb.log
timeout -k 10 120 python3 tools/phase_probe.py probe >> gpurun_out/lb.log 2>&1
grep -v amdgpu.ids gpurun_out/lb.log
