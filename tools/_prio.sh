set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
: > gpurun_out/prio.log
for v in base prio1 prio2 prio3 base prio3; do
  if [ $v = base ]; then L=ppo-rl-satellite_amd/satrl/libsatrl.so; else L=tools/_probe/libsatrl_$v.so; fi
  timeout -k 10 120 python3 tools/rowpass_ab.py $L >> gpurun_out/prio.log 2>&1
  SATRL_LIB_PATH=$L timeout -k 10 120 python3 tools/minibatch_time.py 4096 512 >> gpurun_out/prio.log 2>&1
done
echo "== phase probe pprio3" >> gpurun_out/prio.log
timeout -k 10 120 python3 tools/phase_probe.py probe:tools/_probe/libsatrl_pprio3.so >> gpurun_out/prio.log 2>&1
grep -v amdgpu.ids gpurun_out/prio.log
