set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
: > gpurun_out/ff.log
for v in base ff3 ff3g; do
  if [ $v = base ]; then L=ppo-rl-satellite_amd/satrl/libsatrl.so; else L=tools/_probe/libsatrl_$v.so; fi
  timeout -k 10 120 python3 tools/rowpass_ab.py $L >> gpurun_out/ff.log 2>&1
done
for v in probe pff3 pff3g; do
  echo "== phase probe $v" >> gpurun_out/ff.log
  timeout -k 10 120 python3 tools/phase_probe.py probe:tools/_probe/libsatrl_$v.so >> gpurun_out/ff.log 2>&1
done
grep -v amdgpu.ids gpurun_out/ff.log
