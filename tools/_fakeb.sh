set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
: > gpurun_out/fakeb.log
echo "== base" >> gpurun_out/fakeb.log
timeout -k 10 120 python3 tools/rowpass_ab.py >> gpurun_out/fakeb.log 2>&1
for v in fakeb fakega fakeboth csync1 csync2; do
  echo "== $v" >> gpurun_out/fakeb.log
  timeout -k 10 120 python3 tools/rowpass_ab.py tools/_probe/libsatrl_$v.so >> gpurun_out/fakeb.log 2>&1
done
echo "== fakeb dual" >> gpurun_out/fakeb.log
SATRL_RP_DUAL=1 timeout -k 10 120 python3 tools/rowpass_ab.py tools/_probe/libsatrl_fakeb.so >> gpurun_out/fakeb.log 2>&1
echo "== phase probe" >> gpurun_out/fakeb.log
timeout -k 10 120 python3 tools/phase_probe.py probe >> gpurun_out/fakeb.log 2>&1
grep -v amdgpu.ids gpurun_out/fakeb.log
echo "== env acos A/B" >> gpurun_out/fakeb.log
timeout -k 10 200 python3 -u -m pytest tests/test_env_gpu.py -x -q --timeout 150 --timeout-method thread -k "acos or sincos or trajectory or danger" >> gpurun_out/fakeb.log 2>&1
echo "-- straight-line acos" >> gpurun_out/fakeb.log
timeout -k 10 120 python3 tools/env_sweep.py >> gpurun_out/fakeb.log 2>&1
echo "-- library acos" >> gpurun_out/fakeb.log
SATRL_LIB_PATH=tools/_probe/libsatrl_acoslib.so timeout -k 10 120 python3 tools/env_sweep.py >> gpurun_out/fakeb.log 2>&1
echo "-- straight-line acos again" >> gpurun_out/fakeb.log
timeout -k 10 120 python3 tools/env_sweep.py >> gpurun_out/fakeb.log 2>&1
grep -v amdgpu.ids gpurun_out/fakeb.log | tail -25
