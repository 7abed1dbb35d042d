set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
: > gpurun_out/fakeb.log
for d in 0 1; do
  echo "== fakeb dual=$d" >> gpurun_out/fakeb.log
  SATRL_RP_DUAL=$d timeout -k 10 120 python3 tools/rowpass_ab.py tools/_probe/libsatrl_fakeb.so >> gpurun_out/fakeb.log 2>&1
  SATRL_RP_DUAL=$d SATRL_LIB_PATH=tools/_probe/libsatrl_fakeb.so timeout -k 10 120 python3 tools/minibatch_time.py 4096 >> gpurun_out/fakeb.log 2>&1
done
echo "== base" >> gpurun_out/fakeb.log
timeout -k 10 120 python3 tools/rowpass_ab.py >> gpurun_out/fakeb.log 2>&1
grep -v amdgpu.ids gpurun_out/fakeb.log
