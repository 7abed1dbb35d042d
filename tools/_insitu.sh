set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/minibatch_time.py 4096 512 > gpurun_out/insitu.log 2>&1
timeout -k 10 700 python3 -u tools/dw2_insitu.py 4096 512 --top 10 >> gpurun_out/insitu.log 2>&1
grep -v amdgpu.ids gpurun_out/insitu.log
