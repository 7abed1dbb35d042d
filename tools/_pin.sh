set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/dw2_pin.py gpurun_out/dw2_plans.json > gpurun_out/dw2_pin.log 2>&1
grep -v amdgpu.ids gpurun_out/dw2_pin.log | cut -c1-200
