set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_ppo_gpu.py -x -v --timeout 200 --timeout-method thread -k dual > gpurun_out/dual_test.log 2>&1
SATRL_RP_DUAL=1 timeout -k 10 400 python3 -u -m pytest tests/test_ppo_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dual_ppo_tests.log 2>&1
timeout -k 10 300 python3 -u tools/rowpass_dual_ab.py > gpurun_out/dual_ab.log 2>&1
cat gpurun_out/dual_ab.log
