set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for v in prio tok tokprio; do
  echo "== $v" >> gpurun_out/dual2.log
  SATRL_RP_DUAL=1 timeout -k 10 120 python3 tools/rowpass_ab.py tools/_probe/libsatrl_$v.so >> gpurun_out/dual2.log 2>&1
  SATRL_RP_DUAL=1 SATRL_LIB_PATH=tools/_probe/libsatrl_$v.so timeout -k 10 120 python3 tools/minibatch_time.py 4096 >> gpurun_out/dual2.log 2>&1
done
cat gpurun_out/dual2.log
