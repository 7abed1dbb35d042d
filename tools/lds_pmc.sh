set -euo pipefail
# GPU box: LDS counter pass (bank conflicts, LDS instructions and waits) on the rowpass workload;
# LIBP selects a library build, TAG the output directory suffix (gpurun_out/lds_pmc<TAG>)
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
D=$ROOT/gpurun_out/lds_pmc${TAG:-}; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
export SATRL_LIB_PATH=${LIBP:-$ROOT/ppo-rl-satellite_amd/satrl/libsatrl.so}
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $D -o run -- python3 $ROOT/tools/rowpass_workload.py 20 > $D/log.txt 2>&1
F=$(find $D -name '*counter_collection.csv')
python3 - "$F" <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'rowpass' in r['Kernel_Name']:
        v[r['Counter_Name']].append(float(r['Counter_Value']))
for k, x in v.items():
    x.sort(); print(k, len(x), x[len(x)//2])
PY
