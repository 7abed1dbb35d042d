#!/bin/bash
# development: LDS bank-conflict cycles of the H 256 rowpass, product vs
# tools/_probe/libsatrl_head.so (one --pmc pass each, counters only)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in product head; do
  if [ $b = head ]; then export SATRL_LIB_PATH=$GRAFT_REPO_ROOT/tools/_probe/libsatrl_head.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv \
      -d gpurun_out/ldsc_$b -o run -- python3 tools/rowpass_workload.py 20 > /dev/null 2>&1 || exit 1
done
unset SATRL_LIB_PATH
python3 - <<'PY'
import csv, glob, statistics
for b in ("product", "head"):
    f = glob.glob(f"gpurun_out/ldsc_{b}/**/*counter_collection.csv", recursive=True)[0]
    vals = {}
    for row in csv.DictReader(open(f)):
        if "rowpass_kernel" not in row["Kernel_Name"]: continue
        vals.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
        vals[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    print(b, {k: statistics.median(v.values()) for k, v in vals.items()})
PY
