#!/bin/bash
# development: the H 256 rowpass's issue / stall counters (two --pmc passes of
# tools/rowpass_workload.py, counters only), medians per dispatch
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
P3="SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  # shellcheck disable=SC2086
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/stall_p$i -o run -- python3 tools/rowpass_workload.py 20 > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, json, statistics
out = {}
for i in (1, 2, 3):
    f = glob.glob(f"gpurun_out/stall_p{i}/**/*counter_collection.csv", recursive=True)[0]
    vals = {}
    for row in csv.DictReader(open(f)):
        if "rowpass_kernel" not in row["Kernel_Name"]:
            continue
        vals.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
        vals[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    for k, v in vals.items():
        out.setdefault(k, statistics.median(v.values()))
print(json.dumps(out, indent=1, sort_keys=True))
PY
