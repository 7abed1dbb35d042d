#!/bin/bash
# GPU box: PMC passes (each its own run) of the column-split short rowpass at
# configs[3]'s per-rank minibatch (tools/rowpass_workload.py 40 256 512):
# FETCH_SIZE, WRITE_SIZE, MFMA busy; summary -> gpurun_out/cs_pmc/r6_rowpass_cs_mb512_pmc.json
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$ROOT/gpurun_out/cs_pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
W="$ROOT/tools"
pmc() {
  local d=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  timeout -s KILL 120 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d "$OUT/$d" -o run -- python3 "$@" > /dev/null 2>&1
}
pmc fetch FETCH_SIZE -- "$W/rowpass_workload.py" 40 256 512 || exit 1
pmc write WRITE_SIZE -- "$W/rowpass_workload.py" 40 256 512 || exit 1
pmc mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- "$W/rowpass_workload.py" 40 256 512 || exit 1
cd "$ROOT" && python3 - <<'PY'
import glob, json, os, sys
sys.path.insert(0, "tools")
from summarize_profiles import pmc_per_dispatch
out = os.path.join("gpurun_out", "cs_pmc")
def f(d):
    return glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True)[0]
fk, nf = pmc_per_dispatch(f("fetch"), "rowpass_cs_kernel", "FETCH_SIZE")
wk, nw = pmc_per_dispatch(f("write"), "rowpass_cs_kernel", "WRITE_SIZE")
busy, nb = pmc_per_dispatch(f("mfma"), "rowpass_cs_kernel", "SQ_VALU_MFMA_BUSY_CYCLES")
grbm, ng = pmc_per_dispatch(f("mfma"), "rowpass_cs_kernel", "GRBM_GUI_ACTIVE")
res = {"kernel": "rowpass_cs_kernel (H 256, mb 512: 32 row blocks x 2 nets x 4 column quarters)",
       "workload": "tools/rowpass_workload.py 40 256 512", "dispatches": [nf, nw, nb],
       "FETCH_SIZE_kB_median": fk, "WRITE_SIZE_kB_median": wk,
       "hbm_bytes_per_launch": (2 * fk + wk) * 1024,
       "correction": "FETCH_SIZE x2 (gfx950 16-B/lane reads), WRITE_SIZE x1; kB = 1024 B",
       "mfma_busy_cycles_per_launch": busy, "grbm_gui_active_per_launch": grbm}
json.dump(res, open(os.path.join(out, "r6_rowpass_cs_mb512_pmc.json"), "w"), indent=1)
print(json.dumps(res))
PY
