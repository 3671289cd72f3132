#!/bin/bash
# PMC counters for the GEMM lab kernels at one size (each counter set in its own rocprofv3 pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SIZE=${1:-8192}
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/labpmc$i -o pmc -- ./tools/gemm_lab.bin $SIZE 5 > gpurun_out/labpmc$i.log 2>&1 || { echo "pmc $i failed"; tail -30 gpurun_out/labpmc$i.log; exit 1; }
done
for i in 1 2 3; do f=$(find gpurun_out/labpmc$i -name "*counter_collection.csv" | head -1); echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"][:48]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
for k, d in agg.items():
    n = max(1, len(disp[k]))
    print(k, {c: round(v / n, 1) for c, v in d.items()})
PY
done
