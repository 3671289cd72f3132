#!/bin/bash
# PMC passes over the 8192^3 GEMM (wave / wait, MFMA busy, LDS counters), one rocprofv3 run per counter set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc$i -o pmc -- python tools/gemm_pmc.py 8192 > gpurun_out/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -30 gpurun_out/pmc$i.log; exit 1; }
done
for i in 1 2 3; do f=$(find gpurun_out/pmc$i -name "*counter_collection.csv" | head -1); echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(k, {c: round(v / max(1, cnt[(k, c)]), 1) for c, v in d.items()})
PY
done
