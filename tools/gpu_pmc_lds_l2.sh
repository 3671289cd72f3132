#!/bin/bash
# Counter passes over the LDS test and the per-XCD L2 read (one rocprofv3 run per counter set, kernel
# trace only alongside).  Summaries: gpurun_out/pmc_lds_l2/summary.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_lds_l2
i=0
for set in "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc_lds_l2/p$i -o pmc \
    -- python tools/lds_l2_pmc.py > gpurun_out/pmc_lds_l2/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -20 gpurun_out/pmc_lds_l2/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, collections, glob, json
out = {}
for f in sorted(glob.glob("gpurun_out/pmc_lds_l2/p*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if k.startswith(("lds_test", "l2_read")):
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        for c, v in d.items():
            out.setdefault(k, {})[c] = {"per_dispatch_mean": round(sum(v) / len(v), 1), "dispatches": len(v)}
json.dump(out, open("gpurun_out/pmc_lds_l2/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
