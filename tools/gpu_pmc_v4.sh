#!/bin/bash
# Kernel-trace stats and counters of the bf16 GEMMs at 8192^3: v3, v4 (both bf16 C + fused column sums) and
# hipBLASLt, same operands (tools/gemm_v4_pmc.py).  One counter set per rocprofv3 run; summary in
# gpurun_out/v4pmc_summary.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v4stats -o st -- python3 tools/gemm_v4_pmc.py 8192 > gpurun_out/v4stats.log 2>&1 || { echo "stats failed"; tail -30 gpurun_out/v4stats.log; exit 1; }
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/v4pmc$i -o pmc -- python3 tools/gemm_v4_pmc.py 8192 > gpurun_out/v4pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -30 gpurun_out/v4pmc$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
out = {"counters": {}, "kernel_stats": []}
for d in sorted(glob.glob("gpurun_out/v4pmc*/")):
    fs = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        agg[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, dd in agg.items():
        for c, v in dd.items():
            out["counters"].setdefault(k, {})[c] = round(sorted(v)[len(v) // 2], 1)
for f in glob.glob("gpurun_out/v4stats/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        out["kernel_stats"].append({k: r[k] for k in r if k in ("Name", "Calls", "TotalDurationNs", "AverageNs",
                                                                "Percentage", "MinNs", "MaxNs")})
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/v4pmc_summary.json", "w"), indent=1)
PY
