#!/bin/bash
# Kernel-trace stats and counters of the GEMMs at 8192^3: v3, v4 (both bf16 C + fused column sums) and
# hipBLASLt, same operands (tools/gemm_v4_pmc.py).  One counter set per rocprofv3 run; summary in
# gpurun_out/v4pmc_summary.json (gpurun_out/v4pmc_fp8_summary.json with DTYPE=fp8 for E4M3 operands).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DTYPE=${DTYPE:-bf16}
T=v4${DTYPE/bf16/}
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}stats -o st -- python3 tools/gemm_v4_pmc.py 8192 "$DTYPE" > gpurun_out/${T}stats.log 2>&1 || { echo "stats failed"; tail -30 gpurun_out/${T}stats.log; exit 1; }
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/${T}pmc$i -o pmc -- python3 tools/gemm_v4_pmc.py 8192 "$DTYPE" > gpurun_out/${T}pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -30 gpurun_out/${T}pmc$i.log; exit 1; }
done
T=$T python3 - <<'PY'
import csv, glob, collections, json, os
t = os.environ["T"]
out = {"counters": {}, "kernel_stats": []}
for d in sorted(glob.glob(f"gpurun_out/{t}pmc[0-9]*/")):
    fs = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        agg[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, dd in agg.items():
        for c, v in dd.items():
            out["counters"].setdefault(k, {})[c] = round(sorted(v)[len(v) // 2], 1)
for f in glob.glob(f"gpurun_out/{t}stats/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        out["kernel_stats"].append({k: r[k] for k in r if k in ("Name", "Calls", "TotalDurationNs", "AverageNs",
                                                                "Percentage", "MinNs", "MaxNs")})
print(json.dumps(out, indent=1))
json.dump(out, open(f"gpurun_out/{t}pmc_summary.json" if t == "v4" else "gpurun_out/v4pmc_fp8_summary.json", "w"), indent=1)
PY
