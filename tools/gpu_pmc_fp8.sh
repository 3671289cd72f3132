#!/bin/bash
# Counters of the fp8 v3 GEMM, scaled vs unscaled MFMA form, and hipBLASLt's fp8 GEMM on the same operands
# (tools/gemm_fp8_pmc.py), 8192^3, bf16 C: one rocprofv3 pass per counter group (never more than the blocks
# hold: 8 SQ, FETCH_SIZE alone for TCC, 2 GRBM), each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
n=${1:-8192}
i=0
for set in "GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/fp8pmc$i -o pmc -- python3 tools/gemm_fp8_pmc.py $n > gpurun_out/fp8pmc$i.log 2>&1 || { echo "pmc pass $i ($set) failed"; tail -30 gpurun_out/fp8pmc$i.log; exit 1; }
done
python3 - "$n" <<'PY'
import csv, glob, collections, json, sys
n = sys.argv[1]
out = {}
for d in sorted(glob.glob("gpurun_out/fp8pmc*/")):
    fs = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    rows = list(csv.DictReader(open(fs[0])))
    # gemm_v3_kernel<1, ...> is the scaled form (DT_FP8), <3, ...> the unscaled one (DT_FP8U)
    label = {}
    for r in rows:
        k = r["Kernel_Name"]
        if "gemm_v3_kernel<1," in k:
            label[k] = "v3 fp8 scaled"
        elif "gemm_v3_kernel<3," in k:
            label[k] = "v3 fp8 unscaled"
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        name = r["Kernel_Name"]
        if name not in label and "Cijk" not in name:
            continue  # operand generation and casts
        agg[label.get(name, "hipblaslt " + name[:60])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, dd in agg.items():
        for c, v in dd.items():
            out.setdefault(f"{k} {n}^3", {})[c] = round(sorted(v)[len(v) // 2], 1)
for k, c in out.items():
    if c.get("SQ_WAVE_CYCLES"):
        c["_derived"] = {"wait_any_frac": round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 3),
                         "active_inst_frac": round(c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"], 3)}
    if c.get("SQ_BUSY_CYCLES") and c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        c.setdefault("_derived", {})["mfma_busy_per_busy_cycle"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["SQ_BUSY_CYCLES"], 3)
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/fp8pmc_summary.json", "w"), indent=1)
PY
