#!/bin/bash
# Write / fetch / MFMA counters of the v3 GEMM with fp32 C, with bf16 C + fused column sums, and hipBLASLt
# (bf16 C) on the same operands (tools/gemm_l2_pmc.py), bf16 and MX-fp8 at 4096^3 and 8192^3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for n in 4096 8192; do
for dt in bf16 fp8; do
for set in "WRITE_SIZE GRBM_GUI_ACTIVE" "FETCH_SIZE" "SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/outpmc$i -o pmc -- python3 tools/gemm_l2_pmc.py $n $dt > gpurun_out/outpmc$i.log 2>&1 || { echo "pmc $i failed"; tail -30 gpurun_out/outpmc$i.log; exit 1; }
  echo "$n $dt $set" > gpurun_out/outpmc$i/what.txt
done
done
done
python3 - <<'PY'
import csv, glob, collections, json
out = {}
for d in sorted(glob.glob("gpurun_out/outpmc*/"), key=lambda x: int(x.rstrip("/").split("outpmc")[1])):
    what = open(d + "what.txt").read().split()
    key = f"{what[1]}@{what[0]}"
    fs = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        agg[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, dd in agg.items():
        for c, v in dd.items():
            out.setdefault(key, {}).setdefault(k, {})[c] = round(sorted(v)[len(v) // 2], 1)
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/outpmc_summary.json", "w"), indent=1)
PY
