#!/bin/bash
# L2 / fetch / clock counters of diag v3 vs hipBLASLt on the same operands (tools/gemm_l2_pmc.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for dt in bf16 fp8; do
for set in "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "FETCH_SIZE GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/l2pmc$i -o pmc -- python tools/gemm_l2_pmc.py 8192 $dt > gpurun_out/l2pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -30 gpurun_out/l2pmc$i.log; exit 1; }
done
done
python3 - <<'PY'
import csv, glob, collections, json
out = {}
for d in sorted(glob.glob("gpurun_out/l2pmc*")):
    fs = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not fs:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(fs[0])):
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, dd in agg.items():
        for c, v in dd.items():
            out.setdefault(k, {})[c] = round(sum(v) / len(v), 1)
    ts = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
    if ts:
        dur = collections.defaultdict(list)
        for r in csv.DictReader(open(ts[0])):
            dur[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k, v in dur.items():
            if k in out:
                out[k].setdefault("us", []).append(round(sorted(v)[len(v) // 2], 1))
print(json.dumps(out, indent=1))
json.dump(out, open("gpurun_out/l2pmc_summary.json", "w"), indent=1)
PY
