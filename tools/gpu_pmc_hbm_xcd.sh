#!/bin/bash
# Counter passes over the per-XCD HBM test (one rocprofv3 run per set, kernel trace only alongside).
# Summary: gpurun_out/pmc_hbm_xcd/summary.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_hbm_xcd
i=0
for set in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d gpurun_out/pmc_hbm_xcd/p$i -o pmc \
    -- python tools/hbm_xcd_pmc.py > gpurun_out/pmc_hbm_xcd/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -20 gpurun_out/pmc_hbm_xcd/p$i.log; }
done
python3 - <<'PY'
import csv, collections, glob, json
out = {}
for f in sorted(glob.glob("gpurun_out/pmc_hbm_xcd/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        if k.startswith("hbm_xcd"):
            out.setdefault(k, collections.defaultdict(list))[r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: {c: {"per_dispatch": v, "dispatches": len(v)} for c, v in d.items()} for k, d in out.items()}
json.dump(res, open("gpurun_out/pmc_hbm_xcd/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1)[:3000])
PY
