#!/bin/bash
# Does rocprofv3 itself lower the compute diagnostics' rates?  On one box: the level-1 suite unprofiled twice,
# under `rocprofv3 --kernel-trace --stats` once, then unprofiled again; one JSON line per run with the compute
# rates (gemm, gemm_fp8, mfma kinds) into gpurun_out/diag_profiled_vs_not.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/diag_profiled_vs_not.jsonl
: > "$out"
summ() {
  python3 - "$1" "$2" >> "$out" <<'PY'
import json, sys
doc = json.load(open(sys.argv[2]))
d = next(iter(doc["devices"].values()))["tests"]
row = {"run": sys.argv[1]}
for t, r in d.items():
    if isinstance(r, dict) and isinstance(r.get("rates"), dict):
        row[t] = {k: round(v, 1) for k, v in r["rates"].items()}
        row[t]["fraction"] = r.get("fraction")
row["verdict"] = {t: ("degraded" if r.get("degraded") else "pass" if r.get("pass") else "fail")
                  for t, r in d.items() if isinstance(r, dict) and "pass" in r}
print(json.dumps(row))
PY
}
for run in plain1 plain2; do
  timeout -k 10 120 python3 -m k8s_gpu_node_checker_amd.ops.diag --level 1 > gpurun_out/dpv_$run.json 2> gpurun_out/dpv_$run.err
  rc=$?; [ $rc -le 1 ] || exit $rc
  summ $run gpurun_out/dpv_$run.json || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dpv_prof -o p -- python3 -m k8s_gpu_node_checker_amd.ops.diag --level 1 > gpurun_out/dpv_profiled.json 2> gpurun_out/dpv_profiled.err
rc=$?; [ $rc -le 1 ] || exit $rc
summ profiled gpurun_out/dpv_profiled.json || exit 1
timeout -k 10 120 python3 -m k8s_gpu_node_checker_amd.ops.diag --level 1 > gpurun_out/dpv_plain3.json 2> gpurun_out/dpv_plain3.err
rc=$?; [ $rc -le 1 ] || exit $rc
summ plain3 gpurun_out/dpv_plain3.json
cat "$out"
