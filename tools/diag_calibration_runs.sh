#!/bin/bash
# Cold diagnostic runs for reference calibration on whatever box this lands on: level 1 three times and level 2
# twice (single GPU, no fabric tests), one JSON line of rates and fractions per run into
# gpurun_out/diag_calibration.jsonl, plus the box's identity (VBIOS, driver) from the first run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=gpurun_out/diag_calibration.jsonl
: > "$out"
summ() {
  python3 - "$1" "$2" >> "$out" <<'PY'
import json, sys
doc = json.load(open(sys.argv[2]))
dev = next(iter(doc["devices"].values()))
d = dev["tests"]
row = {"run": sys.argv[1], "info": dev.get("info")}
for t, r in d.items():
    if isinstance(r, dict) and isinstance(r.get("rates"), dict):
        row[t] = {k: round(v, 2) for k, v in r["rates"].items()}
        row[t]["fraction"] = r.get("fraction")
        if r.get("shape"):
            row[t]["shape"] = r["shape"]
row["verdict"] = {t: ("degraded" if r.get("degraded") else "pass" if r.get("pass") else "fail")
                  for t, r in d.items() if isinstance(r, dict) and "pass" in r}
print(json.dumps(row))
PY
}
for run in l1a l1b l1c; do
  timeout -k 10 120 python3 -m k8s_gpu_node_checker_amd.ops.diag --level 1 > gpurun_out/cal_$run.json 2> gpurun_out/cal_$run.err
  rc=$?; [ $rc -le 1 ] || exit $rc
  summ $run gpurun_out/cal_$run.json || exit 1
done
for run in l2a l2b; do
  timeout -k 10 240 python3 -m k8s_gpu_node_checker_amd.ops.diag --level 2 --no-p2p --no-rccl > gpurun_out/cal_$run.json 2> gpurun_out/cal_$run.err
  rc=$?; [ $rc -le 1 ] || exit $rc
  summ $run gpurun_out/cal_$run.json || exit 1
done
cat "$out"
