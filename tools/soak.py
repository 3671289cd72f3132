#!/usr/bin/env python3
"""Soak the level-2 diagnostics on one GPU for a fixed wall time: every test, every round, with its
verdict and rates, plus min/median/max per metric.  A burn-in tool that faults, hangs or drifts under
sustained load is worse than none; this is the evidence that it does not.

    python tools/soak.py --minutes 5 --out gpurun_out/soak.json
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402

METRICS = (("gemm", "tflops"), ("gemm_fp8", "tflops"), ("hbm", "copy_tbs"), ("hbm", "read_tbs"),
           ("hbm", "write_tbs"), ("memtest", "errors"), ("host_link", "h2d_gbps"), ("host_link", "d2h_gbps"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=5.0)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/soak.json")
    args = ap.parse_args()
    deadline = time.monotonic() + args.minutes * 60
    rounds, failures = [], []
    series: dict = {}
    t0 = time.time()
    while time.monotonic() < deadline:
        res = diag.run(2, args.device)
        rnd = {"t": round(time.time() - t0, 1), "pass": all(r.get("pass") for r in res.values())}
        for test, key in METRICS:
            v = (res.get(test) or {}).get(key)
            if isinstance(v, (int, float)):
                series.setdefault(f"{test}.{key}", []).append(v)
        for kind, row in ((res.get("mfma") or {}).get("kinds") or {}).items():
            series.setdefault(f"mfma.{kind}.tflops", []).append(row["tflops"])
            series.setdefault(f"mfma.{kind}.errors", []).append(row["errors"])
        if not rnd["pass"]:
            failures.append({"t": rnd["t"], "failed": {k: v for k, v in res.items() if not v.get("pass")}})
        rounds.append(rnd)
        print(json.dumps({"round": len(rounds), **rnd}), flush=True)
    summary = {k: {"min": min(v), "median": statistics.median(v), "max": max(v), "n": len(v)}
               for k, v in series.items()}
    out = {"device": diag.device_info(args.device), "minutes": args.minutes, "rounds": len(rounds),
           "all_pass": not failures, "failures": failures[:20], "summary": summary}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"rounds": len(rounds), "all_pass": not failures}))
    return 0 if not failures else 1


if __name__ == "__main__":
    raise SystemExit(main())
