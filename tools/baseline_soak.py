#!/usr/bin/env python3
"""Calibrate the per-GPU self-baseline (models/baseline.py) on real hardware: the node agent in this process runs
its level-N diagnostics every cycle on one GPU (``diag_interval=0``), forms the GPU's baseline from its first
``runs`` clean cycles, and every later cycle records each rate's ratio to that baseline, the drift notes and the
verdict.  A healthy GPU must stay above the drift line (0.90) in every cycle -- the run-to-run spread this
records is the margin the threshold has.

    python tools/baseline_soak.py --cycles 40 --level 1 --out gpurun_out/baseline_soak.json
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from k8s_gpu_node_checker_amd.agent.agent import Agent  # noqa: E402
from k8s_gpu_node_checker_amd.models import baseline as B  # noqa: E402
from k8s_gpu_node_checker_amd.models import health as H  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=40)
    ap.add_argument("--level", type=int, default=1, choices=(1, 2))
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--runs", type=int, default=B.BASELINE_RUNS, help="clean runs that form the baseline")
    ap.add_argument("--gap", type=float, default=0.0, help="idle seconds between cycles (a cold GPU each time)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    path = os.path.join(tempfile.mkdtemp(prefix="baseline-soak-"), "baseline.json")
    agent = Agent("soak", source="auto", diag_level=args.level, devices=[args.device], diag_when="always",
                  diag_interval=0.0, diag_timeout=300.0, baseline_file=path)
    agent.baselines.runs = args.runs
    rows = []
    t0 = time.time()
    for c in range(args.cycles):
        if c and args.gap > 0:
            time.sleep(args.gap)
        t = time.time()
        rep = agent.probe_once()
        v = H.evaluate_report(rep, 1)
        g = (rep.get("gpus") or [{}])[0]
        diag = g.get("diag") or {}
        row = {"cycle": c, "s": round(time.time() - t, 1), "state": v.state,
               "fractions": {}, "baseline_ratio": {}, "drift": {}}
        for test, res in diag.items():
            if not isinstance(res, dict) or not isinstance(res.get("rates"), dict):
                continue
            exp = res.get("expect") or {}
            row["fractions"][test] = {m: round(r / exp[m], 3) for m, r in res["rates"].items() if exp.get(m)}
            if isinstance(res.get("baseline"), dict):
                row["baseline_ratio"][test] = res["baseline"].get("ratio")
            if res.get("drift"):
                row["drift"][test] = res["drift"]
        if v.state != H.HEALTHY:
            row["reasons"] = v.reasons + v.warnings
        rows.append(row)
        print(json.dumps(row), flush=True)
    ratios = {}
    for row in rows:
        for test, d in row["baseline_ratio"].items():
            for m, r in (d or {}).items():
                ratios.setdefault(f"{test}/{m}", []).append(r)
    summary = {
        "level": args.level, "cycles": args.cycles, "gap_s": args.gap, "baseline_runs": args.runs, "wall_s": round(time.time() - t0, 1),
        "states": {s: sum(1 for r in rows if r["state"] == s) for s in {r["state"] for r in rows}},
        "drift_flags": sum(1 for r in rows if r["drift"]),
        "ratio_to_baseline": {k: {"min": min(v), "median": statistics.median(v), "max": max(v), "n": len(v)}
                              for k, v in sorted(ratios.items())},
        "drift_line": B.DRIFT_RATIO,
        "baseline": json.load(open(path)) if os.path.exists(path) else None,
    }
    print(json.dumps({"summary": {k: v for k, v in summary.items() if k != "baseline"}}, indent=1), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"summary": summary, "rows": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
