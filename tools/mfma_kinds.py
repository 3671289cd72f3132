#!/usr/bin/env python3
"""Rates and exactness of every matrix-core kind of the burn-in (``ops/diag.mfma_burn``), N cold-to-warm runs.

The reference rate of a kind is the lower of the soak median and what a cold run measures
(``ops/diag.py`` threshold block); this prints both ends:

    python tools/mfma_kinds.py --runs 40 --out gpurun_out/mfma_kinds.json
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


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=40)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    series = {k: [] for k in diag.MFMA_KINDS}
    errors = {k: 0 for k in diag.MFMA_KINDS}
    t0 = time.time()
    for i in range(args.runs):
        r = diag.mfma_burn(args.device)
        for k, row in r["kinds"].items():
            series[k].append(row["tflops"])
            errors[k] += row["errors"]
        print(json.dumps({"run": i, **{k: r["kinds"][k]["tflops"] for k in r["kinds"]}}), flush=True)
    out = {"device": diag.device_info(args.device), "runs": args.runs, "wall_s": round(time.time() - t0, 1),
           "first_run": {k: v[0] for k, v in series.items()},
           "tflops": {k: {"min": min(v), "median": statistics.median(v), "max": max(v)} for k, v in series.items()},
           "errors": errors, "reference": diag.REFERENCE_RATES["mfma"]}
    text = json.dumps(out, indent=1)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    return 0 if not any(errors.values()) else 1


if __name__ == "__main__":
    raise SystemExit(main())
