#!/usr/bin/env python3
"""Cold single runs of the diagnostics, as the agent meets the GPU once per --diag-interval: each run in a
fresh process after an idle gap, one JSON line per run with the GEMM / burn-in rates (the reference rates in
ops/diag.py are the lower of a soak median and these).

    python tools/diag_cold.py --runs 5 --gap 8 --level 1
    python tools/diag_cold.py --runs 5 --level 2 --variants v3,v4   # bf16 GEMM kernels alternated run by run
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = ("import json,sys; sys.path.insert(0, %r)\n"
         "from k8s_gpu_node_checker_amd.ops import diag\n"
         "diag.set_gemm_variant(%r)\n"
         "r = diag.run(%d, 0)\n"
         "print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk in ('tflops', 'kinds', 'copy_tbs', 'read_tbs', "
         "'fraction', 'pass', 'degraded')} for k, v in r.items() if isinstance(v, dict)}))")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--gap", type=float, default=8.0, help="idle seconds before each run")
    ap.add_argument("--level", type=int, default=1, choices=(1, 2))
    ap.add_argument("--variants", default="auto", help="bf16 GEMM kernels (diag.GEMM_VARIANTS), comma-separated: "
                                                        "each run of the loop runs each of them, in turn")
    args = ap.parse_args()
    for i in range(args.runs):
        for variant in args.variants.split(","):
            time.sleep(args.gap)
            p = subprocess.run([sys.executable, "-c", CHILD % (REPO, variant, args.level)], capture_output=True,
                               text=True, timeout=300)
            line = p.stdout.strip().splitlines()[-1] if p.stdout.strip() else "{}"
            print(json.dumps({"run": i, "level": args.level, "variant": variant, "rc": p.returncode,
                              "res": json.loads(line)}), flush=True)
            if p.returncode != 0:
                print(p.stderr[-800:], file=sys.stderr)
                return 1
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
