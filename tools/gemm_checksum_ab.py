#!/usr/bin/env python3
"""Does the whole-output checksum pass change the GEMM tests' measured rate?  The level-2 order (bf16 then
MX-fp8 at 8192^3), rounds alternating with and without the checksums (ck_tol < 0 skips them); the rate is
timed before either check runs, so the two columns should agree within run-to-run noise.

    python tools/gemm_checksum_ab.py --rounds 12
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--size", type=int, default=8192)
    args = ap.parse_args()
    tf = {(dt, ck): [] for dt in ("bf16", "mxfp8") for ck in (True, False)}
    for r in range(args.rounds):
        for ck in ((True, False) if r % 2 == 0 else (False, True)):
            for dt, fn, tol in (("bf16", "diag_gemm_bf16_x", diag.GEMM_CK_TOL),
                                ("mxfp8", "diag_gemm_fp8_x", diag.GEMM_FP8_CK_TOL)):
                rate, _, _, _, out = diag._checked_gemm(fn, 0, args.size, 3, 20, 4096, None, tol if ck else -1.0)
                tf[(dt, ck)].append(rate)
        print(f"round {r + 1} done", file=sys.stderr, flush=True)
    for dt in ("bf16", "mxfp8"):
        a, b = tf[(dt, True)], tf[(dt, False)]
        print(json.dumps({"dtype": dt, "size": args.size, "rounds": args.rounds,
                          "with_checksums_median": round(statistics.median(a), 1),
                          "without_median": round(statistics.median(b), 1),
                          "with_min_max": [round(min(a), 1), round(max(a), 1)],
                          "without_min_max": [round(min(b), 1), round(max(b), 1)]}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
