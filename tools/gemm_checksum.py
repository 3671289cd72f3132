#!/usr/bin/env python3
"""Calibration and cost of the GEMM tests' whole-output tile checksums (``gemm_checksum`` in diag.hip).

For bf16 and MX-fp8 at 4096^3 and 8192^3, several runs each: the healthy checksum error (the largest
|tile column sum - fp64 reference| / sum|a*b| over every column of every tile, which sets GEMM_CK_TOL /
GEMM_FP8_CK_TOL), the wall time the check adds (the same test with and without it), and one run with an
injected output to show it is caught, located to its tile and attributed to an XCD.

    python tools/gemm_checksum.py --out gpurun_out/gemm_checksum.jsonl
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="2048,4096,8192")
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    L = diag.lib()
    lines = []
    for name, fn, plain, tol in (("bf16", "diag_gemm_bf16_x", "diag_gemm_bf16", diag.GEMM_CK_TOL),
                                 ("mxfp8", "diag_gemm_fp8_x", "diag_gemm_fp8", diag.GEMM_FP8_CK_TOL)):
        for size in (int(s) for s in args.sizes.split(",")):
            iters = 20 if size <= 4096 else 10
            errs, with_ck, without = [], [], []
            for _ in range(args.runs):
                t = time.perf_counter()
                _, _, _, ck, out = diag._checked_gemm(fn, 0, size, 3, iters, 4096, None, tol)
                with_ck.append(time.perf_counter() - t)
                errs.append(ck)
                if out[0]:
                    print(json.dumps({"dtype": name, "size": size, "healthy_run_failed": out}), flush=True)
                    return 1
                tf, err, ms = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
                t = time.perf_counter()
                diag._check(getattr(L, plain)(0, size, size, size, 3, iters, 4096, ctypes.byref(tf), ctypes.byref(err),
                                              ctypes.byref(ms)))
                without.append(time.perf_counter() - t)
            # one corrupted output in the middle of the matrix
            elem = (size // 2 + 37) * size + size // 3
            _, _, _, ck, out = diag._checked_gemm(fn, 0, size, 1, 1, 4096, elem, tol)
            row = {"dtype": name, "size": size, "runs": args.runs, "tol": tol,
                   "healthy_checksum_err_max": max(errs), "healthy_checksum_err_median": statistics.median(errs),
                   "margin": round(tol / max(max(errs), 1e-300), 1),
                   "check_ms_median": round((statistics.median(with_ck) - statistics.median(without)) * 1e3, 1),
                   "test_wall_ms_median": round(statistics.median(with_ck) * 1e3, 1),
                   "injected": {"elem_row": elem // size, "elem_col": elem % size, "bad_tiles": out[0],
                                "bad_columns": out[1], "xcd_tiles": out[2:10], "first_bad_tile": out[10:12],
                                "checksum_err": ck}}
            print(json.dumps(row), flush=True)
            lines.append(row)
    if args.out:
        with open(args.out, "w") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
