#!/usr/bin/env python3
"""Output A/B of the v3 GEMM: fp32 C (``gemm_launch`` / ``gemm_fp8_launch``) against bf16 C with fused 128-row
column sums (``gemm_launch_ck``, what the diagnostics time), with torch/hipBLASLt (bf16 C) in the same rounds.

Interleaved rounds in one process on the same random operands; both outputs checked against torch first.
One JSON line per (dtype, size).

    python tools/gemm_output_ab.py --rounds 7
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402
diag.set_gemm_variant("v3")  # a v3 tool: the default (auto) runs the four-wave v4 kernel since round 5


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--sizes", default="4096,8192")
    args = ap.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    one = torch.ones((), device="cuda")
    for n in (int(x) for x in args.sizes.split(",")):
        iters = 40 if n <= 4096 else 15
        g = torch.Generator(device="cuda").manual_seed(n)
        a = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
        b = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
        c32 = torch.empty(n, n, device="cuda")
        c16 = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        cs = torch.empty(n // 128, n, device="cuda", dtype=torch.float64)
        for dt, x, y, launch in (("bf16", a.to(torch.bfloat16), b.to(torch.bfloat16), diag.gemm_launch),
                                 ("fp8", a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn), diag.gemm_fp8_launch)):
            yt = y.t()
            runs = {
                "fp32_out": lambda: launch(x.data_ptr(), y.data_ptr(), c32.data_ptr(), n, n, n, st),
                "bf16_out_fused_ck": lambda: diag.gemm_launch_ck(dt, x.data_ptr(), y.data_ptr(), c16.data_ptr(),
                                                                 cs.data_ptr(), n, n, n, st),
                "hipblaslt_bf16_out": (lambda: torch.matmul(x, yt)) if dt == "bf16" else
                (lambda: torch._scaled_mm(x, yt, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)),
            }
            runs["fp32_out"]()
            runs["bf16_out_fused_ck"]()
            torch.cuda.synchronize()
            exact = torch.equal(c16, c32.to(torch.bfloat16))
            want = c32.double().view(n // 128, 128, n).sum(dim=1)
            ck_err = ((cs - want).abs() / c32.double().abs().view(n // 128, 128, n).sum(dim=1)).max().item()
            tf = {k: [] for k in runs}
            for _ in range(args.rounds):
                for k, fn in runs.items():
                    tf[k].append(2.0 * n ** 3 / timed(fn, iters) / 1e9)
            med = {k: round(statistics.median(v), 1) for k, v in tf.items()}
            lib = med["hipblaslt_bf16_out"]
            print(json.dumps({"dtype": "mxfp8" if dt == "fp8" else dt, "size": n, "median_tflops": med,
                              "best_tflops": {k: round(max(v), 1) for k, v in tf.items()},
                              "fraction_of_hipblaslt": {k: round(med[k] / lib, 3) for k in ("fp32_out",
                                                                                             "bf16_out_fused_ck")},
                              "bf16_out_equals_rounded_fp32_out": exact, "fused_ck_rel_err": ck_err}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
