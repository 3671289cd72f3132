#!/usr/bin/env python3
"""A/B of the fp8 v3 GEMM's MFMA form: ``v_mfma_scale_f32_16x16x128_f8f6f4`` with unit scales (the MX path the
diagnostics have timed) against the unscaled ``v_mfma_f32_16x16x128_f8f6f4`` (what hipBLASLt's fp8 GEMMs issue
on gfx950), both writing bf16 C with fused column sums (``gemm_launch_ck``), with hipBLASLt (``_scaled_mm``, bf16
C) in the same interleaved rounds.  The two forms must produce bit-identical C and column sums.

    python tools/gemm_fp8_mfma_ab.py --rounds 9 --sizes 4096,8192
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
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--sizes", default="4096,8192")
    args = ap.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    one = torch.ones((), device="cuda")
    for n in (int(x) for x in args.sizes.split(",")):
        iters = 40 if n <= 4096 else 15
        g = torch.Generator(device="cuda").manual_seed(n)
        x = (torch.rand(n, n, device="cuda", generator=g) * 2 - 1).to(torch.float8_e4m3fn)
        y = (torch.rand(n, n, device="cuda", generator=g) * 2 - 1).to(torch.float8_e4m3fn)
        yt = y.t()
        outs = {k: (torch.empty(n, n, device="cuda", dtype=torch.bfloat16),
                    torch.empty(n // 128, n, device="cuda", dtype=torch.float64)) for k in ("scaled", "unscaled")}

        def ours(form):
            c, cs = outs[form]

            def run():
                diag.set_gemm_fp8_unscaled(form == "unscaled")
                diag.gemm_launch_ck("fp8", x.data_ptr(), y.data_ptr(), c.data_ptr(), cs.data_ptr(), n, n, n, st)
            return run
        runs = {"scaled": ours("scaled"), "unscaled": ours("unscaled"),
                "hipblaslt": lambda: torch._scaled_mm(x, yt, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)}
        runs["scaled"]()
        runs["unscaled"]()
        torch.cuda.synchronize()
        same = torch.equal(outs["scaled"][0], outs["unscaled"][0]) and torch.equal(outs["scaled"][1], outs["unscaled"][1])
        ref = torch._scaled_mm(x, yt, scale_a=one, scale_b=one, out_dtype=torch.float32)
        err = ((outs["unscaled"][0].float() - ref).abs().max() / ref.abs().max()).item()
        tf = {k: [] for k in runs}
        for _ in range(args.rounds):
            for k, fn in runs.items():
                tf[k].append(2.0 * n ** 3 / timed(fn, iters) / 1e9)
        diag.set_gemm_fp8_unscaled(True)
        med = {k: round(statistics.median(v), 1) for k, v in tf.items()}
        print(json.dumps({"size": n, "rounds": args.rounds, "median_tflops": med,
                          "best_tflops": {k: round(max(v), 1) for k, v in tf.items()},
                          "fraction_of_hipblaslt": {k: round(med[k] / med["hipblaslt"], 3) for k in med if k != "hipblaslt"},
                          "outputs_identical": same, "rel_err_vs_hipblaslt_fp32": err}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
