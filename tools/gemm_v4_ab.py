#!/usr/bin/env python3
"""A/B of the bf16 GEMM kernels in one process: the four-wave v4 kernel (diag.hip ``gemm_v4_kernel``, the default
since round 5) against the 8-wave v3 kernel it replaced and torch.matmul (hipBLASLt), on the same random operands,
interleaved rounds (the clock drifts with temperature: a kernel timed in one block would carry the drift).

Both outputs the diagnostics use are timed: fp32 C (``gemm_launch``) and bf16 C with fused 128-row column sums
(``gemm_launch_ck``, what the ``gemm`` diagnostic times; hipBLASLt writes bf16 C too).  Before timing, v4's fp32 C,
bf16 C and column sums are compared with v3's bit for bit.  One JSON line per size.

    python tools/gemm_v4_ab.py --rounds 7 --sizes 4096,8192,16384
    python tools/gemm_v4_ab.py --sizes 4096x4096x32768,8192x8192x1024   # M x N x K
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402


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
    ap.add_argument("--variants", default="v3,v4", help="diag kernels to time (the first is the baseline)")
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp8"))
    args = ap.parse_args()
    variants = args.variants.split(",")
    st = torch.cuda.current_stream().cuda_stream
    for spec in args.sizes.split(","):
        m, n, k = (int(x) for x in spec.split("x")) if "x" in spec else (int(spec),) * 3
        flop = 2.0 * m * n * k
        iters = max(3, min(40, int(40 * 4096 ** 3 / (m * n * k))))
        g = torch.Generator(device="cuda").manual_seed(n)
        fp8 = args.dtype == "fp8"
        dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
        a = (torch.rand(m, k, device="cuda", generator=g) * 2 - 1).to(dt)
        bt = (torch.rand(n, k, device="cuda", generator=g) * 2 - 1).to(dt)
        launch = diag.gemm_fp8_launch if fp8 else diag.gemm_launch
        one = torch.ones((), device="cuda")
        b = bt.t()
        c32 = torch.empty(m, n, device="cuda")
        c16 = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        cs = torch.empty(m // 128, n, device="cuda", dtype=torch.float64)

        def fp32(variant):
            def go():
                with diag.gemm_config(variant=variant):
                    launch(a.data_ptr(), bt.data_ptr(), c32.data_ptr(), m, n, k, st)
            return go

        def ck(variant):
            def go():
                with diag.gemm_config(variant=variant):
                    diag.gemm_launch_ck(args.dtype, a.data_ptr(), bt.data_ptr(), c16.data_ptr(), cs.data_ptr(), m, n,
                                        k, st)
            return go

        outs = {}
        for v in variants:
            fp32(v)()
            ck(v)()
            torch.cuda.synchronize()
            outs[v] = (c32.clone(), c16.clone(), cs.clone())
        base = variants[0]
        mag = outs[base][0].double().abs().view(m // 128, 128, n).sum(dim=1)
        same = {v: {"fp32_c": torch.equal(outs[base][0], outs[v][0]), "bf16_c": torch.equal(outs[base][1], outs[v][1]),
                    "colsums_bitwise": torch.equal(outs[base][2], outs[v][2]),
                    "colsums_rel_diff": ((outs[base][2] - outs[v][2]).abs() / mag).max().item()}
                for v in variants[1:]}
        last = variants[-1]
        ref_err = ((outs[last][0] - a.float() @ b.float()).abs().max() / k).item() if m * n <= 8192 ** 2 else None
        del outs, mag
        # the knob is switched outside the timed loop: gemm_config per launch would time ctypes calls too
        runs = {}
        for v in variants:
            runs[f"{v}_fp32_out"] = (v, lambda: launch(a.data_ptr(), bt.data_ptr(), c32.data_ptr(), m, n, k, st))
            runs[f"{v}_bf16_out_fused_ck"] = (v, lambda: diag.gemm_launch_ck(args.dtype, a.data_ptr(), bt.data_ptr(),
                                                                             c16.data_ptr(), cs.data_ptr(), m, n, k,
                                                                             st))
        runs["hipblaslt_bf16_out"] = (None, (lambda: torch._scaled_mm(a, b, scale_a=one, scale_b=one,
                                                                       out_dtype=torch.bfloat16)) if fp8 else
                                      (lambda: torch.matmul(a, b)))
        tf = {k: [] for k in runs}
        for _ in range(args.rounds):
            for key, (v, fn) in runs.items():
                if v is None:
                    ms = timed(fn, iters)
                else:
                    with diag.gemm_config(variant=v):
                        ms = timed(fn, iters)
                tf[key].append(flop / ms / 1e9)
        med = {k: round(statistics.median(x), 1) for k, x in tf.items()}
        lib = med["hipblaslt_bf16_out"]
        print(json.dumps({"dtype": args.dtype, "size": n if m == n == k else [m, n, k], "rounds": args.rounds, "median_tflops": med,
                          "best_tflops": {k: round(max(x), 1) for k, x in tf.items()},
                          "fraction_of_hipblaslt": {k: round(med[k] / lib, 3) for k in med if k != "hipblaslt_bf16_out"},
                          "over_" + base: {f"{v}_{o}": round(med[f"{v}_{o}"] / med[f"{base}_{o}"], 3)
                                           for v in variants[1:] for o in ("fp32_out", "bf16_out_fused_ck")},
                          "same_as_" + base: same, last + "_max_abs_err_over_k": ref_err}), flush=True)
        del a, bt, b, c32, c16, cs
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
