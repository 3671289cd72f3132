#!/usr/bin/env python3
"""A/B of v4's tail-wave path (diag.hip ``gemm_v4_tail_kernel``) on the GEMM the diagnostics time:
v4 with a short last wave run as 128x128 quadrants (``tail=True``, the default) against v4 running it as 256x256
tiles (``tail=False``) and hipBLASLt (``torch.matmul``, or ``torch._scaled_mm`` for ``--dtype fp8``; bf16 out),
interleaved round by round on the same operands.  Before timing, both v4 forms' bf16 C and fused column sums are
compared bit for bit.  One JSON line per size (median / best TFLOP/s, the fractions of hipBLASLt).

    python tools/gemm_tail_ab.py --rounds 7 --sizes 4096,6144,8192,10240
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
    ap.add_argument("--sizes", default="4096,6144,8192,10240")
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp8"))
    args = ap.parse_args()
    fp8 = args.dtype == "fp8"
    st = torch.cuda.current_stream().cuda_stream
    for spec in args.sizes.split(","):
        m, n, k = (int(x) for x in spec.split("x")) if "x" in spec else (int(spec),) * 3
        flop = 2.0 * m * n * k
        iters = max(3, min(40, int(40 * 4096 ** 3 / (m * n * k))))
        g = torch.Generator(device="cuda").manual_seed(n)
        dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
        a = (torch.rand(m, k, device="cuda", generator=g) * 2 - 1).to(dt)
        bt = (torch.rand(n, k, device="cuda", generator=g) * 2 - 1).to(dt)
        b = bt.t()
        one = torch.ones((), device="cuda")
        c16 = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        cs = torch.empty(m // 128, n, device="cuda", dtype=torch.float64)

        def ck(tail):
            def go():
                with diag.gemm_config(variant="v4", tail=tail):
                    diag.gemm_launch_ck(args.dtype, a.data_ptr(), bt.data_ptr(), c16.data_ptr(), cs.data_ptr(), m,
                                        n, k, st)
            return go
        outs = {}
        for tail in (True, False):
            c16.fill_(float("nan"))
            cs.fill_(float("nan"))
            ck(tail)()
            torch.cuda.synchronize()
            outs[tail] = (c16.clone(), cs.clone())
        same = torch.equal(outs[True][0], outs[False][0]) and torch.equal(outs[True][1], outs[False][1])
        runs = {"v4_tail": [], "v4_no_tail": [], "hipblaslt_bf16_out": []}
        blas = (lambda: torch._scaled_mm(a, b, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)) if fp8 else (
            lambda: torch.matmul(a, b))
        fns = {"v4_tail": ck(True), "v4_no_tail": ck(False), "hipblaslt_bf16_out": blas}
        for r in range(args.rounds):
            order = list(fns) if r % 2 == 0 else list(reversed(list(fns)))
            for name in order:
                runs[name].append(flop / (timed(fns[name], iters) * 1e-3) / 1e12)
        med = {k2: round(statistics.median(v), 1) for k2, v in runs.items()}
        tiles = (m // 256) * (n // 256)
        print(json.dumps({"dtype": args.dtype, "shape": [m, n, k], "tiles": tiles, "waves": round(tiles / 256, 3),
                          "rounds": args.rounds, "median_tflops": med,
                          "best_tflops": {k2: round(max(v), 1) for k2, v in runs.items()},
                          "fraction_of_hipblaslt": {k2: round(med[k2] / med["hipblaslt_bf16_out"], 3)
                                                    for k2 in ("v4_tail", "v4_no_tail")},
                          "tail_over_no_tail": round(med["v4_tail"] / med["v4_no_tail"], 3),
                          "bit_identical": same}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
