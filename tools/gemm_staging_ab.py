#!/usr/bin/env python3
"""v3 GEMM operand staging A/B: ``global_load_lds_dwordx4`` vs ``buffer_load_dwordx4 ... lds``.

Interleaved rounds in one process (methodology rule: perf deltas from interleaved rounds, same data),
bf16 / MX-fp8 / MX-fp4 at 4096^3 and 8192^3 on random operands, every variant's full output checked
against torch.  One JSON line per (dtype, size) with the median and best TFLOP/s of each path.

    python tools/gemm_staging_ab.py --rounds 7
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
    diag.set_gemm_epilogue(True)
    for n in (int(x) for x in args.sizes.split(",")):
        iters = 40 if n <= 4096 else 15
        g = torch.Generator(device="cuda").manual_seed(n)
        a = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
        b = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
        c = torch.empty(n, n, device="cuda")
        ops = {
            "bf16": (a.to(torch.bfloat16), b.to(torch.bfloat16), diag.gemm_launch, n),
            "mxfp8": (a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn), diag.gemm_fp8_launch, n),
        }
        for name, (x, y, launch, k) in ops.items():
            ref = x.float() @ y.float().t()
            res = {}
            for buf in (False, True):
                diag.set_gemm_buffer_loads(buf)
                c.fill_(float("nan"))
                launch(x.data_ptr(), y.data_ptr(), c.data_ptr(), n, n, k, st)
                torch.cuda.synchronize()
                err = ((c - ref).abs().max() / ref.abs().max()).item()
                res[buf] = {"err": err, "tf": []}
            for _ in range(args.rounds):
                for buf in (False, True):
                    diag.set_gemm_buffer_loads(buf)
                    ms = timed(lambda: launch(x.data_ptr(), y.data_ptr(), c.data_ptr(), n, n, k, st), iters)
                    res[buf]["tf"].append(2.0 * n * n * k / ms / 1e9)
            diag.set_gemm_buffer_loads(False)
            out = {"dtype": name, "size": n}
            for buf, tag in ((False, "global_load_lds"), (True, "buffer_load_lds")):
                tf = res[buf]["tf"]
                out[tag] = {"median_tflops": round(statistics.median(tf), 1), "best_tflops": round(max(tf), 1),
                            "max_err_vs_torch": res[buf]["err"]}
            print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
