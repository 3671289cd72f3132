"""MX-fp8 / MX-fp4 GEMM (diag v3 pipeline) vs bf16 v3 vs torch (hipBLASLt) at 4096^3 / 8192^3, TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402
diag.set_gemm_variant("v3")  # a v3 tool: the default (auto) runs the four-wave v4 kernel since round 5


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    st = torch.cuda.current_stream().cuda_stream
    for n in (4096, 8192):
        it = 50 if n == 4096 else 20
        a = torch.randn(n, n, device="cuda")
        b = torch.randn(n, n, device="cuda")
        a8, b8 = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
        a16, b16 = a.to(torch.bfloat16), b.to(torch.bfloat16)
        c = torch.empty(n, n, device="cuda")
        rows = {}
        ref = a8.float() @ b8.float().t()
        errs = {}
        for epi in (False, True):
            diag.set_gemm_epilogue(epi)
            tag = "_lds_epilogue" if epi else ""
            c.fill_(float("nan"))
            rows["mxfp8_v3" + tag] = timeit(
                lambda: diag.gemm_fp8_launch(a8.data_ptr(), b8.data_ptr(), c.data_ptr(), n, n, n, st), it)
            errs["mxfp8_v3" + tag] = ((c - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
            rows["bf16_v3" + tag] = timeit(
                lambda: diag.gemm_launch(a16.data_ptr(), b16.data_ptr(), c.data_ptr(), n, n, n, st), it)
        diag.set_gemm_epilogue(True)
        codes_a = torch.randint(0, 16, (n, n), device="cuda", dtype=torch.int32)
        codes_b = torch.randint(0, 16, (n, n), device="cuda", dtype=torch.int32)
        a4 = (codes_a[:, 0::2] | (codes_a[:, 1::2] << 4)).to(torch.uint8).contiguous()
        b4 = (codes_b[:, 0::2] | (codes_b[:, 1::2] << 4)).to(torch.uint8).contiguous()
        rows["mxfp4_v3_lds_epilogue"] = timeit(
            lambda: diag.gemm_fp4_launch(a4.data_ptr(), b4.data_ptr(), c.data_ptr(), n, n, n, st), it)
        rows["torch_bf16"] = timeit(lambda: a16 @ b16.t(), it)
        try:
            one = torch.ones((), device="cuda")
            rows["torch_scaled_mm_fp8"] = timeit(
                lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16), it)
        except Exception as e:  # not every build exposes fp8 GEMM
            print(json.dumps({"size": n, "torch_scaled_mm_fp8": f"unavailable: {type(e).__name__}: {e}"[:200]}))
        for k, ms in rows.items():
            print(json.dumps({"size": n, "kernel": k, "ms": round(ms, 4),
                              "tflops": round(2 * n ** 3 / (ms * 1e-3) / 1e12, 1),
                              **({"max_rel_err": errs[k]} if k in errs else {})}), flush=True)


if __name__ == "__main__":
    main()
