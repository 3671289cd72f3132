"""The fp8 v3 GEMM in its two MFMA forms (scaled ``v_mfma_scale_f32_16x16x128_f8f6f4`` with unit scales, and the
unscaled ``v_mfma_f32_16x16x128_f8f6f4`` the diagnostics now run) and hipBLASLt's fp8 GEMM (``_scaled_mm``), all
bf16 C, on the same operands: 3 launches each, for ``rocprofv3 --kernel-trace --pmc ...`` (tools/gpu_pmc_fp8.sh).

    python tools/gemm_fp8_pmc.py [n]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402
diag.set_gemm_variant("v3")  # a v3 tool: the default (auto) runs the four-wave v4 kernel since round 5

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
assert n % 256 == 0, "the v3 kernel tiles 256x256"
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(7)
a = (torch.rand(n, n, device=dev, generator=g) * 2 - 1).to(torch.float8_e4m3fn)
b = (torch.rand(n, n, device=dev, generator=g) * 2 - 1).to(torch.float8_e4m3fn)
st = torch.cuda.current_stream().cuda_stream
c16 = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
cs = torch.empty(n // 128, n, device=dev, dtype=torch.float64)
one = torch.ones((), device=dev)
for unscaled in (False, True):
    diag.set_gemm_fp8_unscaled(unscaled)
    for _ in range(3):
        diag.gemm_launch_ck("fp8", a.data_ptr(), b.data_ptr(), c16.data_ptr(), cs.data_ptr(), n, n, n, st)
    torch.cuda.synchronize()
diag.set_gemm_fp8_unscaled(True)
for _ in range(3):
    torch._scaled_mm(a, b.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
torch.cuda.synchronize()
print("done")
