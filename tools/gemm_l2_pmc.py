"""Same operands, three GEMMs (bf16 or MX-fp8, default 8192^3): diag v3 with fp32 C, diag v3 with bf16 C and fused
column sums (the kernel the diagnostics time), and torch (hipBLASLt, bf16 C).

Run under ``rocprofv3 --kernel-trace --pmc ...`` to compare L2 behaviour (TCC hit/miss, FETCH_SIZE) and the
clock (GRBM_GUI_ACTIVE / kernel time) of the two kernels on identical random data
(tools/gpu_pmc_l2.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402
diag.set_gemm_variant("v3")  # a v3 tool: the default (auto) runs the four-wave v4 kernel since round 5

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dt = sys.argv[2] if len(sys.argv) > 2 else "bf16"
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(7)
a = (torch.rand(n, n, device=dev, generator=g) * 2 - 1)
b = (torch.rand(n, n, device=dev, generator=g) * 2 - 1)
st = torch.cuda.current_stream().cuda_stream
c16 = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
cs = torch.empty(n // 128, n, device=dev, dtype=torch.float64)
if dt == "bf16":
    a, b = a.to(torch.bfloat16), b.to(torch.bfloat16)
    c = torch.empty(n, n, device=dev, dtype=torch.float32)
    for _ in range(3):
        diag.gemm_launch(a.data_ptr(), b.data_ptr(), c.data_ptr(), n, n, n, st)
    torch.cuda.synchronize()
    for _ in range(3):
        diag.gemm_launch_ck("bf16", a.data_ptr(), b.data_ptr(), c16.data_ptr(), cs.data_ptr(), n, n, n, st)
    torch.cuda.synchronize()
    for _ in range(3):
        torch.matmul(a, b.t())
    torch.cuda.synchronize()
else:
    a8, b8 = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
    c = torch.empty(n, n, device=dev, dtype=torch.float32)
    one = torch.ones((), device=dev)
    for _ in range(3):
        diag.gemm_fp8_launch(a8.data_ptr(), b8.data_ptr(), c.data_ptr(), n, n, n, st)
    torch.cuda.synchronize()
    for _ in range(3):
        diag.gemm_launch_ck("fp8", a8.data_ptr(), b8.data_ptr(), c16.data_ptr(), cs.data_ptr(), n, n, n, st)
    torch.cuda.synchronize()
    for _ in range(3):
        torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
print("done")
