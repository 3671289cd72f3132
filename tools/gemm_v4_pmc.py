"""Same operands, three GEMMs with bf16 C (default 8192^3, bf16 operands; ``fp8`` as the second argument for E4M3
operands): diag v3 (8 waves) and v4 (4 waves, asm-ordered loop), both with fused column sums, and torch (hipBLASLt:
``torch.matmul``, or ``torch._scaled_mm`` with unit scales for fp8).  Run under ``rocprofv3 --kernel-trace --pmc ...``
(tools/gpu_pmc_v4.sh) to compare MFMA busy, LDS conflicts, waits and HBM bytes of the three kernels."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16"
assert dtype in ("bf16", "fp8"), dtype
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(7)
dt = torch.float8_e4m3fn if dtype == "fp8" else torch.bfloat16
a = (torch.rand(n, n, device=dev, generator=g) * 2 - 1).to(dt)
b = (torch.rand(n, n, device=dev, generator=g) * 2 - 1).to(dt)
one = torch.ones((), device=dev)
st = torch.cuda.current_stream().cuda_stream
c16 = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
cs = torch.empty(n // 128, n, device=dev, dtype=torch.float64)
# interleaved rounds (the first launches of each kernel run slow: take the median per kernel)
for _ in range(5):
    for variant in ("v3", "v4"):
        with diag.gemm_config(variant=variant):
            for _ in range(2):
                diag.gemm_launch_ck(dtype, a.data_ptr(), b.data_ptr(), c16.data_ptr(), cs.data_ptr(), n, n, n, st)
        torch.cuda.synchronize()
    for _ in range(2):
        if dtype == "fp8":
            torch._scaled_mm(a, b.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        else:
            torch.matmul(a, b.t())
    torch.cuda.synchronize()
print("done")
