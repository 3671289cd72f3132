"""fp8 (E4M3) GEMM numerics on the v3 kernel: three shapes against an fp64 reference of the same operands (error over
the |A||B| magnitude, exact fraction), beside torch's fp32 matmul and _scaled_mm (profiles/fp8_numerics_mi355x.jsonl)."""
import json, sys, torch
sys.path.insert(0, ".")
from k8s_gpu_node_checker_amd.ops import diag
diag.set_gemm_variant("v3")  # a v3 tool: the default (auto) runs the four-wave v4 kernel since round 5
st = torch.cuda.current_stream().cuda_stream
for (m, n, k) in [(256, 256, 128), (512, 256, 384), (1024, 768, 8192)]:
    g = torch.Generator(device="cuda").manual_seed(1)
    a = torch.randn(m, k, device="cuda", generator=g).to(torch.float8_e4m3fn)
    bt = torch.randn(n, k, device="cuda", generator=g).to(torch.float8_e4m3fn)
    c = torch.empty(m, n, device="cuda")
    diag.gemm_fp8_launch(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, st)
    torch.cuda.synchronize()
    ad, bd = a.double(), bt.double()
    ref = ad @ bd.t()
    mag = ad.abs() @ bd.abs().t()
    err = (c.double() - ref).abs()
    out = {"shape": [m, n, k], "max_abs_err": err.max().item(), "max_err_over_mag": (err / mag.clamp_min(1e-30)).max().item(),
           "max_rel_clamp1": (err / ref.abs().clamp_min(1.0)).max().item(), "frac_exact": (err == 0).double().mean().item()}
    ref32 = a.float() @ bt.float().t()
    out["torch_fp32_vs_fp64_max_abs"] = (ref32.double() - ref).abs().max().item()
    try:
        one = torch.ones((), device="cuda")
        sm = torch._scaled_mm(a, bt.t(), scale_a=one, scale_b=one, out_dtype=torch.float32)
        out["scaled_mm_max_err_over_mag"] = ((sm.double() - ref).abs() / mag.clamp_min(1e-30)).max().item()
    except Exception as e:
        out["scaled_mm"] = str(e)[:120]
    print(json.dumps(out), flush=True)
