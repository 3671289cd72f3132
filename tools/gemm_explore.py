"""One-off: v1 / v2 / v3 MFMA GEMM on the box (TFLOP/s + numerics), written to gpurun_out/gemm_explore.json."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag
L = diag.lib()
L.diag_set_gemm_variant.argtypes = [ctypes.c_int]
out = []
names = {1: "v1-128", 2: "v2-256-glds", 3: "v3-256-glds-staggered"}
for variant in (1, 2, 3):
    L.diag_set_gemm_variant(variant)
    for size in (2048, 4096, 8192):
        r = diag.gemm(0, size=size, warmup=3, iters=20, samples=2048)
        r["variant"] = names[variant]
        out.append(r)
        print(json.dumps(r), flush=True)
L.diag_set_gemm_variant(0)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(out, open("gpurun_out/gemm_explore.json", "w"), indent=1)
