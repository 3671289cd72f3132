"""Run the v2 GEMM a few times at 8192^3 (for rocprofv3 --pmc collection)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag
print(diag.gemm(0, size=int(sys.argv[1]) if len(sys.argv) > 1 else 8192, warmup=1, iters=3, samples=256))
