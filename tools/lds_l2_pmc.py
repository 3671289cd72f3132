#!/usr/bin/env python3
"""Driver for hardware-counter passes over the LDS and per-XCD L2 diagnostics (``tools/gpu_pmc_lds_l2.sh``):
runs each test a few times so every counter pass sees the same kernels.

    rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -- python tools/lds_l2_pmc.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402

out = {"lds": [], "l2": []}
for _ in range(3):
    r = diag.lds_test(0)
    out["lds"].append({k: r.get(k) for k in ("pass", "errors", "ms")})
    r = diag.l2_bandwidth(0)
    out["l2"].append({k: r.get(k) for k in ("pass", "errors", "read_tbs")})
print(json.dumps(out))
