#!/usr/bin/env python3
"""Driver for counter passes over the per-XCD HBM test (``tools/gpu_pmc_hbm_xcd.sh``): three runs."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402

print(json.dumps([{k: r.get(k) for k in ("read_tbs", "alone_tbs", "errors")} for r in (diag.hbm_xcd(0) for _ in range(3))]))
