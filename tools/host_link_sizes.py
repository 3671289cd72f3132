#!/usr/bin/env python3
"""The host-link test's rate at 256 / 64 / 32 MiB per copy, interleaved, five rounds (is a smaller pinned buffer the same
measurement?)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402
rows = {}
for r in range(5):
    for mib in (256, 64, 32):
        res = diag.host_link(0, mib=mib)
        rows.setdefault(mib, []).append((res["rates"]["h2d_gbps"], res["rates"]["d2h_gbps"]))
for mib, v in rows.items():
    print(json.dumps({"mib": mib, "h2d_median": round(statistics.median(x[0] for x in v), 2),
                      "d2h_median": round(statistics.median(x[1] for x in v), 2), "runs": v}))
