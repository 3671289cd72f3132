#!/usr/bin/env python3
"""Sweep the per-XCD L2 read test (slice size x passes) on an MI355X: aggregate TB/s, XCD spread, errors.

    python tools/l2_explore.py > profiles/l2_explore_mi355x.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    from k8s_gpu_node_checker_amd.ops import diag
    rows = []
    for slice_kib, passes, bpc in ((2048, 16, 1), (2048, 16, 2), (2048, 16, 4), (2048, 16, 8), (1024, 32, 4),
                                   (3072, 16, 4), (2048, 64, 4), (8192, 8, 4)):
            rs = [diag.l2_bandwidth(0, slice_kib, passes, bpc) for _ in range(3)]
            row = {"slice_kib": slice_kib, "passes": passes, "blocks_per_cu": bpc, "read_tbs": [r["read_tbs"] for r in rs],
                   "slowest_rel": [r["map"].get("slowest_rel") for r in rs], "errors": sum(r["errors"] for r in rs),
                   "wall_s": [r["wall_s"] for r in rs], "cus": rs[-1]["map"]["cus"]}
            rows.append(row)
            print(json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps({"device": diag.device_info(0), "rows": rows}, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
