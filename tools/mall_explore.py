#!/usr/bin/env python3
"""Per-XCD streaming reads (``diag.hbm_xcd``) over slice sizes from L2-sized to far past the 256 MiB MALL:
where the read rate steps down from MALL to HBM, all XCDs together and each alone.

    python tools/mall_explore.py --out gpurun_out/mall_explore.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/mall_explore.json")
    args = ap.parse_args()
    out = []
    for mib, passes in ((4, 32), (8, 32), (16, 16), (24, 16), (32, 8), (64, 4), (128, 2), (256, 2)):
        rs = [diag.hbm_xcd(0, mib, passes) for _ in range(3)]
        row = {"slice_mib": mib, "total_mib": 8 * mib, "passes": passes, "together_tbs": [r["read_tbs"] for r in rs],
               "alone_min_tbs": [min(r["alone_tbs"].values()) for r in rs],
               "alone_max_tbs": [max(r["alone_tbs"].values()) for r in rs], "errors": sum(r["errors"] for r in rs)}
        out.append(row)
        print(json.dumps(row), flush=True)
    json.dump(out, open(args.out, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
