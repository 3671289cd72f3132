#!/usr/bin/env python3
"""Sweep the per-XCD HBM read test (``diag.hbm_xcd``) over slice size, passes and workgroups per CU, and
repeat the default a few times: the aggregate TB/s and the XCD spread a healthy MI355X shows.

    python tools/hbm_xcd_explore.py --out gpurun_out/hbm_xcd_explore.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/hbm_xcd_explore.json")
    args = ap.parse_args()
    rows = []
    for slice_mib, passes, bpc in ((64, 4, 4), (128, 2, 4), (256, 1, 4), (256, 2, 2), (256, 2, 4), (256, 2, 8),
                                   (512, 1, 4), (512, 2, 4)):
        r = diag.hbm_xcd(0, slice_mib, passes, bpc)
        m = r["map"]
        row = {"slice_mib": slice_mib, "passes": passes, "blocks_per_cu": bpc, "read_tbs": r["read_tbs"],
               "errors": r["errors"], "wall_s": r["wall_s"], "slowest_xcd": r.get("slowest_xcd"),
               "slowest_xcd_rel": r.get("slowest_xcd_rel"), "alone_tbs": r.get("alone_tbs"),
               # wave time per XCD while all stream together (the contended shares, reported only)
               "together_rel_time": {k: v["rel_time"] for k, v in m.get("xcds", {}).items()}}
        rows.append(row)
        print(json.dumps(row), flush=True)
    reps = []
    for _ in range(20):
        r = diag.hbm_xcd(0)
        reps.append({"read_tbs": r["read_tbs"], "errors": r["errors"], "alone_tbs": r.get("alone_tbs"),
                     "slowest_xcd_rel": r.get("slowest_xcd_rel"), "pass": r["pass"], "degraded": r["degraded"],
                     "together_rel_time": {k: v["rel_time"] for k, v in r["map"].get("xcds", {}).items()}})
    print(json.dumps({"repeat_default": reps}), flush=True)
    hbm = diag.hbm(0)
    json.dump({"sweep": rows, "repeat_default": reps, "hbm_stream": hbm}, open(args.out, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
