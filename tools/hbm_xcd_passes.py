#!/usr/bin/env python3
"""Spread of the per-XCD HBM test at 2 and 4 passes (30 runs each): how much averaging the lone-XCD rates need.

    python tools/hbm_xcd_passes.py --out gpurun_out/hbm_xcd_passes.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default="gpurun_out/hbm_xcd_passes.json")
args = ap.parse_args()
out = {}
for p in (2, 4):
    rs = [diag.hbm_xcd(0, 256, p) for _ in range(30)]
    out[p] = {"together_tbs": [r["read_tbs"] for r in rs], "slowest_xcd_rel": [r["slowest_xcd_rel"] for r in rs],
              "alone_min_tbs": [min(r["alone_tbs"].values()) for r in rs], "wall_s": [r["wall_s"] for r in rs]}
    v = out[p]
    print(p, "rel min", min(v["slowest_xcd_rel"]), "alone min", min(v["alone_min_tbs"]), "together min",
          min(v["together_tbs"]), "wall median", sorted(v["wall_s"])[15], flush=True)
json.dump(out, open(args.out, "w"), indent=1)
