#!/usr/bin/env python3
"""Spread of the MFMA burn-in's per-XCD wave time on a healthy MI355X (calibrates diag.XCD_SLOW_RATIO).

    python tools/xcd_map.py --rounds 20 > profiles/mfma_xcd_map_mi355x.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    from k8s_gpu_node_checker_amd.ops import diag
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args()
    rounds = []
    for i in range(args.rounds):
        r = diag.mfma_burn(args.device)
        m = r["map"]
        rounds.append({"round": i, "cus": m["cus"], "slowest_xcd": m.get("slowest_xcd"),
                       "slowest_rel": m.get("slowest_rel"), "slowest_cu": m.get("slowest_cu"),
                       "slowest_cu_rel": m.get("slowest_cu_rel"), "waves_per_cu": m.get("waves_per_cu"),
                       "rel_time": {x: v["rel_time"] for x, v in m["xcds"].items()},
                       "cus_per_xcd": {x: v["cus"] for x, v in m["xcds"].items()},
                       "tflops": {k: v["tflops"] for k, v in r["kinds"].items()}, "errors": sum(
                           v["errors"] for v in r["kinds"].values())})
        print(json.dumps(rounds[-1]), file=sys.stderr, flush=True)
    rel = sorted(x["slowest_rel"] for x in rounds if x["slowest_rel"] is not None)
    cu_rel = sorted(x["slowest_cu_rel"] for x in rounds if x["slowest_cu_rel"] is not None)
    l2 = [diag.l2_bandwidth(args.device)["map"] for _ in range(10)]
    print(json.dumps({"device": diag.device_info(args.device), "rounds": rounds,
                      "slowest_cu_rel": {"min": cu_rel[0], "median": cu_rel[len(cu_rel) // 2], "max": cu_rel[-1]}
                      if cu_rel else None,
                      "l2_slowest_cu_rel": [m.get("slowest_cu_rel") for m in l2],
                      "l2_waves_per_cu": [m.get("waves_per_cu") for m in l2],
                      "slowest_rel": {"min": rel[0], "median": rel[len(rel) // 2], "max": rel[-1]} if rel else None,
                      "xcd_slow_ratio": diag.XCD_SLOW_RATIO}, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
