#!/usr/bin/env python3
"""Peak RSS of the isolated agent's diagnostic children from the first cycle on: ``--level`` cycles of the agent with
process isolation, one JSON line per cycle with the child's peak (the first cycle on a fresh box is the largest:
what the DaemonSet's memory limit must hold).

    python tools/first_child_rss.py --level 2 --cycles 3
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--level", type=int, default=1, choices=(1, 2))
    ap.add_argument("--cycles", type=int, default=3)
    args = ap.parse_args()
    from k8s_gpu_node_checker_amd.agent.agent import Agent
    ag = Agent("gpu-node", source="native", diag_level=args.level, devices=[0], diag_when="always",
               diag_interval=0.0, isolation="process")
    for i in range(args.cycles):
        rep = ag.probe_once()
        g = rep["gpus"][0]
        print(json.dumps({"level": args.level, "cycle": i, "peak_rss_mib": (g.get("diag_proc") or {}).get("peak_rss_mib"),
                          "state": rep.get("state"), "skipped": g.get("diag_skipped")}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
