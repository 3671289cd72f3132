#!/usr/bin/env python3
"""Check latency of the report-reading modes at fleet scale: default (condition path), --json-extended
(fleet view: every report annotation parsed), --health-reeval (every report re-judged), both; 8-GPU nodes
with gzip report annotations against the in-process mock apiserver.  Min and median of interleaved runs.

    python tools/extended_modes.py --nodes 1000 --runs 10 --out profiles/extended_modes_cpu.json
"""
import argparse
import io
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.checker import CheckOptions, check_and_report  # noqa: E402
from k8s_gpu_node_checker_amd.kube.config import ClusterConnection  # noqa: E402
from k8s_gpu_node_checker_amd.testing import fixtures  # noqa: E402
from k8s_gpu_node_checker_amd.testing.mock_apiserver import MockApiServer  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    srv = MockApiServer(fixtures.cluster(args.nodes, "amd", gpus_per_node=8, with_health=True,
                                         annotation_encoding="gzip"), "127.0.0.1", 0).start()
    c = ClusterConnection(srv.url)
    modes = {"default": (False, False), "json_extended": (True, False), "health_reeval": (False, True),
             "both": (True, True)}
    ts = {m: [] for m in modes}
    for _ in range(args.runs + 1):
        for m, (ext, reeval) in modes.items():
            opts = CheckOptions(json=True, json_extended=ext)
            opts.health_reeval = reeval
            t = time.perf_counter()
            check_and_report(c, opts, out=io.StringIO(), err=io.StringIO())
            ts[m].append((time.perf_counter() - t) * 1e3)
    out = {"nodes": args.nodes, "gpus_per_node": 8, "runs": args.runs, "cpus": len(os.sched_getaffinity(0)),
           "ms": {m: {"min": round(min(v[1:]), 1), "median": round(statistics.median(v[1:]), 1)} for m, v in ts.items()}}
    print(json.dumps(out))
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)
    srv.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
