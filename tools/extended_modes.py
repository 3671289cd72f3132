#!/usr/bin/env python3
"""Check latency of the report-reading modes at fleet scale: default (condition path), --json-extended
(fleet view: every report annotation parsed), --health-reeval (every report re-judged), both; 8-GPU nodes
with gzip report annotations against the in-process mock apiserver.  Min and median of interleaved runs.

    python tools/extended_modes.py --nodes 1000 --runs 10 --out profiles/extended_modes_cpu.json
    python tools/extended_modes.py --with-diag ...   # reports carry level-1 diagnostics: the fleet judgement runs

``--with-diag`` builds each node's report with a node agent's level-1 cycle on the fake C ABI
(``testing/fake_native.py``), every node a little different, so the reports are the size the DaemonSet writes and
``models/fleet.py`` has rates to compare.
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


def _diag_cluster(n: int) -> list:
    """``n`` 8-GPU nodes whose gzip report annotations and conditions come from agent cycles with level-1
    diagnostics on the fake ABI (one cycle per distinct rate, reused with the node's name)."""
    import copy
    from k8s_gpu_node_checker_amd.agent import agent as A
    from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag, fabric
    from k8s_gpu_node_checker_amd.testing.fake_native import FakeDiagLib, FakeFabricLib
    fabric._lib = FakeFabricLib()
    amdsmi_probe.probe = lambda nd, src, fx: fixtures.mi355x_probe_report(nd, gpus=8)
    base = {}
    for rate in (0.96, 0.98, 1.0, 1.02):
        lib = FakeDiagLib(n=8, rate=rate)
        diag.lib = lambda lib=lib: lib
        base[rate] = A.Agent("n", source="fake", diag_level=1, expect_gpus=8, diag_timeout=60,
                             diag_baseline=False).probe_once()
    nodes = []
    for i in range(n):
        rep = copy.deepcopy(base[(0.96, 0.98, 1.0, 1.02)[i % 4]])
        rep["node"] = f"mi355x-node-{i:04d}"
        nodes.append(fixtures.realistic_node(rep["node"], "amd.com/gpu", 8, index=i,
                                             annotations=fixtures.health_annotation(rep, "gzip"),
                                             extra_conditions=[fixtures.health_condition(rep, 8)]))
    return nodes


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--out", default="")
    ap.add_argument("--with-diag", action="store_true")
    args = ap.parse_args()
    nodes = (_diag_cluster(args.nodes) if args.with_diag else
             fixtures.cluster(args.nodes, "amd", gpus_per_node=8, with_health=True, annotation_encoding="gzip"))
    srv = MockApiServer(nodes, "127.0.0.1", 0).start()
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
           "reports": "level-1 diagnostics (fake ABI)" if args.with_diag else "probe only",
           "ms": {m: {"min": round(min(v[1:]), 1), "median": round(statistics.median(v[1:]), 1)} for m, v in ts.items()}}
    print(json.dumps(out))
    if args.out:
        json.dump(out, open(args.out, "w"), indent=1)
    srv.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
