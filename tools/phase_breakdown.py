#!/usr/bin/env python3
"""Per-phase latency distribution of one check against the mock apiserver (list / parse / health / render).

Also times a raw paginated GET that reads the bodies without parsing them, so the server's share
of ``list`` is visible.  Prints one JSON object with p50/p90/p99 per phase.

    python tools/phase_breakdown.py --nodes 1000 --steps 100
"""

from __future__ import annotations

import argparse
import io
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(round(q * (len(xs) - 1))))], 3) if xs else None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--page-size", type=int, default=500)
    ap.add_argument("--kind", default="amd", help="amd | nvidia | mixed | cpu (mock_apiserver --kind)")
    ap.add_argument("--gpus-per-node", type=int, default=1)
    ap.add_argument("--no-health", action="store_true", help="serve nodes without MI355X health data")
    args = ap.parse_args()

    from k8s_gpu_node_checker_amd.checker import CheckOptions, check_and_report
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    from k8s_gpu_node_checker_amd.utils.http import Connection
    from k8s_gpu_node_checker_amd.utils.timing import Tracer

    env = dict(os.environ, PYTHONPATH=REPO)
    srv = subprocess.Popen([sys.executable, "-m", "k8s_gpu_node_checker_amd.testing.mock_apiserver", "--nodes",
                            str(args.nodes), "--kind", args.kind, "--gpus-per-node", str(args.gpus_per_node)]
                           + ([] if args.no_health else ["--with-health"]),
                           stdout=subprocess.PIPE, text=True, env=env)
    try:
        info = json.loads(srv.stdout.readline())
        cluster = ClusterConnection(server=info["url"])
        opts = CheckOptions(json=True, page_size=args.page_size, health_policy="auto")
        phases: dict = {}
        for i in range(args.warmup + args.steps):
            tr = Tracer()
            check_and_report(cluster, opts, out=io.StringIO(), err=io.StringIO(), tracer=tr)
            tr.finish()
            if i >= args.warmup:
                for k, v in tr.as_ms().items():
                    phases.setdefault(k, []).append(v)
        raw = []
        nbytes = 0
        for i in range(args.warmup + args.steps):
            t = time.perf_counter()
            conn = Connection(info["url"])
            cont, nbytes = None, 0
            while True:
                path = f"/api/v1/nodes?limit={args.page_size}" + (f"&continue={cont}" if cont else "")
                resp = conn.request("GET", path, {"Accept": "application/json"})
                nbytes += len(resp.body)
                meta = resp.body[:300]
                j = meta.find(b'"continue":"')
                cont = meta[j + 12:meta.index(b'"', j + 12)].decode() if j >= 0 else None
                if not cont:
                    break
            conn.close()
            if i >= args.warmup:
                raw.append((time.perf_counter() - t) * 1e3)
        phases["raw_get"] = raw
        out = {k: {"p50": _pct(v, .5), "p90": _pct(v, .9), "p99": _pct(v, .99), "min": round(min(v), 3)}
               for k, v in phases.items()}
        print(json.dumps({"nodes": args.nodes, "steps": args.steps, "bytes": nbytes, "phases_ms": out,
                          "cpus": len(os.sched_getaffinity(0))}))
    finally:
        srv.terminate()
        srv.wait(timeout=5)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
