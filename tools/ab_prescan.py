#!/usr/bin/env python3
"""A/B of the page reader's pass-1 prescan: full ``check --json`` cycles against the mock apiserver,
with and without the prescan, interleaved in one process (rounds alternate, so drift hits both).

    python tools/ab_prescan.py --nodes 1000 --rounds 60
"""

from __future__ import annotations

import argparse
import gc
import io
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--rounds", type=int, default=60)
    ap.add_argument("--page-size", type=int, default=500)
    args = ap.parse_args()

    from k8s_gpu_node_checker_amd.checker import CheckOptions, check_and_report
    from k8s_gpu_node_checker_amd.kube import client as C
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection

    srv = subprocess.Popen([sys.executable, "-m", "k8s_gpu_node_checker_amd.testing.mock_apiserver", "--nodes",
                            str(args.nodes), "--kind", "mixed", "--with-health"],
                           stdout=subprocess.PIPE, text=True, env=dict(os.environ, PYTHONPATH=REPO))
    with_pre = C._PageReader

    class NoPrescan(with_pre):
        def __init__(self, conn, path, keys=None):
            super().__init__(conn, path, None)

    try:
        cluster = ClusterConnection(server=json.loads(srv.stdout.readline())["url"])
        opts = CheckOptions(json=True, page_size=args.page_size, health_policy="auto")
        ms = {"prescan": [], "no_prescan": []}
        for r in range(args.rounds + 5):
            for name, cls in (("prescan", with_pre), ("no_prescan", NoPrescan)):
                C._PageReader = cls
                gc.collect()
                t = time.perf_counter()
                res = check_and_report(cluster, opts, out=io.StringIO(), err=io.StringIO())
                if r >= 5:
                    ms[name].append((time.perf_counter() - t) * 1e3)
                assert res.exit_code == 0
    finally:
        C._PageReader = with_pre
        srv.terminate()
        srv.wait(timeout=5)
    out = {k: {"p50": round(statistics.median(v), 3), "min": round(min(v), 3)} for k, v in ms.items()}
    print(json.dumps({"nodes": args.nodes, "rounds": args.rounds, "page_size": args.page_size, "ms": out}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
