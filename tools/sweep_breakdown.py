#!/usr/bin/env python3
"""Where a sweep step's time goes (bench.py --mode sweep: re-probe + re-PATCH inside the step): the native amd-smi
probe alone, the agent's whole probe_once (diagnostics not due), and the publish, ten times each, medians in ms."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.agent.agent import Agent  # noqa: E402
from k8s_gpu_node_checker_amd.kube.client import KubeClient  # noqa: E402
from k8s_gpu_node_checker_amd.kube.config import ClusterConnection  # noqa: E402
from k8s_gpu_node_checker_amd.ops import amdsmi_probe  # noqa: E402
from k8s_gpu_node_checker_amd.testing import fixtures  # noqa: E402
from k8s_gpu_node_checker_amd.testing.mock_apiserver import MockApiServer  # noqa: E402


def timed(fn, n=10):
    fn()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t) * 1e3)
    return round(statistics.median(ts), 2)


out = {"probe_native_ms": timed(lambda: amdsmi_probe.probe_native("n"))}
rep = amdsmi_probe.probe_native("n")
out["probe_ms_field"] = rep.get("probe_ms")
out["procs_field"] = [g.get("procs") for g in rep.get("gpus", [])][:1]
ag = Agent("mi355x-node-0000", source="auto", diag_level=0, annotation_encoding="gzip")
out["probe_once_ms"] = timed(ag.probe_once)
srv = MockApiServer(fixtures.cluster(1, "amd", gpus_per_node=1), "127.0.0.1", 0).start()
try:
    r = ag.probe_once()
    cl = ClusterConnection(srv.url)

    def pub():
        with KubeClient(cl) as kc:
            ag.publish(kc, r, force=True)
    out["publish_ms"] = timed(pub)
finally:
    srv.stop()
print(json.dumps(out))
