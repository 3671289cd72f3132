#!/usr/bin/env python3
"""The watcher (``check-gpu-node --watch``, ``kube/watch.NodeWatcher``) at fleet scale: a mock apiserver process with
N realistic MI355X nodes (8 GPUs each, gzip report annotations, AMDGPUHealthy conditions), the watcher on a thread
here, and a second process PATCHing node status as the agents do -- heartbeats at ``--rate`` per second for
``--seconds``, then one node's Ready flipped to False.  Reports the initial LIST-to-first-report time, the events the
watcher consumed per second, how many reports it emitted (it reports only outcome changes), how long the flip took
to show in a report, and this process's CPU time per event.  One JSON line.

    python tools/watch_scale.py --nodes 5000 --rate 200 --seconds 10
"""
import argparse
import json
import multiprocessing
import os
import resource
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def patcher(url: str, names: list, rate: float, seconds: float, flip: str, out) -> None:
    """Agent-like status PATCHes (the AMDGPUHealthy heartbeat) at ``rate``/s, then ``flip`` goes NotReady."""
    from k8s_gpu_node_checker_amd.kube.client import KubeClient
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    from k8s_gpu_node_checker_amd.models import health as H
    cl = ClusterConnection(url)
    sent = 0
    t0 = time.monotonic()
    with KubeClient(cl) as kc:
        while time.monotonic() - t0 < seconds:
            name = names[sent % len(names)]
            cond = {"type": H.HEALTH_CONDITION, "status": "True", "reason": "MI355XHealthy",
                    "message": "8/8 MI355X GPUs healthy", "lastHeartbeatTime": H.format_k8s_time(time.time()),
                    "lastTransitionTime": "2026-01-01T00:00:00Z"}
            kc.request("PATCH", f"/api/v1/nodes/{name}/status", body=json.dumps(
                {"status": {"conditions": [cond]}}).encode(), content_type="application/strategic-merge-patch+json")
            sent += 1
            behind = sent / rate - (time.monotonic() - t0)
            if behind > 0:
                time.sleep(behind)
        t_flip = time.time()
        ready = {"type": "Ready", "status": "False", "reason": "KubeletNotReady", "message": "flip",
                 "lastHeartbeatTime": H.format_k8s_time(time.time()), "lastTransitionTime": H.format_k8s_time(time.time())}
        kc.request("PATCH", f"/api/v1/nodes/{flip}/status", body=json.dumps(
            {"status": {"conditions": [ready]}}).encode(), content_type="application/strategic-merge-patch+json")
    out.put({"sent": sent, "t_flip": t_flip, "patch_s": round(time.monotonic() - t0, 2)})


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--rate", type=float, default=200.0, help="status PATCHes per second")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--debounce", type=float, default=0.2)
    args = ap.parse_args()

    from k8s_gpu_node_checker_amd.checker import CheckOptions, CheckResult, apply_health
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    from k8s_gpu_node_checker_amd.kube.watch import NodeWatcher
    from k8s_gpu_node_checker_amd.utils.timing import NullTracer

    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    srv = subprocess.Popen([sys.executable, "-m", "k8s_gpu_node_checker_amd.testing.mock_apiserver", "--nodes",
                            str(args.nodes), "--kind", "amd", "--gpus-per-node", "8", "--with-health",
                            "--annotation-encoding", "gzip"], stdout=subprocess.PIPE, text=True, env=env)
    try:
        url = json.loads(srv.stdout.readline())["url"]
        opts = CheckOptions(json=True)
        reports = []

        def evaluate(scan):
            return CheckResult(scan, apply_health(scan, opts, NullTracer()), NullTracer())

        def report(result):
            reports.append((time.time(), len(result.ready_gpu_nodes)))

        w = NodeWatcher(ClusterConnection(url), opts, watch_timeout=300, debounce=args.debounce)
        stop = threading.Event()
        t_start = time.time()
        cpu0 = resource.getrusage(resource.RUSAGE_SELF)
        th = threading.Thread(target=lambda: w.run(evaluate, report, should_stop=stop.is_set), daemon=True)
        th.start()
        while not reports and time.time() - t_start < 120:
            time.sleep(0.01)
        first_report_s = time.time() - t_start
        ready0 = reports[0][1] if reports else None
        names = [f"mi355x-node-{i:04d}" for i in range(1, args.nodes)]
        q = multiprocessing.get_context("spawn").Queue()
        p = multiprocessing.get_context("spawn").Process(
            target=patcher, args=(url, names, args.rate, args.seconds, "mi355x-node-0000", q))
        ev0 = w.events
        t_events = time.time()
        p.start()
        info = q.get(timeout=args.seconds + 120)
        p.join(30)
        deadline = time.time() + 30
        while time.time() < deadline and not (reports and reports[-1][1] == (ready0 or 0) - 1):
            time.sleep(0.005)
        flip_seen = next((t for t, n in reports if n == (ready0 or 0) - 1), None)
        events = w.events - ev0
        span = time.time() - t_events
        stop.set()
        th.join(10)
        cpu1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu_s = (cpu1.ru_utime - cpu0.ru_utime) + (cpu1.ru_stime - cpu0.ru_stime)
        out = {"nodes": args.nodes, "gpus_per_node": 8, "first_report_s": round(first_report_s, 3),
               "ready_at_start": ready0, "patches_sent": info["sent"], "patch_rate_per_s": round(info["sent"] / info["patch_s"], 1),
               "events_consumed": events, "events_per_s": round(events / span, 1),
               "reports": len(reports), "flip_to_report_ms": round((flip_seen - info["t_flip"]) * 1e3, 1) if flip_seen else None,
               "watcher_cpu_s": round(cpu_s, 2), "cpu_ms_per_event": round(cpu_s * 1e3 / max(events, 1), 3),
               "maxrss_mib": round(cpu1.ru_maxrss / 1024, 1), "relists": w.relists, "debounce_s": args.debounce}
        print(json.dumps(out), flush=True)
        return 0 if flip_seen else 1
    finally:
        srv.terminate()
        srv.wait(10)


if __name__ == "__main__":
    sys.exit(main())
