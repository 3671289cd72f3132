#!/usr/bin/env python3
"""Scaling curve on one machine: this checker vs the unmodified reference, same mock apiserver.

For each cluster size N the mock kube-apiserver runs in its own process; both
programs are timed *in-process* per check (the survey's `one_shot` method,
SURVEY §4.3 item 5), median of `--reps`:

* ours: `checker.check_and_report(... --json ...)`
* reference: `one_shot(args)` of `/root/reference/check-gpu-node.py` imported with
  the test stand-ins for `kubernetes`/`dotenv` (tests/refstub) -- lighter than the
  real client, so the reference numbers are a lower bound.

Writes a JSON summary (default `profiles/scaling_cpu.json`).

``--pin S,C`` pins the mock server to CPU S and both measured programs to CPU C.  Unpinned, the
server's per-connection thread and the client migrate between cores and the 1-16 node numbers are
dominated by wake-up latency (ours: 0.43 ms unpinned vs 0.23 ms pinned at 1 node on an 8-vCPU VM);
pinning both sides the same way keeps the comparison fair.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/check-gpu-node.py"

REF_TIMER = r'''
import argparse, importlib.util, io, json, statistics, sys, time, contextlib
sys.path.insert(0, {stubs!r})
spec = importlib.util.spec_from_file_location("refcheck", {ref!r})
m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
from kubernetes import config
config.load_kube_config({kc!r})
args = argparse.Namespace(json=True, slack_webhook=None, slack_username="k8s-gpu-checker", slack_only_on_error=False,
                          slack_retry_count=3, slack_retry_delay=30, kubeconfig={kc!r})
ts = []
for i in range({reps} + {warm}):
    buf = io.StringIO()
    t = time.perf_counter()
    with contextlib.redirect_stdout(buf):
        m.one_shot(args)
    if i >= {warm}:
        ts.append(time.perf_counter() - t)
print(json.dumps({{"median_ms": statistics.median(ts) * 1e3}}))
'''


def ours(url, reps, warm, page_size):
    sys.path.insert(0, REPO)
    import io
    from k8s_gpu_node_checker_amd.checker import CheckOptions, check_and_report
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    cl = ClusterConnection(url)
    opts = CheckOptions(json=True, page_size=page_size)
    ts = []
    for i in range(reps + warm):
        t = time.perf_counter()
        check_and_report(cl, opts, out=io.StringIO())
        if i >= warm:
            ts.append(time.perf_counter() - t)
    return statistics.median(ts) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,2,4,8,16,1000,5000")
    ap.add_argument("--reps", type=int, default=51)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "scaling_cpu.json"))
    ap.add_argument("--pin", help="SERVER_CPU,CLIENT_CPU: pin the mock server and both clients")
    args = ap.parse_args()
    pin = [int(x) for x in args.pin.split(",")] if args.pin else None
    if pin:
        os.sched_setaffinity(0, {pin[1]})
    rows = []
    for n in [int(x) for x in args.sizes.split(",")]:
        kind = "mixed" if n >= 1000 else "amd"
        env = dict(os.environ, PYTHONPATH=REPO)
        srv = subprocess.Popen([sys.executable, "-m", "k8s_gpu_node_checker_amd.testing.mock_apiserver", "--nodes",
                                str(n), "--kind", kind], stdout=subprocess.PIPE, text=True, env=env)
        if pin:
            os.sched_setaffinity(srv.pid, {pin[0]})
        try:
            url = json.loads(srv.stdout.readline())["url"]
            kc = f"/tmp/scaling-kc-{n}.yaml"
            sys.path.insert(0, REPO)
            from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
            write_kubeconfig(kc, url)
            reps = args.reps if n < 1000 else max(7, args.reps // 5)
            row = {"nodes": n, "ours_ms": round(ours(url, reps, 20, 500), 3),
                   "ours_unpaginated_ms": round(ours(url, reps, 20, 0), 3) if n >= 1000 else None}
            if os.path.exists(REF):
                code = REF_TIMER.format(stubs=os.path.join(REPO, "tests", "refstub"), ref=REF, kc=kc, reps=reps,
                                        warm=20)
                p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=900,
                                   preexec_fn=(lambda: os.sched_setaffinity(0, {pin[1]})) if pin else None)
                row["reference_ms"] = round(json.loads(p.stdout.strip().splitlines()[-1])["median_ms"], 3) \
                    if p.returncode == 0 else None
                if row["reference_ms"]:
                    row["speedup"] = round(row["reference_ms"] / row["ours_ms"], 2)
            row["ours_nodes_per_s"] = round(n / (row["ours_ms"] / 1e3), 1)
            rows.append(row)
            print(json.dumps(row), flush=True)
        finally:
            srv.terminate()
            srv.wait(timeout=10)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"host": os.uname().nodename, "cpus": os.cpu_count(), "method": "in-process median per check",
                   "pinned": args.pin, "rows": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
