#!/usr/bin/env python3
"""The five BASELINE.json configs, this checker vs the unmodified reference, same machine.

For each config one mock kube-apiserver (and, where the config has Slack, one webhook sink) runs in
its own process; both programs are timed in-process per check (the survey's ``one_shot`` method,
SURVEY §4.3), median of ``--reps``, and their stdout / exit code of one run are compared byte for
byte.  The reference is imported with the test stand-ins for ``kubernetes`` / ``dotenv``
(tests/refstub: lighter than the real client, so its numbers are a lower bound).

  1  1 node, amd.com/gpu:1, --json, no Slack
  2  8 nodes, all Ready, amd.com/gpu:8 each, Slack to a local 200 sink
  3  8 nodes, 2 NotReady, --slack-only-on-error (6 Ready: no Slack)
  4  16 CPU-only nodes (exit 2), Slack against a forced-500 sink: the reference retries at once;
     ours is timed with --slack-retry-policy reference (same schedule) and with the default
     backoff policy (PARITY #2: sleeps between attempts, by design)
  5  1000 nodes, mixed amd.com/gpu / nvidia.com/gpu, --json

    python tools/baseline_configs.py [--reps 51] [--pin 2,5] [--out profiles/baseline_configs_cpu.json]
"""

from __future__ import annotations

import argparse
import io
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/check-gpu-node.py"
sys.path.insert(0, REPO)

CONFIGS = [
    {"id": 1, "nodes": 1, "kind": "amd", "gpus": 1, "not_ready": 0, "json": True, "slack": None},
    {"id": 2, "nodes": 8, "kind": "amd", "gpus": 8, "not_ready": 0, "json": False, "slack": "200"},
    {"id": 3, "nodes": 8, "kind": "amd", "gpus": 8, "not_ready": 2, "json": False, "slack": "200",
     "only_on_error": True},
    {"id": 4, "nodes": 16, "kind": "cpu", "gpus": 0, "not_ready": 0, "json": False, "slack": "500",
     "retry_delay": 0},
    {"id": 5, "nodes": 1000, "kind": "mixed", "gpus": 8, "not_ready": 0, "json": True, "slack": None},
]

REF_RUNNER = r'''
import argparse, contextlib, importlib.util, io, json, statistics, sys, time
sys.path.insert(0, {stubs!r})
spec = importlib.util.spec_from_file_location("refcheck", {ref!r})
m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
from kubernetes import config
config.load_kube_config({kc!r})
args = argparse.Namespace(json={json_mode!r}, slack_webhook={slack!r}, slack_username="k8s-gpu-checker",
                          slack_only_on_error={only!r}, slack_retry_count=3, slack_retry_delay={delay!r},
                          kubeconfig={kc!r})
def once():
    out, err = io.StringIO(), io.StringIO()
    with contextlib.redirect_stdout(out), contextlib.redirect_stderr(err):
        code = m.one_shot(args)
    return code, out.getvalue()
code, first = once()
ts = []
for i in range({reps} + {warm}):
    t = time.perf_counter()
    once()
    if i >= {warm}:
        ts.append(time.perf_counter() - t)
print(json.dumps({{"median_ms": statistics.median(ts) * 1e3, "exit": code, "stdout": first}}))
'''


def ours(url: str, cfg: dict, reps: int, warm: int, policy: str):
    from k8s_gpu_node_checker_amd.checker import CheckOptions, check_and_report
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    cl = ClusterConnection(url)
    opts = CheckOptions(json=cfg["json"], slack_webhook=cfg.get("webhook"),
                        slack_only_on_error=cfg.get("only_on_error", False),
                        slack_retry_delay=cfg.get("retry_delay", 30), slack_retry_policy=policy)

    def once():
        out, err = io.StringIO(), io.StringIO()
        res = check_and_report(cl, opts, out=out, err=err)
        return res.exit_code, out.getvalue()
    code, first = once()
    ts = []
    for i in range(reps + warm):
        t = time.perf_counter()
        once()
        if i >= warm:
            ts.append(time.perf_counter() - t)
    return statistics.median(ts) * 1e3, code, first


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=51)
    ap.add_argument("--pin", help="SERVER_CPU,CLIENT_CPU")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "baseline_configs_cpu.json"))
    args = ap.parse_args()
    pin = [int(x) for x in args.pin.split(",")] if args.pin else None
    if pin:
        os.sched_setaffinity(0, {pin[1]})
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    env = dict(os.environ, PYTHONPATH=REPO)
    rows = []
    for cfg in CONFIGS:
        procs = []
        try:
            srv = subprocess.Popen([sys.executable, "-m", "k8s_gpu_node_checker_amd.testing.mock_apiserver",
                                    "--nodes", str(cfg["nodes"]), "--kind", cfg["kind"], "--gpus-per-node",
                                    str(max(1, cfg["gpus"])), "--not-ready", str(cfg["not_ready"])],
                                   stdout=subprocess.PIPE, text=True, env=env)
            procs.append(srv)
            url = json.loads(srv.stdout.readline())["url"]
            if pin:
                os.sched_setaffinity(srv.pid, {pin[0]})
            cfg = dict(cfg)
            if cfg["slack"]:
                sink = subprocess.Popen([sys.executable, "-m", "k8s_gpu_node_checker_amd.testing.webhook_sink"],
                                        stdout=subprocess.PIPE, text=True, env=env)
                procs.append(sink)
                cfg["webhook"] = json.loads(sink.stdout.readline())["url"] + "/" + cfg["slack"]
                if pin:
                    os.sched_setaffinity(sink.pid, {pin[0]})
            kc = f"/tmp/baseline-kc-{cfg['id']}.yaml"
            write_kubeconfig(kc, url)
            reps = args.reps if cfg["nodes"] < 1000 else max(7, args.reps // 5)
            if cfg["slack"] == "500":
                reps = max(5, reps // 5)
            row = {"config": cfg["id"], "nodes": cfg["nodes"], "kind": cfg["kind"], "slack": cfg["slack"]}
            ms, code, out = ours(url, cfg, reps, 5, "reference")
            row.update(ours_ms=round(ms, 3), ours_exit=code)
            if cfg["slack"] == "500":
                ms_b, _, _ = ours(url, cfg, 3, 0, "backoff")
                row["ours_backoff_policy_ms"] = round(ms_b, 1)
            if os.path.exists(REF):
                code_s = REF_RUNNER.format(stubs=os.path.join(REPO, "tests", "refstub"), ref=REF, kc=kc,
                                           json_mode=cfg["json"], slack=cfg.get("webhook"),
                                           only=cfg.get("only_on_error", False), delay=cfg.get("retry_delay", 30),
                                           reps=reps, warm=5)
                p = subprocess.run([sys.executable, "-c", code_s], capture_output=True, text=True, timeout=1800,
                                   preexec_fn=(lambda: os.sched_setaffinity(0, {pin[1]})) if pin else None)
                if p.returncode == 0:
                    ref = json.loads(p.stdout.strip().splitlines()[-1])
                    row.update(reference_ms=round(ref["median_ms"], 3), reference_exit=ref["exit"],
                               speedup=round(ref["median_ms"] / ms, 2), stdout_identical=ref["stdout"] == out,
                               exit_identical=ref["exit"] == code)
                else:
                    row["reference_error"] = p.stderr[-500:]
            rows.append(row)
            print(json.dumps(row), flush=True)
        finally:
            for p_ in procs:
                p_.terminate()
                p_.wait(timeout=10)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"host": os.uname().nodename, "cpus": os.cpu_count(), "pinned": args.pin,
                   "method": "in-process median per check; stdout/exit of one run compared", "rows": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
