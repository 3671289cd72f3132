#!/usr/bin/env python3
"""Soak the node agent as it runs in the DaemonSet: the real agent process (native amd-smi probe, HIP
diagnostics on every probe, gzip annotation, labels, HTTP /probe /metrics /healthz) against a mock
kube-apiserver, for a fixed wall time; then the checker's ``--mi355x`` verdict on the node it wrote.

Every ``--sample`` seconds it records the Node's ``AMDGPUHealthy`` condition (status, heartbeat age),
``/healthz``, the agent's RSS and the VRAM amd-smi reports in use, so a leak, a stalled heartbeat or a
flapping verdict shows as drift.  This process never touches the GPU (the agent is a child process).

    python tools/agent_soak.py --minutes 4 --out gpurun_out/agent_soak.json
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time
import urllib.request

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from k8s_gpu_node_checker_amd.models import health as H  # noqa: E402
from k8s_gpu_node_checker_amd.testing import fixtures  # noqa: E402
from k8s_gpu_node_checker_amd.testing.mock_apiserver import MockApiServer, write_kubeconfig  # noqa: E402


def _baseline_summary(path: str):
    """The baseline file the agent wrote: per GPU its epoch, the tests with a formed baseline and their values."""
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return {"file": None}
    gpus = {}
    for k, v in (doc.get("gpus") or {}).items():
        tests = v.get("tests") or {}
        gpus[k] = {"epoch": v.get("epoch"),
                   "formed": {t: e["baseline"] for t, e in tests.items() if isinstance(e, dict) and "baseline" in e},
                   "forming": sorted(t for t, e in tests.items() if isinstance(e, dict) and "baseline" not in e)}
    return {"schema": doc.get("schema"), "gpus": gpus}


def _rss_mb(pid: int):
    try:
        with open(f"/proc/{pid}/status") as f:
            for line in f:
                if line.startswith("VmRSS:"):
                    return round(int(line.split()[1]) / 1024, 1)
    except OSError:
        return None
    return None


def _proc_counts(pid: int):
    """Open file descriptors and threads of ``pid`` (what a leak per diagnostic child would grow: pipe ends, reader
    threads)."""
    try:
        fds = len(os.listdir(f"/proc/{pid}/fd"))
        with open(f"/proc/{pid}/status") as f:
            threads = next(int(line.split()[1]) for line in f if line.startswith("Threads:"))
        return fds, threads
    except (OSError, StopIteration, ValueError):
        return None, None


def _zombies(pids):
    """How many of ``pids`` are zombies (ended, never reaped)."""
    n = 0
    for p in pids:
        try:
            with open(f"/proc/{p}/stat") as f:
                n += f.read().rsplit(")", 1)[1].split()[0] == "Z"
        except (OSError, IndexError):
            pass
    return n


def _descendant_pids(pid: int):
    """Every descendant of ``pid``, zombies included."""
    kids = {}
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open(f"/proc/{d}/stat") as f:
                ppid = int(f.read().rsplit(")", 1)[1].split()[1])
        except (OSError, ValueError, IndexError):
            continue
        kids.setdefault(ppid, []).append(int(d))
    out, todo = [], list(kids.get(pid, []))
    while todo:
        c = todo.pop()
        out.append(c)
        todo.extend(kids.get(c, []))
    return out


def _descendants(pid: int):
    """RSS (MiB) of every live descendant of ``pid`` (process isolation: the forkserver, and a diagnostic child if
    one is running at the sample), by pid."""
    kids = {}
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open(f"/proc/{d}/stat") as f:
                ppid = int(f.read().rsplit(")", 1)[1].split()[1])
        except (OSError, ValueError, IndexError):
            continue
        kids.setdefault(ppid, []).append(int(d))
    out, todo = {}, list(kids.get(pid, []))
    while todo:
        c = todo.pop()
        out[c] = _rss_mb(c)
        todo.extend(kids.get(c, []))
    return {k: v for k, v in out.items() if v is not None}


def _get(url: str, timeout: float = 5.0):
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.status, r.read()
    except urllib.error.HTTPError as e:
        return e.code, e.read()
    except OSError as e:
        return None, str(e).encode()


def _spread(xs):
    xs = [x for x in xs if isinstance(x, (int, float))]
    return {"min": min(xs), "median": statistics.median(xs), "max": max(xs), "n": len(xs)} if xs else None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=4.0)
    ap.add_argument("--interval", type=float, default=2.0, help="agent --interval (s)")
    ap.add_argument("--diag-level", type=int, default=1, choices=(0, 1, 2))
    ap.add_argument("--diag-interval", type=float, default=0.0, help="agent --diag-interval (0: every probe)")
    ap.add_argument("--sample", type=float, default=10.0)
    ap.add_argument("--port", type=int, default=19464)
    ap.add_argument("--out", default="gpurun_out/agent_soak.json")
    ap.add_argument("--diag-isolation", choices=("process", "thread"), default="process",
                    help="agent --diag-isolation (default process, as deployed)")
    ap.add_argument("--baseline", action="store_true",
                    help="run the agent with --diag-baseline-file, report the baselines it formed (epoch, ratios) "
                         "and drop them at the end through POST /baseline/reset")
    args = ap.parse_args()

    nodes = fixtures.cluster(1, "amd", gpus_per_node=1)
    name = nodes[0]["metadata"]["name"]
    srv = MockApiServer(nodes, "127.0.0.1", 0).start()
    kc = write_kubeconfig(os.path.join(tempfile.mkdtemp(prefix="agent-soak"), "config"), srv.url)
    cmd = [sys.executable, "-m", "k8s_gpu_node_checker_amd.agent.agent", "--node", name, "--source", "native",
           "--interval", str(args.interval), "--diag-level", str(args.diag_level),
           "--diag-interval", str(args.diag_interval), "--publish", "annotation,http",
           "--listen", f"127.0.0.1:{args.port}", "--kubeconfig", kc, "--annotation-encoding", "gzip",
           "--label-node", "--xgmi-links", "0", "--ignore-pid", str(os.getpid()),
           "--diag-isolation", args.diag_isolation]
    baseline_path = os.path.join(os.path.dirname(kc), "baseline.json")
    if args.baseline:
        cmd += ["--diag-baseline-file", baseline_path]
    baseline = None
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    err_path = os.path.join(os.path.dirname(os.path.abspath(args.out)), "agent_soak.stderr")
    os.makedirs(os.path.dirname(err_path), exist_ok=True)
    samples = []
    with open(err_path, "w") as err:
        agent = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=err, env=env)
        t0 = time.monotonic()
        deadline = t0 + args.minutes * 60
        try:
            while time.monotonic() < deadline and agent.poll() is None:
                time.sleep(args.sample)
                with srv.state.lock:
                    node = json.loads(json.dumps(next(n for n in srv.state.nodes if n["metadata"]["name"] == name)))
                cond = next((c for c in (node.get("status") or {}).get("conditions") or []
                             if c.get("type") == H.HEALTH_CONDITION), None)
                hb = H.parse_k8s_time(cond.get("lastHeartbeatTime")) if cond else None
                hz, _ = _get(f"http://127.0.0.1:{args.port}/healthz")
                kids = _descendants(agent.pid)
                fds, threads = _proc_counts(agent.pid)
                pc, body = _get(f"http://127.0.0.1:{args.port}/probe")
                rep = json.loads(body) if pc == 200 else {}
                g = (rep.get("gpus") or [{}])[0]
                diag = g.get("diag") or {}
                s = {"t": round(time.monotonic() - t0, 1), "condition": cond and cond.get("status"),
                     "reason": cond and cond.get("reason"),
                     "heartbeat_age_s": round(time.time() - hb, 1) if hb else None, "healthz": hz,
                     "state": rep.get("state"), "agent_rss_mb": _rss_mb(agent.pid),
                     # process isolation: the forkserver (and a child caught mid-diagnostic), and the peak RSS of the
                     # child that produced the last result (its own getrusage, reported over the pipe)
                     "children_rss_mb": kids,
                     "zombies": _zombies(_descendant_pids(agent.pid)),
                     "agent_fds": fds, "agent_threads": threads,
                     "diag_child_peak_mb": (g.get("diag_proc") or {}).get("peak_rss_mib"),
                     "diag_child_pid": (g.get("diag_proc") or {}).get("pid"),
                     "vram_used_mb": g.get("vram_used_mb"), "diag_pass": {k: v.get("pass") for k, v in diag.items()
                                                                          if isinstance(v, dict)},
                     # what a not-healthy sample was about: each failed or degraded test's fraction, rates, detail
                     "diag_notes": {k: {"pass": v.get("pass"), "degraded": v.get("degraded"),
                                        "fraction": v.get("fraction"), "rates": v.get("rates"),
                                        "detail": (v.get("detail") or "")[:160]}
                                    for k, v in diag.items() if isinstance(v, dict)
                                    and (v.get("pass") is False or v.get("degraded"))},
                     "reasons": (rep.get("reasons") or [])[:4], "warnings": (rep.get("warnings") or [])[:4],
                     "labels": {k: v for k, v in (node["metadata"].get("labels") or {}).items()
                                if k.startswith("amd.com/")}}
                samples.append(s)
                print(json.dumps(s), flush=True)
            if args.baseline and agent.poll() is None:
                baseline = _baseline_summary(baseline_path)
                req = urllib.request.Request(f"http://127.0.0.1:{args.port}/baseline/reset", data=b"", method="POST")
                with urllib.request.urlopen(req, timeout=10) as r:
                    baseline["reset"] = json.loads(r.read())
                baseline["after_reset"] = _baseline_summary(baseline_path)
        finally:
            alive = agent.poll() is None
            agent.terminate()
            try:
                agent.wait(30)
            except subprocess.TimeoutExpired:
                agent.kill()
                agent.wait()
    checker = subprocess.run([sys.executable, os.path.join(REPO, "check-gpu-node.py"), "--kubeconfig", kc, "--json",
                              "--mi355x", "--json-extended"], capture_output=True, text=True, env=env, timeout=60)
    try:
        verdict = json.loads(checker.stdout)
    except ValueError:
        verdict = {"raw": checker.stdout[-2000:]}
    explain = subprocess.run([sys.executable, os.path.join(REPO, "check-gpu-node.py"), "--kubeconfig", kc,
                              "--explain", name], capture_output=True, text=True, env=env, timeout=60)
    writes = [e for e in srv.log if e["method"] in ("PATCH", "POST")]
    rss = [s["agent_rss_mb"] for s in samples if s["agent_rss_mb"]]
    resident = set.intersection(*(set(int(k) for k in s["children_rss_mb"]) for s in samples)) if samples else set()
    out = {
        "minutes": args.minutes, "agent_cmd": cmd[2:], "agent_alive_at_end": alive, "samples": len(samples),
        "conditions_seen": sorted({str(s["condition"]) for s in samples}),
        "states_seen": sorted({str(s["state"]) for s in samples}),
        "healthz_seen": sorted({str(s["healthz"]) for s in samples}),
        "heartbeat_age_s": _spread([s["heartbeat_age_s"] for s in samples]),
        "agent_rss_mb": _spread(rss), "agent_rss_first_last": [rss[0], rss[-1]] if rss else None,
        "diag_isolation": args.diag_isolation,
        # what stays resident: the agent plus the descendants present at every sample (process isolation: the
        # forkserver and multiprocessing's resource tracker; a diagnostic child lives for seconds, between samples)
        "resident_children": sorted(resident),
        "resident_total_mb": _spread([s["agent_rss_mb"] + sum(v for k, v in s["children_rss_mb"].items()
                                                              if int(k) in resident)
                                      for s in samples if s["agent_rss_mb"]]),
        "diag_child_peak_mb": _spread([s["diag_child_peak_mb"] for s in samples]),
        "diag_children_seen": len({s["diag_child_pid"] for s in samples if s["diag_child_pid"]}),
        "vram_used_mb": _spread([s["vram_used_mb"] for s in samples]),
        # leak watch over the run's diagnostic children: the agent's fds and threads, unreaped children
        "agent_fds": _spread([s["agent_fds"] for s in samples]),
        "agent_fds_first_last": [samples[0]["agent_fds"], samples[-1]["agent_fds"]] if samples else None,
        "agent_threads": _spread([s["agent_threads"] for s in samples]),
        "zombies_max": max((s["zombies"] for s in samples), default=0),
        "diag_failures": sum(1 for s in samples for v in s["diag_pass"].values() if v is False),
        "apiserver_writes": {p: sum(1 for e in writes if e["path"] == p) for p in sorted({e["path"] for e in writes})},
        "labels_last": samples[-1]["labels"] if samples else None,
        "baseline": baseline,
        "checker": {"exit_code": checker.returncode, "output": verdict},
        "explain": {"exit_code": explain.returncode, "text": explain.stdout.splitlines()},
        "series": samples,
    }
    out["ok"] = (alive and out["conditions_seen"] == ["True"] and out["healthz_seen"] == ["200"]
                 and out["diag_failures"] == 0 and checker.returncode == 0)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "series"}), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
