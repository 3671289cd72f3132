#!/usr/bin/env python3
"""Headline benchmark: end-to-end GPU-node check latency + nodes/s against a mock kube-apiserver.

Metric of record (BASELINE.json): "end-to-end check latency (ms) + nodes/sec,
mock kube-API at 1/2/4/8 GPU nodes".  One rank per GPU; GPU ``r`` *is* cluster
node ``mi355x-node-r`` (``amd.com/gpu: 1``), so the cluster grows with the
job (weak scaling: fixed work per GPU).

Setup (untimed)
  * rank 0 starts the mock kube-apiserver in its own process (before any GPU
    work) serving N realistic ~5.9 KB Node objects;
  * every rank runs the MI355X node agent on its own GPU: native amd-smi probe
    (``libmi355x_probe.so``) + level-1 HIP diagnostics (``libmi355x_diag.so``:
    MFMA bf16 GEMM with fp32-reference check, HBM bandwidth) and PATCHes the
    ``amd.com/mi355x-health`` annotation of its node over HTTP.

Timed step (rank 0, identical to ``check-gpu-node --json``; other ranks wait at
the closing barrier):  fresh TCP connection -> paginated ``GET
/api/v1/nodes`` -> native NodeList scan -> MI355X health gate on every node's
annotation -> JSON report rendered -> exit code.  Nothing is cached between
steps.  ``--mode sweep`` additionally re-probes every GPU and re-PATCHes its
annotation inside each step.

Untimed extras (coldstart runs, the agent's diagnostics, the RCCL fabric check and the multi-GPU node
cycle) share one wall-clock budget (``--extras-budget``, 180 s from start): an extra that would not fit in
what is left is recorded as ``{"skipped": "budget"}``, the node-cycle child is killed at the budget, and the
timed loop never waits on any of them.  Every phase's wall time is in the line (``phases_s``), and where a
timed step's milliseconds go -- connect, first byte, body, scan, health gate, render -- as medians
(``step_ms``).

Node-count curve (``curve``; rank 0, after the headline, others at the closing barrier): the same check, same
``--steps`` / ``--warmup``, against one mock cluster per node count of ``--curve`` (1/2/4/8/16/1000; each server
started with the headline's, before any GPU work, its nodes carrying the recorded MI355X probe annotation).  Every
row -- the headline's own is one -- has ms per check, nodes/s, the survey proxy's ms at that count
(``baseline_basis``: a different machine), ``vs_baseline``, and ``checker_ms``: the checker's own part of a check
(scan + client + health + render + other), apart from ``transport_ms`` (connect + first byte + body: the socket
and the mock's time).

Placement (``cpu_pair``; ``--no-pin``): the mock apiservers run on one CPU and rank 0's checking thread on the
other CPUs of that CPU's L3 domain, for the timed steps and the curve; the line's ``pinning`` says which, and
``unpinned`` is the headline's check timed once more at the end with neither side pinned.

Prints ONE JSON line (rank 0): value = nodes/s over the whole job (headline node count = GPUs).
"""

from __future__ import annotations

import argparse
import io
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# reference in-process one_shot median (ms, no Slack) at N GPU nodes
REF_MS = {1: 2.17, 2: 1.68, 4: 1.74, 8: 2.30, 16: 2.23, 1000: 92.7}
REF_MS_SLACK = {1: 4.43, 2: 4.02, 4: 3.08, 8: 3.08, 16: 3.57, 1000: 86.1}


def _cpu_list(text: str) -> set:
    """``0-3,8,10-11`` -> {0, 1, 2, 3, 8, 10, 11} (sysfs CPU lists)."""
    out = set()
    for part in text.strip().split(","):
        if part:
            lo, _, hi = part.partition("-")
            out.update(range(int(lo), int(hi or lo) + 1))
    return out


def cpu_pair() -> "dict | None":
    """CPUs of one L3 domain this process may run on: one for the mock apiserver, the others (on another physical
    core first) for the checking thread.  A request is a wake-up of the server and a wake-up back; across
    dies that costs more than the server's own work, so where the scheduler happens to put the two is the box, not the
    code.  None when no two allowed CPUs share an L3 or the topology is unreadable (then nothing is pinned)."""
    try:
        allowed = os.sched_getaffinity(0)
    except (AttributeError, OSError):
        return None
    sysfs = "/sys/devices/system/cpu/cpu{}/{}"
    seen: set = set()
    try:  # the domain of the CPU this process runs on first (the scheduler put it where there was room)
        with open("/proc/self/stat") as f:
            here = int(f.read().rsplit(")", 1)[1].split()[36])
    except (OSError, ValueError, IndexError):
        here = -1
    try:
        for c in sorted(allowed, key=lambda x: (x != here, x)):
            if c in seen:
                continue
            with open(sysfs.format(c, "cache/index3/shared_cpu_list")) as f:
                group = _cpu_list(f.read())
            seen |= group
            usable = sorted(group & allowed)
            if len(usable) < 2:
                continue
            client = usable[0]
            with open(sysfs.format(client, "topology/thread_siblings_list")) as f:
                siblings = _cpu_list(f.read())
            server = next((x for x in usable if x not in siblings), usable[1])
            with open(sysfs.format(server, "topology/thread_siblings_list")) as f:
                core = _cpu_list(f.read()) | {server}
            # the checker's own threads (the paged LIST's prefetch, the Slack sender) get the rest of the domain, off
            # the server's physical core where that leaves any
            client_cpus = sorted(set(usable) - core) or sorted(set(usable) - {server})
            return {"client_cpus": client_cpus, "server_cpu": server, "l3_cpus": len(group)}
    except (OSError, ValueError):
        return None
    return None


def _start(module: str, *args: str) -> subprocess.Popen:
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    return subprocess.Popen([sys.executable, "-m", module, *args], stdout=subprocess.PIPE, env=env, text=True)


def _ready(proc: subprocess.Popen, module: str) -> dict:
    """The first stdout line of a started control-plane process (its URL), once it is serving."""
    assert proc.stdout is not None
    line = proc.stdout.readline()
    if not line:
        raise RuntimeError(f"{module} failed to start")
    return json.loads(line)


def _spawn(module: str, *args: str) -> "tuple[subprocess.Popen, dict]":
    proc = _start(module, *args)
    return proc, _ready(proc, module)


MOCK = "k8s_gpu_node_checker_amd.testing.mock_apiserver"
# the BASELINE metric's node counts (1/2/4/8) plus the survey's 16 and 1000-node proxy points
CURVE_NODES = "1,2,4,8,16,1000"
BASELINE_BASIS = ("SURVEY §6 proxy: the unmodified reference (check-gpu-node.py:215-293) with a stub kubernetes "
                  "client, in-process one_shot median, 8-vCPU Xeon VM -- a different machine from this run")


def _curve_servers(sizes: "list[int]", procs: list, pin: "list | None" = None) -> dict:
    """One mock apiserver per curve point, all started at once (before any GPU work): ``n`` realistic MI355X
    nodes (``amd.com/gpu: 1``) carrying the recorded probe annotation and condition the DaemonSet writes
    (gzip-encoded), so every node goes through the same health gate as the headline's live ones.  Each process
    goes into ``procs`` as soon as it starts (the caller ends them, whatever fails after)."""
    started = []
    for n in sizes:
        p = _start(MOCK, "--nodes", str(n), "--kind", "amd", "--gpus-per-node", "1", "--annotation-encoding", "gzip",
                   "--with-health", *(pin or []))
        procs.append(p)
        started.append((n, p))
    return {n: _ready(p, MOCK)["url"] for n, p in started}


def _own_gpu(gpus, local_rank, cuda):
    """amd-smi sees every GPU of the host; keep the one this rank drives (matched by PCI address)."""
    if len(gpus) <= 1:
        return gpus
    mine = []
    if cuda:
        from k8s_gpu_node_checker_amd.ops import diag
        bdf = diag.device_info(local_rank)["bdf"].lower()
        mine = [g for g in gpus if str(g.get("bdf", "")).lower() == bdf]
    mine = mine or [g for g in gpus if g.get("index") == local_rank] or gpus[:1]
    mine = [dict(mine[0], index=0)]
    return mine


def _fabric_check(world, local_rank, cuda):
    """Untimed: bus bandwidth + correctness of all-reduce / reduce-scatter / all-gather / all-to-all over
    the job's process group (RCCL over xGMI on GPUs, gloo on CPU) -- the node-fabric health the passive
    probe can only infer from link state."""
    from k8s_gpu_node_checker_amd.parallel import collectives
    import torch
    sizes = [64 << 20, 256 << 20] if cuda else [1 << 20]
    try:
        rows = collectives.collective_bench(sizes, iters=10, warmup=3,
                                            device=torch.device(f"cuda:{local_rank}") if cuda else None)
        return {"backend": "nccl(rccl)" if cuda else "gloo", "rows": rows, **collectives.verdict(rows, world)}
    except Exception as e:  # report, never lose the benchmark line over the fabric check
        return {"backend": "nccl(rccl)" if cuda else "gloo", "pass": False, "detail": f"{type(e).__name__}: {e}"}


class Budget:
    """Wall clock left for the untimed extras (from process start) and the phases' wall times."""

    def __init__(self, total_s: float):
        self.total = total_s
        self.t0 = time.monotonic()
        self.phases: dict = {}

    def left(self) -> float:
        return self.total - (time.monotonic() - self.t0)

    def fits(self, need_s: float) -> bool:
        """Whether an extra that needs ``need_s`` may start (a small budget scales the need down with it)."""
        return self.left() >= min(need_s, 0.25 * self.total) and self.left() > 0

    class _Phase:
        def __init__(self, b: "Budget", name: str):
            self.b, self.name = b, name

        def __enter__(self):
            self.t = time.monotonic()

        def __exit__(self, *exc):
            self.b.mark(self.name, self.t)

    def phase(self, name: str) -> "Budget._Phase":
        return Budget._Phase(self, name)

    def mark(self, name: str, since: float) -> None:
        """Add the time since ``since`` (monotonic) to phase ``name`` (for phases that are not one block)."""
        self.phases[name] = round(self.phases.get(name, 0.0) + time.monotonic() - since, 3)


# the least budget an extra must have left to start (s): RCCL's first communicator loads comgr cold
FABRIC_MIN_S = 60.0
NODE_CYCLE_MIN_S = 30.0
AGENT_DIAG_MIN_S = 10.0
COLDSTART_MIN_S = 5.0


def _node_cycle(world: int, timeout_s: float = 150.0, cmd: "list | None" = None, kill_after_s: "float | None" = None) -> dict:
    """Untimed, rank 0, world > 1 on GPUs: the node agent's multi-device cycle over every GPU of the job
    (``agent/node_cycle.py``: per-device diagnostic threads at once, xGMI pair matrix, in-process RCCL suite
    under its deadline) in a child process with a time limit, so a failure there is reported in the bench
    line and never costs the benchmark.  The other ranks wait on a CPU (gloo) barrier meanwhile: no spinning
    collective kernel on their GPUs."""
    cmd = cmd or [sys.executable, "-m", "k8s_gpu_node_checker_amd.agent.node_cycle", "--devices",
                  ",".join(str(d) for d in range(world)), "--level", "1", "--timeout", str(round(timeout_s, 1))]
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    limit = kill_after_s if kill_after_s is not None else 2 * timeout_s + 60
    t = time.perf_counter()
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=limit)
    except subprocess.TimeoutExpired:
        return {"pass": False, "killed": "budget", "child_wall_s": round(time.perf_counter() - t, 2),
                "detail": f"node cycle did not finish within the {limit:.0f} s left of the extras budget"}
    line = next((x for x in reversed(p.stdout.splitlines()) if x.startswith("{")), None)
    if p.returncode != 0 or line is None:
        return {"pass": False, "rc": p.returncode, "detail": (p.stderr or p.stdout)[-400:]}
    res = json.loads(line)
    res["pass"] = all(d.get("pass") for d in res.get("per_device", {}).values()) and all(
        (r or {}).get("pass") is not False for r in (res.get("fabric") or {}).values())
    res["child_wall_s"] = round(time.perf_counter() - t, 2)
    return res


def _coldstart(api_url: str, runs: int) -> dict:
    """Whole-process wall clock of ``check-gpu-node --json`` against the same mock (what a cron / CI user
    pays per check), measured in child processes before this process touches the GPU: median of
    ``runs`` after one untimed run (byte-code cache), and the interpreter's own start-up for scale."""
    import statistics
    import tempfile
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
    kc = write_kubeconfig(os.path.join(tempfile.mkdtemp(prefix="bench-kc"), "config"), api_url)
    cmd = [sys.executable, os.path.join(REPO, "check-gpu-node.py"), "--kubeconfig", kc, "--json"]
    env = {k: v for k, v in os.environ.items() if k not in ("SLACK_WEBHOOK_URL",)}

    def wall(c):
        t = time.perf_counter()
        rc = subprocess.run(c, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env).returncode
        return (time.perf_counter() - t) * 1e3, rc
    _, rc = wall(cmd)
    runs_ms = [wall(cmd)[0] for _ in range(runs)]
    floor = [wall([sys.executable, "-c", "pass"])[0] for _ in range(runs)]
    return {"ms": round(statistics.median(runs_ms), 2), "min_ms": round(min(runs_ms), 2), "runs": runs,
            "exit_code": rc, "python_startup_ms": round(statistics.median(floor), 2)}


def _pctl(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    i = min(len(xs) - 1, max(0, int(round(q * (len(xs) - 1)))))
    return xs[i]


def _step_breakdown(spans: list, lat: list) -> "dict | None":
    """Median per-step milliseconds of each part of a check (``utils/timing.Tracer`` spans of the timed steps):
    ``connect`` (TCP to the apiserver), ``first_byte`` (LIST sent to response head: the server's time),
    ``body`` (the rest of the response), ``scan`` (NodeList scan), ``client`` (the rest of the LIST call:
    client setup, headers, close), ``health`` (MI355X gate), ``render`` (JSON), ``other`` (what the step spent
    outside those: Slack join when on, GC switch, the output sink).

    ``checker`` is the checker's own cost -- scan + client + health + render + other, summed per step -- and
    ``transport`` the rest (connect + first_byte + body: the socket and the mock apiserver's time), so a
    comparison across boxes or rounds can tell the code's milliseconds from the mock's."""
    if not spans or len(spans) != len(lat):
        return None
    rows = []
    for sp, total in zip(spans, lat):
        g = sp.get
        lst = g("list", 0.0)
        r = {"connect": g("connect", 0.0), "first_byte": g("first_byte", 0.0), "body": g("body", 0.0),
             "scan": g("parse", 0.0),
             "client": lst - g("connect", 0.0) - g("first_byte", 0.0) - g("body", 0.0) - g("parse", 0.0),
             "health": g("health", 0.0), "render": g("render", 0.0),
             "other": total - lst - g("health", 0.0) - g("render", 0.0)}
        r["transport"] = r["connect"] + r["first_byte"] + r["body"]
        r["checker"] = total - r["transport"]
        rows.append(r)
    out = {k: round(_pctl([r[k] for r in rows], 0.5) * 1e3, 4) for k in rows[0]}
    if any("slack" in sp for sp in spans):
        out["slack"] = round(_pctl([sp.get("slack", 0.0) for sp in spans], 0.5) * 1e3, 4)
    out["step"] = round(_pctl(lat, 0.5) * 1e3, 4)
    return out


def _timed_checks(cluster, opts, steps: int, warmup: int) -> "tuple[float, list, list, object]":
    """``warmup`` untimed then ``steps`` timed ``check_and_report`` calls against ``cluster`` (the bench step):
    (elapsed s, per-step latencies, per-step tracer spans, the last result)."""
    from k8s_gpu_node_checker_amd.checker import check_and_report
    from k8s_gpu_node_checker_amd.utils.timing import Tracer
    sink_out, sink_err = io.StringIO(), io.StringIO()
    last = None
    for _ in range(warmup):
        sink_out.seek(0)
        sink_out.truncate()
        last = check_and_report(cluster, opts, out=sink_out, err=sink_err)
    lat, spans = [], []
    t0 = time.perf_counter()
    for _ in range(steps):
        sink_out.seek(0)
        sink_out.truncate()
        s = time.perf_counter()
        tr = Tracer()
        last = check_and_report(cluster, opts, out=sink_out, err=sink_err, tracer=tr)
        lat.append(time.perf_counter() - s)
        spans.append(tr.spans)
    return time.perf_counter() - t0, lat, spans, last


def curve_row(nodes: int, elapsed: float, steps: int, lat: list, spans: list, last, slack: bool,
              annotations: str) -> dict:
    """One point of the node-count curve: the same numbers as the headline (ms per check, nodes/s, the
    survey proxy's ms at that node count and the ratio) plus where a check's milliseconds go."""
    ms = elapsed / max(steps, 1) * 1e3
    ref = (REF_MS_SLACK if slack else REF_MS).get(nodes)
    bd = _step_breakdown(spans, lat)
    return {"nodes": nodes, "ms_per_step": round(ms, 4), "p50_ms": round(_pctl(lat, 0.5) * 1e3, 4),
            "nodes_per_s": round(nodes / (ms / 1e3), 2) if ms > 0 else None,
            "checker_ms": bd["checker"] if bd else None, "transport_ms": bd["transport"] if bd else None,
            "baseline_ms": ref, "vs_baseline": round(ref / ms, 3) if ref and ms > 0 else None,
            "check_ok": last is not None and last.exit_code == 0 and len(last.ready_gpu_nodes) == nodes,
            "exit_code": last.exit_code if last is not None else None, "annotations": annotations,
            "step_ms": bd}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--nodes", type=int, default=0, help="cluster size override (default: one node per GPU)")
    ap.add_argument("--mode", choices=("check", "sweep"), default="check")
    ap.add_argument("--diag-level", type=int, default=1, choices=(0, 1, 2))
    ap.add_argument("--slack", action="store_true", help="also POST the Slack report to a local sink each step")
    ap.add_argument("--page-size", type=int, default=500)
    ap.add_argument("--curve", default=CURVE_NODES, metavar="N,N,...",
                    help="also time the same check (same --steps / --warmup, rank 0, after the headline) against one "
                         f"mock cluster per node count (default {CURVE_NODES}; '' to skip); the headline's own node "
                         "count is its row")
    ap.add_argument("--no-pin", dest="pin", action="store_false",
                    help="leave the checking thread and the mock apiservers where the scheduler puts them (default: two "
                         "CPUs of one L3 domain, cpu_pair())")
    ap.add_argument("--coldstart-runs", type=int, default=11,
                    help="child-process runs of check-gpu-node --json for coldstart_ms (rank 0, before GPU work; 0: skip)")
    ap.add_argument("--no-fabric-check", dest="fabric_check", action="store_false",
                    help="skip the untimed all-reduce fabric check (world > 1)")
    ap.add_argument("--no-node-cycle", dest="node_cycle", action="store_false",
                    help="skip the untimed multi-GPU node-agent cycle (world > 1 on GPUs)")
    ap.add_argument("--extras-budget", type=float, default=180.0, metavar="S",
                    help="wall clock for all untimed extras together (coldstart, agent diagnostics, fabric check, "
                         "node cycle); what does not fit is skipped and recorded (default 180)")
    # tests: run the node cycle without GPUs / replace its command (e.g. a child that sleeps past the budget)
    ap.add_argument("--node-cycle-always", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--node-cycle-cmd", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    budget = Budget(args.extras_budget)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = world if world > 1 else args.gpus
    n_nodes = args.nodes or n_gpus

    # --- control-plane processes first: nothing below has touched the GPU yet
    procs = []
    ctrl = {}
    t_control = time.monotonic()
    if rank == 0:
        pair = cpu_pair() if args.pin else None
        ctrl["pinning"] = pair or {"skipped": "--no-pin" if not args.pin else "no two allowed CPUs share an L3"}
        pin = ["--cpu", str(pair["server_cpu"])] if pair else []
        # nodes beyond the GPU count start with a recorded MI355X probe (condition + annotation, gzip-encoded
        # as the DaemonSet writes it); the ranks' own nodes get their live probe PATCHed below
        p, info = _spawn("k8s_gpu_node_checker_amd.testing.mock_apiserver", "--nodes", str(n_nodes), "--kind", "amd",
                         "--gpus-per-node", "1", "--annotation-encoding", "gzip",
                         *(["--with-health"] if n_nodes > n_gpus else []), *pin)
        procs.append(p)
        ctrl["api"] = info["url"]
        ctrl["api_pid"] = p.pid
        if args.slack:
            p, sinfo = _spawn("k8s_gpu_node_checker_amd.testing.webhook_sink")
            procs.append(p)
            ctrl["slack"] = sinfo["url"] + "/200"
        sizes = sorted({int(x) for x in args.curve.split(",") if x.strip()} - {n_nodes})
        if sizes:
            try:
                ctrl["curve_api"] = _curve_servers(sizes, procs, pin)
            except Exception as e:  # the curve is an extra: its servers failing must not cost the headline
                ctrl["curve_error"] = f"{type(e).__name__}: {e}"[:300]
    budget.mark("control_plane", t_control)
    if rank == 0 and args.coldstart_runs > 0:
        if budget.fits(COLDSTART_MIN_S):
            with budget.phase("coldstart"):
                ctrl["coldstart"] = _coldstart(ctrl["api"], args.coldstart_runs)
        else:
            ctrl["coldstart"] = {"skipped": "budget"}
    try:
        return _run(args, world, rank, local_rank, n_gpus, n_nodes, ctrl, budget)
    finally:
        for p in procs:
            p.terminate()
            try:
                p.wait(timeout=5)
            except subprocess.TimeoutExpired:
                p.kill()


def _run(args, world, rank, local_rank, n_gpus, n_nodes, ctrl, budget) -> int:
    t_init = time.monotonic()  # phase "init": torch import, process group, control-plane broadcast
    import torch
    import torch.distributed as dist

    from k8s_gpu_node_checker_amd.agent.agent import Agent
    from k8s_gpu_node_checker_amd.checker import CheckOptions, check_and_report
    from k8s_gpu_node_checker_amd.kube.client import KubeClient
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    from k8s_gpu_node_checker_amd.ops import fastpath
    from k8s_gpu_node_checker_amd.testing import fixtures
    from k8s_gpu_node_checker_amd.utils.timing import Tracer

    cuda = torch.cuda.is_available()
    if cuda:
        torch.cuda.set_device(local_rank)
    group = None
    if world > 1:
        from datetime import timedelta
        if cuda:
            # RCCL carries only the fabric check (an untimed extra): the group is created lazily, so its
            # communicator -- and comgr's cold code-object load -- is paid inside the extras budget or not at all,
            # and a collective that hangs raises at the timeout instead of killing the rank (CleanUpOnly)
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
            dist.init_process_group("nccl", timeout=timedelta(seconds=max(30.0, min(300.0, budget.left()))))
        else:
            dist.init_process_group("gloo")
        # control plane (URLs, decisions, the timing barriers and the MAX over ranks): gloo on the CPU, with room
        # for rank 0's node cycle (up to the whole extras budget) at the barrier the others wait at
        group = dist.new_group(backend="gloo", timeout=timedelta(seconds=budget.total + 600.0))
        box = [ctrl]
        dist.broadcast_object_list(box, src=0, group=group)
        ctrl = box[0]

    def barrier():
        if cuda:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier(group=group)  # gloo: the timed region never waits on an RCCL communicator
        if cuda:
            torch.cuda.synchronize()

    def agree(flag: bool) -> bool:
        """Rank 0's decision for every rank (an extra that involves all of them runs everywhere or nowhere)."""
        if world <= 1:
            return flag
        box = [flag]
        dist.broadcast_object_list(box, src=0, group=group)
        return bool(box[0])

    cluster = ClusterConnection(ctrl["api"])
    node = f"mi355x-node-{rank:04d}"
    budget.mark("init", t_init)
    skipped = {}

    # --- node agent on this rank's GPU: probe (+ diagnostics), publish annotation
    # diag_when="always": this process is the GPU's only user and runs the diagnostics on purpose
    # the DaemonSet's publishing configuration (deploy/daemonset.yaml: gzip-encoded report annotation)
    # The diagnostics get what is left of the extras budget as their watchdog (a GPU still running then is
    # reported failed and the bench goes on); with less than AGENT_DIAG_MIN_S left only the probe runs.
    diag_level = args.diag_level if cuda else 0
    if diag_level and not agree(budget.fits(AGENT_DIAG_MIN_S)):
        diag_level = 0
        skipped["agent_diag"] = "budget"
    agent = Agent(node, source="auto", diag_level=diag_level,
                  devices=[local_rank] if cuda else [], diag_when="always", annotation_encoding="gzip",
                  diag_timeout=max(AGENT_DIAG_MIN_S, min(300.0, budget.left())))
    t0 = time.perf_counter()
    with budget.phase("agent_cycle"):
        rep = agent.probe_once()
    probe_source = rep.get("probe")
    if rep.get("error") or not rep.get("gpus"):
        # no amdgpu driver (CPU CI): publish a recorded MI355X report instead, and say so
        rep = fixtures.mi355x_probe_report(node, gpus=1)
        probe_source = "fixture"
    else:
        rep["gpus"] = _own_gpu(rep["gpus"], local_rank, cuda)
    probe_ms = (time.perf_counter() - t0) * 1e3
    with budget.phase("publish"), KubeClient(cluster) as kc:
        agent.publish(kc, rep, force=True)  # AMDGPUHealthy NodeCondition + full report annotation
    diag = {}
    for g in rep.get("gpus") or []:
        diag = g.get("diag") or {}
    if skipped.get("agent_diag"):
        diag = {"skipped": "budget"}
    fabric = None
    if world > 1 and args.fabric_check:
        if agree(budget.fits(FABRIC_MIN_S)):
            with budget.phase("fabric"):
                fabric = _fabric_check(world, local_rank, cuda)
        else:
            fabric = {"skipped": "budget"}
    node_cycle = None
    if world > 1 and args.node_cycle and (cuda or args.node_cycle_always):
        if agree(budget.fits(NODE_CYCLE_MIN_S)):
            dist.barrier(group=group)  # CPU barrier: every rank's own setup is done, its GPU idle
            with budget.phase("node_cycle"):
                if rank == 0:
                    left = budget.left()
                    node_cycle = _node_cycle(world, timeout_s=min(150.0, max(5.0, (left - 10.0) / 2)),
                                             cmd=args.node_cycle_cmd.split() if args.node_cycle_cmd else None,
                                             kill_after_s=max(1.0, left))
            dist.barrier(group=group)
        else:
            node_cycle = {"skipped": "budget"}
    barrier()

    opts = CheckOptions(json=True, page_size=args.page_size, health_policy="auto",
                        slack_webhook=ctrl.get("slack"), slack_retry_policy="backoff")
    sink_out, sink_err = io.StringIO(), io.StringIO()

    def step():
        if args.mode == "sweep":
            r = agent.probe_once() if probe_source != "fixture" else fixtures.mi355x_probe_report(node, gpus=1)
            if probe_source != "fixture":
                r["gpus"] = _own_gpu(r["gpus"], local_rank, cuda)
            with KubeClient(cluster) as kc2:
                agent.publish(kc2, r, force=True)  # the full write cycle (a live agent skips unchanged writes)
            barrier()
        if rank == 0:
            sink_out.seek(0)
            sink_out.truncate()
            tr = Tracer()  # per-step spans (utils/timing): a few perf_counter calls, ~2 us of the step
            res = check_and_report(cluster, opts, out=sink_out, err=sink_err, tracer=tr)
            spans.append(tr.spans)
            return res
        return None

    last = None
    spans: list = []
    # rank 0 checks from the CPU beside the mock apiserver's (cpu_pair); this thread only, put back after the curve
    pinned = ctrl.get("pinning") if rank == 0 and "client_cpus" in (ctrl.get("pinning") or {}) else None
    mask = None
    if pinned:
        try:
            mask = os.sched_getaffinity(0)
            os.sched_setaffinity(0, set(pinned["client_cpus"]))
        except OSError:
            mask = None
    with budget.phase("warmup"):
        for _ in range(args.warmup):
            last = step()
        barrier()
    spans.clear()
    lat = []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        s = time.perf_counter()
        last = step()
        lat.append(time.perf_counter() - s)
    barrier()
    elapsed = time.perf_counter() - t_start
    budget.phases["timed"] = round(elapsed, 3)

    if world > 1:
        import torch as _t
        t = _t.tensor([elapsed], dtype=_t.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)  # the slowest rank's clock (gloo, CPU tensor)
        elapsed = float(t.item())

    curve = None
    if rank == 0:
        # the BASELINE metric's node-count axis (the reference's one LIST + per-node loop,
        # check-gpu-node.py:215-226): the headline's row, then one mock cluster per other node count, each timed
        # like the headline; the other ranks wait at the closing gloo barrier meanwhile
        curve = [curve_row(n_nodes, elapsed, args.steps, lat, spans, last, bool(args.slack),
                           "live" if probe_source != "fixture" else "fixture")]
        with budget.phase("curve"):
            for n, url in sorted((ctrl.get("curve_api") or {}).items()):
                try:
                    el, lt, sp, ls = _timed_checks(ClusterConnection(url), opts, args.steps, args.warmup)
                    curve.append(curve_row(n, el, args.steps, lt, sp, ls, bool(args.slack), "recorded"))
                except Exception as e:  # a row that fails is reported as such; the line still prints
                    curve.append({"nodes": n, "check_ok": False, "error": f"{type(e).__name__}: {e}"[:300]})
            if ctrl.get("curve_error"):
                curve.append({"nodes": None, "check_ok": False, "error": ctrl["curve_error"]})
        curve.sort(key=lambda r: (r["nodes"] is None, r["nodes"] or 0))
    unpinned = None
    if mask is not None:
        os.sched_setaffinity(0, mask)
        # the headline once more with neither side pinned (the server's new request threads inherit its main
        # thread's mask): how much of the number is placement, measured in every run rather than asserted
        try:
            os.sched_setaffinity(ctrl["api_pid"], mask)
            el, lt, _, _ = _timed_checks(ClusterConnection(ctrl["api"]), opts, args.steps, args.warmup)
            unpinned = {"ms_per_step": round(el / max(args.steps, 1) * 1e3, 4),
                        "p50_ms": round(_pctl(lt, 0.5) * 1e3, 4), "steps": args.steps}
        except Exception as e:  # an extra: never costs the line
            unpinned = {"error": f"{type(e).__name__}: {e}"[:200]}

    if rank == 0:
        ok = last is not None and last.exit_code == 0 and len(last.ready_gpu_nodes) == n_nodes
        verdicts = [v.state for v in (last.verdicts or []) if v is not None] if last else []
        ms = elapsed / max(args.steps, 1) * 1e3
        value = n_nodes * args.steps / elapsed
        ref = (REF_MS_SLACK if args.slack else REF_MS).get(n_nodes)
        vs = round(value / (n_nodes / (ref / 1e3)), 3) if ref else None
        node_bytes = len(json.dumps(fixtures.realistic_node("x", "amd.com/gpu", 1), separators=(",", ":")))
        out = {
            "metric": "end-to-end GPU-node check throughput (nodes/s) against a mock kube-apiserver; "
                      "ms_per_step = check latency",
            "value": round(value, 2),
            "unit": "nodes/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": vs,
            "dtype": "n/a (control plane; agent diagnostics bf16 MFMA)",
            "data": "synthetic: mock kube-apiserver, realistic Node objects, live MI355X probe annotations"
                    if probe_source != "fixture" else "synthetic: mock kube-apiserver, fixture probe annotations (no GPU)",
            "config": {"model": f"{n_nodes}-node MI355X mock cluster (amd.com/gpu:1 per node = 1 GPU per rank)",
                       "global_batch": n_nodes, "seq_len": None, "node_bytes": node_bytes,
                       "parallelism": f"dp{n_gpus}" if n_gpus > 1 else "single",
                       "mode": args.mode, "slack": bool(args.slack), "page_size": args.page_size},
            # p99 of fewer than 100 samples is the max: reported as null then
            "latency_ms": {"p50": round(_pctl(lat, 0.5) * 1e3, 4), "p90": round(_pctl(lat, 0.9) * 1e3, 4),
                           "p99": round(_pctl(lat, 0.99) * 1e3, 4) if len(lat) >= 100 else None,
                           "min": round(min(lat) * 1e3, 4), "samples": len(lat)},
            # where a step's milliseconds go: medians over the timed steps of the check's own spans
            "step_ms": _step_breakdown(spans, lat),
            # the checker's own milliseconds per check (scan + client + health + render + other), without the
            # socket and the mock apiserver's time: what says something about the code across boxes and rounds
            "checker_ms": (_step_breakdown(spans, lat) or {}).get("checker"),
            "baseline_basis": BASELINE_BASIS,
            # where the checking thread and the mock apiservers ran (cpu_pair), or why they were not pinned, and the
            # headline's check timed again afterwards with neither side pinned
            "pinning": ctrl.get("pinning"),
            "unpinned": unpinned,
            # ms per check, nodes/s, checker_ms and vs_baseline at every node count (headline row included)
            "curve": curve,
            "coldstart_ms": (ctrl.get("coldstart") or {}).get("ms"),
            "coldstart": ctrl.get("coldstart"),
            "baseline_ms": ref,
            "check_ok": ok,
            "exit_code": last.exit_code if last else None,
            "health": {s: verdicts.count(s) for s in sorted(set(verdicts))},
            "backend": fastpath.backend(),
            "probe": {"source": probe_source, "setup_ms": round(probe_ms, 1), "diag": diag},
            "fabric": fabric,
            "node_cycle": node_cycle,
            "phases_s": budget.phases,
            "extras_budget_s": {"budget": budget.total,
                                "used": round(sum(v for k, v in budget.phases.items()
                                                  if k in ("coldstart", "agent_cycle", "fabric", "node_cycle")), 3),
                                "skipped": sorted(k for k, v in (("coldstart", ctrl.get("coldstart")),
                                                                 ("agent_diag", diag), ("fabric", fabric),
                                                                 ("node_cycle", node_cycle))
                                                  if isinstance(v, dict) and v.get("skipped") == "budget")},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier(group=group)
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
