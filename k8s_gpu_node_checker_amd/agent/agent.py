"""MI355X node agent (DaemonSet): probe -> publish (SURVEY §7.2 layer 5 source (a)/(b)).

Every ``--interval`` seconds the agent runs the passive amd-smi probe
(``ops/amdsmi_probe.py``, native library) and, every ``--diag-interval``
seconds, the active HIP diagnostics (``ops/diag.py``: MFMA GEMM + numerics,
HBM bandwidth, memtest) at ``--diag-level``.  The merged report is published

* as the NodeCondition ``AMDGPUHealthy`` (strategic-merge PATCH of
  ``nodes/status``, node-problem-detector style: the checker reads the
  verdict from the LIST it already does, zero extra API calls, no JSON to
  parse per node) plus the full report as the annotation
  ``amd.com/mi355x-health`` (``--json-extended`` details, ``--health-reeval``), and/or
* over HTTP at ``/probe`` (JSON), ``/metrics`` (Prometheus) and ``/status`` (text, for a person with
  ``kubectl port-forward``) for the
  checker's ``--probe-endpoint`` fan-out, and/or
* on stdout (``--publish stdout``, one JSON line per probe).

Each verdict change is also posted as a Kubernetes Event on the node (``Warning MI355XUnhealthy``,
``Normal MI355XHealthy ... (was unhealthy)``), and with ``--taint-unhealthy`` the node carries
``amd.com/gpu-unhealthy=true:NoSchedule`` while it is unhealthy (read-modify-write under the node's
``resourceVersion``, so a concurrent ``kubectl taint`` is never lost).

RBAC: ``nodes: get, patch``, ``nodes/status: patch`` and ``events: create`` (``deploy/rbac.yaml``), narrowed to
the agent's own node and to the fields it owns by ``deploy/agent-policy.yaml`` (a ValidatingAdmissionPolicy on the
node-name claim of its pod-bound token) and by :class:`_OwnNodeClient` here.

Where the HIP work runs (``--diag-isolation``, ``agent/isolation.py``): by default in disposable child processes of
a forkserver started before the agent touches amd-smi or HIP -- one per GPU, narrowed to that GPU, then one for the
node-level tests -- so the agent itself never initialises HIP (65 MiB resident between cycles on MI355X), a
diagnostic that outlives ``--diag-timeout`` is SIGKILLed and its GPU published as failed while the agent keeps
probing, and a GPU fault that aborts the HIP runtime costs one child.  ``thread`` keeps the work in the agent.

Multi-device nodes (8 GPUs, or 64 CPX partitions): per-device diagnostic jobs, at most ``--diag-parallel`` at
once, tests of shared host resources serialized across them (``ops/diag.SHARED_TESTS``); the RCCL suite aborts its
own communicators at its deadline (``csrc/fabric/fabric.hip``) and the xGMI copies are polled against theirs
(``diag_p2p_copy_t``, ``diag_p2p_fan_t``).  With thread isolation a hung diagnostic cannot be ended: one that
outlives twice its watchdog fails ``/healthz`` (fresh process), and a node-level test given up at its deadline is not
run again in the same process (:func:`fabric_abandoned`).
"""

from __future__ import annotations

import argparse
import functools
import json
import os
import socket
import sys
import threading
import time
from typing import Any, Dict, List, Optional, Sequence

from ..models.health import (HEALTHY, UNHEALTHY, UNHEALTHY_TAINT, UNKNOWN, XGMI_LINKS_EXPECTED,
                              HealthExpectations, Verdict,
                              condition_for, condition_reason, driver_release, encode_annotation, evaluate_report,
                              format_k8s_time,
                              throttle_window)
from ..models.baseline import Baselines, epoch_of, gpu_key
from ..models.node import HEALTH_ANNOTATION
from ..models.resources import PRIMARY_GPU_KEY, gpu_breakdown
from .isolation import ISOLATION, Job, Workers
from .server import _metrics, serve, tls_context  # noqa: F401  (the agent's HTTP side; re-exported)


# Report fields that change on every probe without saying anything about health; ignored when deciding
# whether the annotation must be rewritten.
_VOLATILE = frozenset(("ts", "probe_ms", "probe_us", "hotspot_c", "wall_s", "ms_per_gemm", "setup_ms",
                       "power_w", "hbm_temp_c", "gfxclk_mhz", "vram_used_mb", "processes", "throttle_acc",
                       "throttle", "procs", "gfx_activity", "diag_skipped", "xgmi_kb", "ecc_ce_per_h",
                       "diag_proc"))

# correctable-ECC trend: the rate is taken over the probes of the last hour, once they span 10 minutes
CE_WINDOW_S = 3600.0
CE_MIN_SPAN_S = 600.0

DIAG_WHEN = ("idle", "always")
# a GPU's latest diagnostic result counts as a peer of the others' for this long (a busy GPU keeps an older one)
PEER_MAX_AGE_S = 86400.0


def baseline_key(entry: Dict[str, Any], bdf: str, device: int) -> str:
    """Whose self-baseline a device's result feeds: amd-smi UUID, else PCI address, else the HIP ordinal."""
    return gpu_key(entry) or (f"bdf:{bdf}" if bdf else f"hip:{device}")
# per-GPU fields kept out of the node annotation (Agent.annotation)
_ANNOTATION_DROP = frozenset(("xgmi_kb", "throttle_acc", "procs", "probe_us", "diag_proc"))
# a JSON report annotation above this goes out gzip-encoded (the apiserver caps a node's annotations at 256 KiB)
ANNOTATION_JSON_MAX = 128 << 10


def gpu_busy(g: Dict[str, Any], own_pids: frozenset = frozenset(), busy_vram_mb: int = 2048,
             busy_gfx_activity: int = 10) -> Optional[str]:
    """Why a workload holds this GPU, so active diagnostics must not run on it; None when it is idle.

    Busy means a process other than the agent holding at least ``busy_vram_mb`` of VRAM (the probe's
    ``procs``; without that list, the device's total VRAM in use), or a graphics engine at least
    ``busy_gfx_activity`` % busy.  The agent's own HIP context holds a few hundred MB between
    diagnostics, so the VRAM floor also covers a pod without hostPID, where amd-smi's host-namespace
    PIDs never match the agent's own.
    """
    procs = g.get("procs")
    if isinstance(procs, list):
        holders = [p for p in procs if isinstance(p, dict) and p.get("pid") not in own_pids
                   and isinstance(p.get("vram_mb"), int) and p["vram_mb"] >= busy_vram_mb]
        if holders:
            return "in use: " + ", ".join(f"pid {p.get('pid')} holds {p['vram_mb']} MB" for p in holders[:4])
    elif isinstance(g.get("vram_used_mb"), int) and g["vram_used_mb"] >= busy_vram_mb:
        return f"in use: {g['vram_used_mb']} MB of VRAM allocated"
    act = g.get("gfx_activity")
    if isinstance(act, (int, float)) and act >= busy_gfx_activity:
        return f"in use: graphics engine {act}% busy"
    return None


def power_fraction(g: Dict[str, Any]) -> Optional[float]:
    """The GPU's power cap as a share of its default (amd-smi), None when unknown.  A capped GPU runs its matrix
    cores at a lower clock; the compute references are scaled by it so a deliberate cap is not a failed GPU
    (models/health.py warns about the cap itself)."""
    cap, dflt = g.get("power_cap_w"), g.get("power_cap_default_w")
    if isinstance(cap, int) and isinstance(dflt, int) and not isinstance(cap, bool) and cap > 0 and dflt > 0:
        return min(1.0, cap / dflt)
    return None


# HIP errors that say this process's runtime lost its devices (a driver reload or GPU reset under a running
# agent): not the GPU's fault, and not curable in-process -- the agent needs a fresh process
_HIP_RUNTIME_LOST = ("no ROCm-capable device", "invalid device ordinal", "initialization error",
                     "context is destroyed", "hipErrorNoDevice", "hipErrorInvalidDevice", "hipErrorNotInitialized",
                     "hipErrorContextIsDestroyed")


# a diagnostic result that is not clean is run again this soon (s), not a whole --diag-interval later --
# once per distinct result: a GPU that keeps failing the same way goes back to --diag-interval instead of
# being stressed (memtest, HBM) every few minutes while it is already known bad
DIAG_RECHECK_S = 300.0
# diagnostic threads running at once (--diag-parallel): every GPU of an SPX node together, a CPX node's 64
# partitions in waves of 8
DIAG_PARALLEL = 8
# /healthz fails once a diagnostic thread has outlived this many --diag-timeout: its verdict (watchdog) went
# out at 1x; a thread in a hung HIP call cannot be cancelled, so only a fresh process frees its GPU
HUNG_RESTART_FACTOR = 2.0
from ..ops.diag import P2P_SHARE  # noqa: E402  (share of --diag-timeout the xGMI pair matrix may use)


# Host memory (MiB), measured on one MI355X with process isolation, the DaemonSet's mode (tools/agent_soak.py):
# resident between cycles, the agent (31) + the forkserver (17) + multiprocessing's resource tracker (16) --
# profiles/agent_soak_isolated_l{1,2}_r06_mi355x.json, flat over 48 / 36 cycles.  This is the pod's request.
MEM_RESIDENT_MIB = 65
# one diagnostic child's peak, its own getrusage (HIP runtime, comgr's code objects, the level's buffers; the child
# sees one GPU, isolation.narrow_to, so it is the same process on a one-GPU box and on an 8-GPU node), the first one
# on a fresh box, which is the largest: level 1 493 MiB (its runtime starts without the SDMA engines,
# ops/diag.DMA_TESTS; later children 437-445), level 2 1,128 MiB (the host link's pinned buffer and the 8192^3 GEMMs
# included; later children 1,074-1,082) -- profiles/first_child_rss_r06_mi355x.jsonl,
# profiles/agent_soak_isolated_l{1,2}_r06b_mi355x.json
MEM_CHILD_PEAK_MIB = {1: 493, 2: 1128}
# a one-GPU HIP process with its SDMA queues (the fabric child copies between GPUs over them): a level-1 suite with
# the engines on peaks at 628-682 MiB (profiles/child_peak_rss_sdma_r06_mi355x.jsonl)
MEM_GPU_WITH_SDMA_MIB = 682
# the node-level child (xGMI matrix, in-process RCCL suite; level 2, >= 2 GPUs) with a warm comgr cache: 2,712 MiB
# for the suite on one GPU (profiles/rccl_rss_comgr_cache_mi355x.json).  Each further GPU is counted at
# MEM_GPU_WITH_SDMA_MIB -- an upper bound, unmeasured: no multi-GPU box was available to this project
MEM_FABRIC_ONE_GPU_MIB = 2712
# ... and with a cold comgr cache: comgr decompresses RCCL's compressed code objects on the first load, peak 11,786
# MiB (profiles/rccl_rss_comgr_cache_mi355x.json); the level-2 overlay keeps the cache on the node
# (AMD_COMGR_CACHE_DIR on a hostPath) and fills it from an init container with its own limit
MEM_RCCL_COLD_PEAK_MIB = 11786


def memory_budget_mib(devices: int, level: int, rccl: bool = False, parallel: int = DIAG_PARALLEL) -> int:
    """Upper bound of the agent pod's host memory for ``devices`` GPUs at diagnostics ``level`` (the DaemonSet's
    limit; tests/test_deploy.py holds the manifests to it): what stays resident, plus the larger of the device
    children running together (at most ``parallel``, each a measured one-GPU process) and the node-level child,
    which runs alone after them.  :data:`MEM_RESIDENT_MIB` alone is the request."""
    mib = MEM_RESIDENT_MIB
    if level >= 1:
        children = min(max(1, devices), max(1, parallel)) * MEM_CHILD_PEAK_MIB[min(level, 2)]
        fabric = 0
        if level >= 2 and rccl and devices >= 2:
            fabric = MEM_FABRIC_ONE_GPU_MIB + (devices - 1) * MEM_GPU_WITH_SDMA_MIB
        mib += max(children, fabric)
    return mib


class _DiagRun:
    """One device's (or the node-level suite's) diagnostic job (``isolation.Job``: a child process or a thread):
    wall-clock start (reported), monotonic start (watchdog), result box."""
    __slots__ = ("job", "started", "mono", "box")

    def __init__(self, job: Job, started: float, mono: float):
        self.job, self.started, self.mono, self.box = job, started, mono, job.box

    def is_alive(self) -> bool:
        return self.job.is_alive()


def result_signature(res: Dict[str, Any]) -> str:
    """Which tests of a result failed or were degraded (what a recheck is keyed on)."""
    return ",".join(sorted(k for k, r in res.items() if isinstance(r, dict)
                           and (r.get("pass") is False or r.get("degraded"))))


def not_clean(res: Dict[str, Any]) -> bool:
    """Any test of one GPU's diagnostic result failed or came back degraded."""
    return any(isinstance(r, dict) and (r.get("pass") is False or r.get("degraded")) for r in res.values())


HELD_NOTE = "below its failure line once on a shared PCIe path: measured again before it fails the GPU"


def _rate_only_failure(r: Dict[str, Any]) -> bool:
    """A rate test that failed on its rates alone: correct data, measured (not skipped)."""
    return r.get("pass") is False and not r.get("numerics") and "skipped" not in r and bool(r.get("rates"))


def apply_holds(res: Dict[str, Any]) -> None:
    """Publish a ``held`` test (``Agent._hold_unconfirmed``) that failed on rate alone as degraded, in place; run
    after every judgement of the result, which re-derives ``pass`` from the raw rates."""
    for r in res.values():
        if isinstance(r, dict) and r.get("held") and _rate_only_failure(r):
            r["pass"], r["degraded"] = True, True
            if HELD_NOTE not in (r.get("detail") or ""):
                r["detail"] = f"{r.get('detail') or ''}; {HELD_NOTE}".lstrip("; ")


def runtime_lost(res: Dict[str, Any]) -> Optional[str]:
    """The first detail when every test of one GPU's diagnostic result failed because the HIP runtime lost
    its devices, else None."""
    tests = [r for r in res.values() if isinstance(r, dict)]
    details = [str(r.get("detail", "")) for r in tests if r.get("pass") is False]
    if details and len(details) == len(tests) and all(any(m in d for m in _HIP_RUNTIME_LOST) for d in details):
        return details[0]
    return None


def fabric_abandoned(fab: Optional[Dict[str, Any]]) -> Optional[str]:
    """Why a node-level suite that returned had to give a test up at its deadline (an xGMI pair whose copies
    never completed, collectives aborted with ``ncclCommAbort``), else None.  What such a test leaves behind --
    copies still queued on a copy engine, the buffers they target, aborted communicators' memory -- stays
    with the process."""
    if not isinstance(fab, dict):
        return None
    p2p, rccl = fab.get("p2p"), fab.get("rccl")
    if isinstance(p2p, dict) and " hung" in str(p2p.get("stopped") or ""):
        return f"xGMI pair test abandoned: {p2p['stopped']}"[:200]
    if isinstance(rccl, dict) and rccl.get("aborted"):
        # at their deadline, or on a communicator's async error: either way ncclCommAbort ran and the buffers stay
        return f"RCCL collectives aborted: {rccl.get('detail') or ''}"[:200]
    return None


def misdirected(expected_bdf: str, meta: Any) -> Optional[str]:
    """Why a narrowed diagnostic child's result is not the expected GPU's (it reports the PCI address it ran on,
    agent/isolation.device_main), else None: a HIP visibility mapping that disagrees with the enumeration must not
    put one GPU's numbers under another's name."""
    got = normalize_bdf((meta or {}).get("bdf")) if isinstance(meta, dict) else ""
    if expected_bdf and got and got != normalize_bdf(expected_bdf):
        return f"diagnostic process ran on {got}, not {normalize_bdf(expected_bdf)}: HIP device visibility mismatch"
    return None


def normalize_bdf(bdf: Any) -> str:
    """PCI address in amd-smi's form (``0000:05:00.0``, lower case); a domain-less ``05:00.0`` gets 0000."""
    b = str(bdf or "").strip().lower()
    return "0000:" + b if b.count(":") == 1 else b


def report_digest(rep: Dict[str, Any]) -> str:
    """Stable digest of a report minus its volatile fields (timestamps, timings, temperature)."""
    import hashlib

    def strip(x: Any) -> Any:
        if isinstance(x, dict):
            return {k: strip(v) for k, v in x.items() if k not in _VOLATILE}
        if isinstance(x, list):
            return [strip(v) for v in x]
        if isinstance(x, float):
            return round(x, 0)  # measured rates: only a real change (>= 1 unit) counts
        return x
    return hashlib.sha256(json.dumps(strip(rep), sort_keys=True).encode()).hexdigest()


#: labels the agent maintains with ``--label-node`` (for nodeSelector / nodeAffinity and inventory)
NODE_LABELS = ("amd.com/mi355x-health", "amd.com/gpu.count", "amd.com/gpu.compute-partition",
               "amd.com/gpu.memory-partition", "amd.com/gpu.vbios", "amd.com/gpu.driver")


def label_value(v: Any) -> str:
    """A Kubernetes label value: at most 63 characters of ``[A-Za-z0-9._-]``, starting and ending
    alphanumeric (other characters dropped; the driver version amd-smi reports for an in-tree
    kernel driver is the whole uname string)."""
    s = "".join(c for c in str(v) if c.isascii() and (c.isalnum() or c in "._-"))[:63]
    while s and not s[0].isalnum():
        s = s[1:]
    while s and not s[-1].isalnum():
        s = s[:-1]
    return s


def node_labels(rep: Dict[str, Any], state: str) -> Dict[str, Optional[str]]:
    """The ``--label-node`` labels for a report: the verdict, the GPU count amd-smi sees, the partition
    modes (``mixed`` when the GPUs disagree), the VBIOS and the amdgpu driver; a value the probe cannot
    give removes the label (``None``)."""
    gpus = [g for g in rep.get("gpus") or [] if isinstance(g, dict) and not g.get("error")]

    def common(key: str) -> Optional[str]:
        vals = {str(g.get(key)) for g in gpus if g.get(key)}
        return None if not vals else ("mixed" if len(vals) > 1 else vals.pop())
    drv = rep.get("driver") if isinstance(rep.get("driver"), dict) else {}
    raw = {"amd.com/mi355x-health": state, "amd.com/gpu.count": str(len(rep.get("gpus") or [])),
           "amd.com/gpu.compute-partition": common("compute_partition"),
           "amd.com/gpu.memory-partition": common("memory_partition"),
           "amd.com/gpu.vbios": common("vbios_version"),
           "amd.com/gpu.driver": driver_release(drv.get("version")) if drv.get("version") else None}
    return {k: (label_value(v) or None) if v is not None else None for k, v in raw.items()}


def node_event(node: str, verdict: Verdict, previous: Optional[str], namespace: str = "default",
               now: Optional[float] = None) -> Dict[str, Any]:
    """A core/v1 Event on the Node for one verdict change -- what ``kubectl describe node`` and event
    exporters show.  Node events live in a namespace (``default``, as the kubelet's) with
    ``involvedObject.uid`` = the node name, the kubelet's convention that ``kubectl describe node``
    searches for besides the real UID."""
    ts = format_k8s_time(time.time() if now is None else now)
    if verdict.state == HEALTHY:
        msg = f"{verdict.gpus_ok}/{verdict.gpus_seen} MI355X GPUs healthy" + (f" (was {previous})" if previous else "")
    else:
        msg = "; ".join(verdict.reasons or verdict.warnings) or verdict.state
    return {"apiVersion": "v1", "kind": "Event",
            "metadata": {"generateName": f"{node}.mi355x-", "namespace": namespace},
            "involvedObject": {"apiVersion": "v1", "kind": "Node", "name": node, "uid": node},
            "reason": condition_reason(verdict.state), "message": msg[:1024],
            "type": "Normal" if verdict.state == HEALTHY else "Warning",
            "source": {"component": "mi355x-node-agent", "host": node},
            "reportingComponent": "mi355x-node-agent", "reportingInstance": node,
            "firstTimestamp": ts, "lastTimestamp": ts, "count": 1}


def token_node_name(token: Optional[str]) -> Optional[str]:
    """The node a pod-bound ServiceAccount token was issued for (its ``kubernetes.io.node.name`` claim, the one
    the API server exposes to admission as ``authentication.kubernetes.io/node-name``), None when the token has
    none or is not a JWT.  Read without verifying the signature: it only tells the agent which node the API
    server will let it write (deploy/agent-policy.yaml), so a mismatch with ``--node`` is caught at start-up."""
    import base64
    parts = (token or "").strip().split(".")
    if len(parts) != 3:
        return None
    try:
        claims = json.loads(base64.urlsafe_b64decode(parts[1] + "=" * (-len(parts[1]) % 4)))
        name = ((claims.get("kubernetes.io") or {}).get("node") or {}).get("name")
    except (ValueError, AttributeError, TypeError):
        return None
    return name if isinstance(name, str) and name else None


class ForeignNodeError(RuntimeError):
    """A write for a node other than the agent's own (``--node``): refused before it reaches the API server."""


class _OwnNodeClient:
    """The kube client as the agent may use it: every node-addressed call must name the agent's own node, and
    Events must be about it.  Defense in depth under deploy/agent-policy.yaml, which enforces the same on the
    API server side."""

    _NODE_CALLS = ("get_node", "patch_node_condition", "patch_node_annotations", "patch_node_labels",
                   "update_node_taints")

    def __init__(self, client: Any, node: str):
        self._client, self._node = client, node

    def __getattr__(self, name: str) -> Any:
        fn = getattr(self._client, name)
        if name in self._NODE_CALLS:
            def own(node: str, *a: Any, **kw: Any) -> Any:
                if node != self._node:
                    raise ForeignNodeError(f"refusing {name} on node {node!r}: this agent writes only {self._node!r}")
                return fn(node, *a, **kw)
            return own
        if name == "create_event":
            def event(namespace: str, ev: Dict[str, Any], *a: Any, **kw: Any) -> Any:
                obj = ev.get("involvedObject") or {}
                if obj.get("kind") != "Node" or obj.get("name") != self._node:
                    raise ForeignNodeError(f"refusing an Event about {obj.get('kind')} {obj.get('name')!r}: this "
                                           f"agent reports only on node {self._node!r}")
                return fn(namespace, ev, *a, **kw)
            return event
        return fn


class PublishError(RuntimeError):
    """Some of a publish's writes failed (message: which, and why); ``wrote`` is what did go out."""

    def __init__(self, message: str, wrote: Dict[str, bool]):
        super().__init__(message)
        self.wrote = wrote


def _annotation_gpu(g: Dict[str, Any]) -> Dict[str, Any]:
    """One GPU entry as the node annotation carries it (``Agent.annotation``)."""
    from ..models.node import DIAG_AGENT_ONLY
    out = {k: v for k, v in g.items() if k not in _ANNOTATION_DROP}
    diag = out.get("diag")
    if isinstance(diag, dict):
        out["diag"] = {t: ({k: v for k, v in r.items() if k not in DIAG_AGENT_ONLY} if isinstance(r, dict) else r)
                       for t, r in diag.items()}
    return out


def _fabric_suite(devices: List[int], timeout_s: Optional[float] = None, link: Optional[float] = None) -> Dict[str, Any]:
    """The node-level tests (``ops/diag.fabric_tests``): the xGMI pair matrix (pairs, then every source's fan to all
    its peers; ``link`` = one link's GB/s from amd-smi's training, the absolute floor's anchor) and the RCCL
    collectives, both under the watchdog's deadline -- the matrix within ``P2P_SHARE`` of it, the collectives
    within what is left up to 90 % -- so a hung copy or collective is given up, and named in the report,
    rather than left holding the fabric job."""
    from ..ops import diag
    try:
        res = diag.fabric_tests(devices, timeout_s=timeout_s or None, link=link)
    except Exception as e:  # the diag library itself is missing
        return {"p2p": {"pass": False, "detail": f"{type(e).__name__}: {e}"[:200]}}
    m, r = res.get("p2p") or {}, res.get("rccl") or {}
    out: Dict[str, Any] = {"p2p": {k: m[k] for k in ("pass", "median_gbps", "min_gbps", "floor_gbps", "link_gbps",
                                                     "detail", "wall_s", "stopped") if k in m}}
    if isinstance(m.get("fan"), dict):  # the fan's summary (its per-destination rows stay with mi355x-diag)
        out["p2p"]["fan"] = {k: v for k, v in m["fan"].items() if k != "to"}
    out["rccl"] = {k: r.get(k) for k in ("pass", "best_busbw_gbps", "best_busbw_by_op", "detail", "wall_s",
                                         "rccl", "aborted") if k in r or k not in ("aborted",)}
    return out


class Agent:
    _fabric_suite = staticmethod(_fabric_suite)

    def __init__(self, node: str, source: str = "auto", fixture: Optional[str] = None, diag_level: int = 0,
                 diag_interval: float = 3600.0, devices: Optional[List[int]] = None,
                 annotation_refresh: float = 900.0, heartbeat_interval: float = 300.0,
                 events: bool = True, event_namespace: str = "default", taint_unhealthy: bool = False,
                 diag_when: str = "idle", busy_vram_mb: int = 2048, busy_gfx_activity: int = 10,
                 diag_timeout: float = 300.0, ignore_pids: Sequence[int] = (),
                 expect_gpus: Optional[int] = None, expectations: Optional[HealthExpectations] = None,
                 pod_resources_socket: Optional[str] = None, gpu_resources: Sequence[str] = (PRIMARY_GPU_KEY,),
                 label_node: bool = False, annotation_encoding: str = "json", diag_parallel: int = DIAG_PARALLEL,
                 diag_baseline: bool = True, baseline_file: Optional[str] = None, isolation: str = "thread",
                 diag_setup: Optional[tuple] = None):
        self.node = node
        if isolation not in ISOLATION:
            raise ValueError(f"isolation must be one of {ISOLATION}")
        # where the HIP work runs (agent/isolation.py): "process" -- disposable children of a forkserver started
        # here, before this process calls amd-smi or HIP, so the agent itself never initialises HIP (the
        # DaemonSet); "thread" -- threads of this process (library use: the benchmark, tests scripting ops.diag)
        self.workers = Workers(isolation if diag_level > 0 else "thread", diag_setup)
        self.isolation = self.workers.mode
        # process isolation: HIP's device count and PCI addresses from the last enumeration child
        self._hip_view: Optional[Dict[str, Any]] = None
        # the last diagnostic child of each device (and "fabric"): pid, peak RSS, wall time (isolation._meta)
        self.diag_procs: Dict[Any, Dict[str, Any]] = {}
        if diag_parallel < 1:
            raise ValueError("diag_parallel must be >= 1")
        # at most this many per-device diagnostic threads at once (hung ones count: they still hold their GPU)
        self.diag_parallel = diag_parallel
        # "json" (readable with kubectl) or "gzip" (gz: + base64, ~12x smaller in every node LIST / watch)
        if annotation_encoding not in ("json", "gzip"):
            raise ValueError("annotation_encoding must be json or gzip")
        self.annotation_encoding = annotation_encoding
        self._gz_fallback_noted = False
        # --label-node: node_labels() kept on the Node, written when they change
        self.label_node = label_node
        self._labels: Optional[Dict[str, Optional[str]]] = None
        # the kubelet's PodResources socket: a GPU allocated to a pod is never diagnosed, even before the
        # pod touches it (None: not consulted; a missing socket falls back to the amd-smi heuristic)
        self.pod_resources_socket = pod_resources_socket
        self.gpu_resources = tuple(gpu_resources)
        self.pod_resources_state: Optional[str] = None
        # the verdict is taken against the GPU count the node registered (amd.com/gpu capacity /
        # allocatable, read from the Node object) unless --expect-gpus pins it; a GPU that fell off
        # the bus after the device plugin counted it then makes the node unhealthy at the source
        self.expect_gpus = expect_gpus
        self.node_gpus = 0
        self.expectations = expectations or HealthExpectations()
        self.source = source
        self.fixture = fixture
        self.diag_level = diag_level
        self.diag_interval = diag_interval
        self.devices = devices
        # active diagnostics run per GPU when its last run is `diag_interval` old and (diag_when=idle)
        # no workload holds it; a GPU found busy keeps its previous result and is tried again at the
        # next probe instead of a full interval later
        if diag_when not in DIAG_WHEN:
            raise ValueError(f"diag_when must be one of {DIAG_WHEN}")
        self.diag_when = diag_when
        self.busy_vram_mb = busy_vram_mb
        self.busy_gfx_activity = busy_gfx_activity
        # processes whose VRAM never makes a GPU busy: the agent itself and, for harnesses that start
        # the agent as a child of a GPU-holding process (a test runner), the PIDs given with --ignore-pid
        self.ignore_pids = frozenset((os.getpid(),) + tuple(int(p) for p in ignore_pids))
        self._diag_cache: Dict[int, Dict[str, Any]] = {}
        self._diag_at: Dict[int, float] = {}  # schedule: when the next run counts from (a recheck moves it back)
        self._diag_ran: Dict[int, float] = {}  # when the cached result was measured (reported as diag_at)
        self._diag_threads: Dict[int, _DiagRun] = {}  # device -> its diagnostic thread until it returns
        self._diag_done = threading.Event()  # set by every diagnostic thread as it returns
        self._rechecked: Dict[int, str] = {}  # device -> result_signature of the not-clean result rechecked
        # device -> {shared-resource test: "held" (its last run failed on rate alone, published degraded) or
        # "confirmed" (failed again: failures stand until it passes)}
        self._held: Dict[int, Dict[str, str]] = {}
        self._hip_count0: Optional[int] = None  # HIP device count the process saw first (runtime_lost)
        self._hip_ok: set = set()  # devices whose diagnostics ran without a runtime error in this process
        self._driver_version: Any = None  # amdgpu driver of the latest probe (the baselines' epoch)
        self.diag_timeout = diag_timeout
        self._diag_skipped: Dict[int, str] = {}
        # node-level findings of the last judgement (models/peers.judge_node): every GPU slow alike
        self.diag_findings: List[Dict[str, Any]] = []
        # per-GPU self-baselines of the diagnostics' rates (models/baseline.py); None: not kept
        self.baselines = Baselines(baseline_file) if diag_baseline else None
        # set when the HIP runtime lost its devices (runtime_lost): no further diagnostics in this process,
        # /healthz answers 503 so the liveness probe restarts the agent
        self.hip_lost: Optional[str] = None
        self._fabric: Optional[Dict[str, Any]] = None
        self._fabric_at = float("-inf")
        self._fabric_thread: Optional[_DiagRun] = None  # the node-level suite's thread until it returns
        # set when the node-level suite gave a test up at its deadline (fabric_abandoned): that suite is not run
        # again in this process, so what the abandoned test left queued and allocated is left once, not once per
        # --diag-interval; its failed result stays in the report until the agent is restarted
        self.fabric_abandoned: Optional[str] = None
        self.fabric_skipped: Optional[str] = None  # why the last node-level child left no result (killed from outside)
        self._bdf: Dict[int, str] = {}  # HIP ordinal -> PCI address (amd-smi and HIP enumerate independently)
        self.last: Optional[Dict[str, Any]] = None
        self.last_probe_done: Optional[float] = None  # monotonic time of the last completed probe (/healthz)
        self._last_condition: Optional[Dict[str, Any]] = None
        # the annotation (KBs per node, a new object revision per write) is rewritten only when the
        # report changed or every `annotation_refresh` s; the condition heartbeat goes out every probe
        self.annotation_refresh = annotation_refresh
        self._annotated: Optional[str] = None
        self._annotated_at = 0.0
        # the condition is re-sent on a verdict change at once, else every `heartbeat_interval` s (the
        # kubelet's own node-status report cadence is 5 min); the checker's --probe-max-age (15 min
        # default) must stay above it
        self.heartbeat_interval = heartbeat_interval
        self._cond_key: Optional[tuple] = None
        self._cond_at = 0.0
        # previous throttle-residency sample per GPU (bdf or index) -> (monotonic time, accumulators)
        self._acc_prev: Dict[str, Any] = {}
        # correctable ECC count history per GPU (bdf or index) -> [(monotonic time, count)], last CE_WINDOW_S
        self._ce_hist: Dict[str, List[Any]] = {}
        # remediation signals, both driven by verdict *changes*: an Event per change (advisory, never
        # repeated) and, opt-in, the UNHEALTHY_TAINT while unhealthy (retried until written)
        self.events = events
        self.event_namespace = event_namespace
        self.taint_unhealthy = taint_unhealthy
        self._verdict: Optional[Verdict] = None
        self._event_state: Optional[str] = None
        self._taint_state: Optional[str] = None
        self.lock = threading.Lock()

    @property
    def expected_gpus(self) -> int:
        """GPUs amd-smi must see: ``--expect-gpus`` when given, else the Node's ``amd.com/gpu`` (0: unknown)."""
        return self.expect_gpus if self.expect_gpus is not None else self.node_gpus

    def observe_node(self, node: Any) -> None:
        """Take the ``amd.com/gpu`` count from the agent's own Node object (GET, or a PATCH response)."""
        if not isinstance(node, dict):
            return
        status = node.get("status") or {}
        counts = [gpu_breakdown(status.get(k), (PRIMARY_GPU_KEY,)).get(PRIMARY_GPU_KEY, 0)
                  for k in ("capacity", "allocatable")]
        self.node_gpus = max(counts)

    def evaluate(self, rep: Dict[str, Any]) -> Verdict:
        return evaluate_report(rep, self.expected_gpus, self.expectations)

    def _entries_by_device(self, gpus: List[Dict[str, Any]], devices: List[int]) -> Dict[int, Dict[str, Any]]:
        """The probe entry of each HIP device: by PCI address, by index when HIP cannot say."""
        from ..ops import diag
        by_bdf = {normalize_bdf(g.get("bdf")): g for g in gpus if g.get("bdf")}
        out: Dict[int, Dict[str, Any]] = {}
        for d in devices:
            if d not in self._bdf:
                if self.workers.isolated:  # never a HIP call in this process: the enumeration child's answer
                    self._bdf[d] = normalize_bdf(((self._hip_view or {}).get("bdf") or {}).get(d, ""))
                else:
                    try:
                        self._bdf[d] = normalize_bdf(diag.device_info(d)["bdf"])
                    except Exception:
                        self._bdf[d] = ""
            g = by_bdf.get(self._bdf[d]) if self._bdf[d] else (gpus[d] if 0 <= d < len(gpus) else None)
            if g is not None:
                out[d] = g
        return out

    def _hip_devices(self, gpus: List[Dict[str, Any]], refresh: bool) -> Optional[int]:
        """HIP's device count: from ``ops.diag`` in this process (thread isolation), else from an enumeration child
        (re-run when ``refresh``, i.e. when a diagnostic may start) -- None with ``_diag_skipped`` filled when that
        child failed."""
        from ..ops import diag
        if not self.workers.isolated:
            return diag.device_count()
        if refresh or self._hip_view is None:
            view = self.workers.enumerate(min(60.0, max(5.0, self.diag_timeout)))
            if "count" in view:
                if self._hip_view is None or view.get("bdf") != self._hip_view.get("bdf"):
                    self._bdf = {}  # ordinals -> PCI addresses changed (or first seen): map them again
                self._hip_view = view
            else:
                for i in range(len(gpus)):
                    self._diag_skipped[i] = f"HIP device enumeration failed: {view.get('error')}"[:200]
                return None
        return int(self._hip_view["count"])

    def _diagnostics(self, gpus: List[Dict[str, Any]]) -> Dict[int, Dict[str, Any]]:
        self._diag_skipped = {}
        if self.diag_level <= 0:
            return {}
        from ..ops import diag
        isolated = self.workers.isolated
        now = time.time()
        # an enumeration child is worth its HIP start-up only when something may run this cycle
        candidates = self.devices if self.devices is not None else list(range(len(gpus)))
        maybe_due = any(now - self._diag_at.get(d, float("-inf")) >= self.diag_interval for d in candidates) or (
            self.diag_level >= 2 and now - self._fabric_at >= self.diag_interval)
        visible = self._hip_devices(gpus, refresh=maybe_due)
        if visible is None:
            return {d: self._diag_cache[d] for d in candidates if d in self._diag_cache}
        if self.devices is not None:
            visible = len(self.devices)
        if self._hip_count0 is None:
            self._hip_count0 = (diag.device_count() if not isolated else int(self._hip_view["count"])) \
                if self.devices is not None else visible
        elif not isolated and self.hip_lost is None and self.devices is None and visible != self._hip_count0:
            # HIP enumerates once per process: a count that moved is a driver reload or reset under the agent
            # (process isolation: every child enumerates afresh, so there is no stale runtime to lose)
            self.hip_lost = f"HIP device count changed from {self._hip_count0} to {visible}"
            print(f"{self.hip_lost}; diagnostics stop, /healthz fails so the agent is restarted", file=sys.stderr,
                  flush=True)
        if self.devices is None and gpus and visible == 0:
            # amd-smi sees GPUs but HIP sees none: a deployment fault (device files not mounted, wrong
            # container), said per GPU rather than silently running no diagnostics
            for i in range(len(gpus)):
                self._diag_skipped[i] = "no HIP device visible to the agent (/dev/kfd and /dev/dri mounted?)"
            return {}
        devices = self.devices if self.devices is not None else list(range(min(len(gpus), visible)))
        if self.devices is not None:
            # a configured ordinal HIP does not have is a configuration error of that device, said as such: run
            # on it, every call would fail with "invalid device ordinal", which is neither the GPU's fault nor a
            # lost runtime
            count = self._hip_count0 if not isolated else int(self._hip_view["count"])
            for d in [d for d in devices if not 0 <= d < count]:
                self._diag_skipped[d] = f"device {d} is not a HIP device of the agent ({count} visible): check --devices"
            devices = [d for d in devices if 0 <= d < count]
        entries = self._entries_by_device(gpus, devices)
        due = [d for d in devices if now - self._diag_at.get(d, float("-inf")) >= self.diag_interval]
        fabric_busy = self._fabric_thread is not None and self._fabric_thread.is_alive()
        if fabric_busy and due:
            # a node-level suite that outlived its watchdog still holds every GPU (a collective's kernels stay
            # queued): per-GPU tests would contend with it or queue behind it and muddy their own verdict
            for d in due:
                self._diag_skipped[d] = ("node-level xGMI/RCCL tests still running past their watchdog: per-GPU "
                                         "diagnostics wait")
            due = []
        allocated = self._allocated() if due and self.diag_when == "idle" else None
        unmatched = self._unmatched_allocations(allocated, entries, devices) if allocated else None
        run = []
        for d in due:
            why = unmatched
            if why is None and allocated:
                owner = allocated.get(normalize_bdf((entries.get(d) or {}).get("bdf") or self._bdf.get(d, "")))
                if owner:
                    why = f"allocated to pod {owner}"
            if why is None and self.diag_when == "idle":
                why = gpu_busy(entries.get(d) or {}, self.ignore_pids, self.busy_vram_mb, self.busy_gfx_activity)
            if why:
                self._diag_skipped[d] = why
            else:
                run.append(d)
        # one job per GPU, at most `diag_parallel` at once: a child process each (process isolation) or a thread
        # each whose ctypes calls release the GIL -- either way every device is driven at once, so an 8-GPU node is
        # checked in the time of one GPU and a 64-partition CPX node in 8 waves.  A GPU whose diagnostic outlives
        # `diag_timeout` s is reported failed instead of freezing the agent into a stale report: its child is
        # SIGKILLed (freeing its slot and its GPU); a thread cannot be, so nothing new starts on that GPU while it
        # lives, and /healthz fails once it has outlived HUNG_RESTART_FACTOR x diag_timeout (hung_diagnostic).
        queue = [d for d in run if d not in self._diag_threads] if self.hip_lost is None else []
        memory_partition = {d: (entries.get(d) or {}).get("memory_partition") for d in queue}
        power = {d: power_fraction(entries.get(d) or {}) for d in queue}
        host = self.workers.host_lock() if queue else (None, None)
        while True:
            self._diag_done.clear()
            while queue and sum(r.is_alive() for r in self._diag_threads.values()) < self.diag_parallel:
                d = queue.pop(0)
                self._start_diag(d, memory_partition.get(d), power.get(d), host)
            if isolated:
                for r in self._diag_threads.values():
                    if not r.job.killed and r.is_alive() and time.monotonic() >= r.mono + self.diag_timeout:
                        r.job.kill()  # its slot frees (unless the child is stuck in the driver)
            waiting = [r for r in self._diag_threads.values()
                       if r.is_alive() and time.monotonic() < r.mono + self.diag_timeout]
            if not waiting and not (queue and isolated and
                                    sum(r.is_alive() for r in self._diag_threads.values()) < self.diag_parallel):
                break
            if waiting:
                self._diag_done.wait(max(0.0, min(min(r.mono for r in waiting) + self.diag_timeout - time.monotonic(),
                                                  1.0)))
        for d in queue:  # every slot is held by a diagnostic that outlived its watchdog
            self._diag_skipped[d] = (f"waiting for a diagnostic slot: {self.diag_parallel} of {self.diag_parallel} "
                                     "held by hung diagnostics")
        finished: Dict[int, Dict[str, Any]] = {}
        for d, r in list(self._diag_threads.items()):
            if "meta" in r.box:
                self.diag_procs[d] = r.box["meta"]
            if not r.is_alive():
                del self._diag_threads[d]
                if r.box.get("external_kill"):
                    # SIGKILLed from outside the agent (the pod's memory limit?): not this GPU's finding -- its last
                    # results stand, the report says why there is no new one, and the next cycle diagnoses it again
                    self._diag_skipped[d] = r.box["external_kill"][:200]
                    self._diag_at[d] = float("-inf")
                    continue
                wrong = misdirected(self._bdf.get(d, ""), r.box.get("meta"))
                if r.job.killed:
                    finished[d] = {"watchdog": {
                        "pass": False, "detail": f"diagnostics did not finish within {self.diag_timeout:g} s (GPU "
                                                 f"hang?): diagnostic process {r.job.pid} killed"}}
                elif wrong:
                    finished[d] = {"run": {"pass": False, "detail": wrong}}
                elif "res" in r.box:
                    finished[d] = r.box["res"]
                self._diag_at[d] = r.started
            else:
                stuck = f": diagnostic process {r.job.pid} did not exit after SIGKILL" if r.job.killed else ""
                self._diag_cache[d] = {"watchdog": {
                    "pass": False,
                    "detail": f"diagnostics did not finish within {self.diag_timeout:g} s (GPU hang?){stuck}"}}
                self._diag_ran[d] = r.started
                self._diag_at[d] = r.started
        lost_devs = {d: runtime_lost(res) for d, res in finished.items()} if not isolated else {}
        lost_devs = {d: why for d, why in lost_devs.items() if why is not None}
        if lost_devs and self.hip_lost is None:
            # the HIP runtime, not a GPU, is gone only when
            # * the device count changed under the process, or
            # * a device that ran fine earlier in this process now fails that way (a driver reload under a running
            #   agent: whatever else is busy or rescheduled, a GPU HIP served before is refused now), or
            # * every device of the node (two or more) failed that way together.
            # Devices that never ran fine here -- two broken GPUs rechecked on their own (DIAG_RECHECK_S) while the
            # others passed, or the only idle ones of a busy node -- are those GPUs' failures and stay in their
            # verdicts: restarting the agent for them would only loop, diagnosing the same GPUs after every start.
            # (Process isolation: each child's runtime is fresh, so such an error there is the device's own.)
            now_count = diag.device_count()
            whole_node = len(lost_devs) >= 2 and set(lost_devs) >= set(devices)
            was_fine = any(d in self._hip_ok for d in lost_devs)
            if (self._hip_count0 is not None and now_count != self._hip_count0) or whole_node or was_fine:
                lost = next(iter(lost_devs.values()))
                print(f"HIP runtime lost its devices ({lost}); diagnostics stop, /healthz fails so the "
                      "agent is restarted", file=sys.stderr, flush=True)
                self.hip_lost = lost
        self._hip_ok.update(d for d in finished if d not in lost_devs)
        fresh = []
        for d, res in finished.items():
            if self.hip_lost is not None and d in lost_devs:
                continue
            self._hold_unconfirmed(d, res)
            self._diag_cache[d] = res
            self._diag_ran[d] = self._diag_at[d]
            fresh.append(d)
        self._judge_diagnostics(devices, entries, fresh)
        for d in fresh:
            res = self._diag_cache[d]
            started = self._diag_ran[d]
            sig = result_signature(res) if not_clean(res) else ""
            if sig and sig != self._rechecked.get(d) and self.diag_interval > DIAG_RECHECK_S:
                # a slow or failed result is measured again after DIAG_RECHECK_S instead of a whole interval
                # later: a one-off (a burst of power management) clears before the 30-minute degraded alert, a
                # real fault is confirmed -- once; the same result again goes back to the full interval
                self._diag_at[d] = started - self.diag_interval + DIAG_RECHECK_S
                self._rechecked[d] = sig
            elif not sig:
                self._rechecked.pop(d, None)
        if self.hip_lost is not None:
            for d in devices:
                self._diag_skipped[d] = f"HIP runtime lost its devices ({self.hip_lost[:120]}): agent restart pending"
        # a GPU whose last diagnostic hung (its child killed, or its thread still stuck) would take the node-level
        # suite down with it: that waits for a cycle in which every GPU came back
        hung_gpu = any("watchdog" in (self._diag_cache.get(d) or {}) for d in devices)
        if (self.diag_level >= 2 and self.devices is None and len(devices) >= 2 and not self._diag_skipped
                and not self._diag_threads and not hung_gpu and self._fabric_thread is None
                and self.fabric_abandoned is None and now - self._fabric_at >= self.diag_interval):
            # node-level: every ordered GPU pair over xGMI (after the per-GPU tests, so no contention) and the
            # RCCL collectives; it touches every GPU, so it waits until none is busy.  Under the same watchdog as
            # the per-GPU tests: a collective that never completes (a link that stopped passing traffic) is a
            # failed fabric, not a frozen agent.
            done = threading.Event()
            # the absolute floor's link rate: the median GPU's trained xGMI link (amd-smi), so one GPU whose links
            # trained down is judged against its hive's links, not the other way round
            links = sorted(diag.link_gbs(g.get("xgmi_width"), g.get("xgmi_speed_gbps"))
                           for g in (entries.get(d) or {} for d in devices))
            suite = functools.partial(_fabric_suite, link=links[len(links) // 2] if links else None)
            job = self.workers.fabric(suite, devices, self.diag_timeout, done)
            self._fabric_thread = _DiagRun(job, now, time.monotonic())
        if self._fabric_thread is not None:
            r = self._fabric_thread
            deadline = r.mono + self.diag_timeout
            while r.is_alive() and time.monotonic() < deadline:
                time.sleep(min(0.05, max(0.0, deadline - time.monotonic())))
            if isolated and r.is_alive() and not r.job.killed:
                r.job.kill()
            self._fabric_at = r.started
            if "meta" in r.box:
                self.diag_procs["fabric"] = r.box["meta"]
            if not r.is_alive() and r.box.get("external_kill"):
                # as for a GPU's child: not the fabric's finding; the last result stands, retried next cycle
                self._fabric_thread = None
                self._fabric_at = float("-inf")
                self.fabric_skipped = r.box["external_kill"][:200]
            elif not r.is_alive():
                self._fabric_thread = None
                self.fabric_skipped = None
                if r.job.killed:
                    self._fabric = {"watchdog": {
                        "pass": False, "detail": f"node-level xGMI/RCCL tests did not finish within "
                                                 f"{self.diag_timeout:g} s (fabric hang?): diagnostic process "
                                                 f"{r.job.pid} killed"}}
                else:
                    self._fabric = r.box.get("res")
                why = fabric_abandoned(self._fabric) if not isolated else None
                if why:
                    # an abandoned test's queued copies and aborted communicators stay with this process (thread
                    # isolation); in a child they ended with it, so the suite simply runs again next interval
                    self.fabric_abandoned = why
                    for res in self._fabric.values():
                        if isinstance(res, dict) and res.get("pass") is False:
                            res["retest"] = "not re-run in this process: restart the agent to re-test"
                    print(f"{why}; the node-level tests are not re-run until the agent restarts", file=sys.stderr,
                          flush=True)
            else:
                stuck = f": diagnostic process {r.job.pid} did not exit after SIGKILL" if r.job.killed else ""
                self._fabric = {"watchdog": {
                    "pass": False,
                    "detail": f"node-level xGMI/RCCL tests did not finish within {self.diag_timeout:g} s (fabric "
                              f"hang?){stuck}"}}
        return {d: self._diag_cache[d] for d in devices if d in self._diag_cache}

    def _hold_unconfirmed(self, d: int, res: Dict[str, Any]) -> None:
        """A test of a resource the GPU shares with the host's other GPUs and processes (``ops/diag.SHARED_TESTS``:
        the PCIe host link, through the CPU's root complex) that fails on its rate alone is contention as often as a
        fault.  Its first such failure is marked ``held`` -- published as *degraded* (:func:`apply_holds`, after
        every judgement) and measured again after ``DIAG_RECHECK_S`` (the not-clean recheck); a second one in a row
        fails the GPU, and so does every one after it until the test passes.  A link that trained down is the probe's
        finding at once (amd-smi's PCIe width and speed)."""
        from ..ops import diag
        state = self._held.setdefault(d, {})
        for t in diag.SHARED_TESTS:
            r = res.get(t)
            if not isinstance(r, dict):
                continue
            if not _rate_only_failure(r):
                state.pop(t, None)  # passed (or failed on its data): the next rate-only failure is held again
            elif t not in state:
                state[t] = "held"
                r["held"] = HELD_NOTE
            else:
                state[t] = "confirmed"  # the second in a row and every one after it until a pass: failures

    def _judge_diagnostics(self, devices: List[int], entries: Dict[int, Dict[str, Any]], fresh: List[int]) -> None:
        """Judge the GPUs' latest diagnostic results together (``models/peers.judge_node``): each rate against the
        node's other GPUs measured within ``PEER_MAX_AGE_S`` (a lone GPU against the references), a shortfall
        every GPU shares as one node-level finding (``self.diag_findings``).  Fresh results also update their
        GPU's self-baseline (``models/baseline.py``), whose drift notes the judgement then includes."""
        from ..models import peers
        now = time.time()
        pool = {d: self._diag_cache[d] for d in devices
                if d in self._diag_cache and now - self._diag_ran.get(d, float("-inf")) <= PEER_MAX_AGE_S}
        label = {d: f"gpu{(entries.get(d) or {}).get('index', d)}" for d in pool}
        self.diag_findings = peers.judge_node(pool, label)
        if self.baselines is not None and fresh:
            for d in fresh:
                key = baseline_key(entries.get(d) or {}, self._bdf.get(d, ""), d)
                # the software the rates were measured under: a driver or firmware change re-forms the baseline
                self.baselines.observe(key, self._diag_cache[d], now, epoch_of(entries.get(d), self._driver_version))
            self.diag_findings = peers.judge_node(pool, label)
        for res in pool.values():  # after the last judgement, which re-derives pass from the rates
            apply_holds(res)

    def _start_diag(self, d: int, memory_partition: Any, power: Optional[float], host: tuple = (None, None)) -> None:
        """Start device ``d``'s diagnostics as its own job (the partition's memory share comes from amd-smi's NPS
        mode, CUs and VRAM from HIP; a lowered power cap scales the compute references)."""
        kw: Dict[str, Any] = {"memory_partition": memory_partition}
        if power is not None and power < 1.0:
            kw["power_fraction"] = power
        # the host-link turn is waited for only within this device's watchdog (a GPU stuck in its turn is that
        # GPU's hang, not every GPU's); CLOCK_MONOTONIC is one clock for the agent and its children
        kw["deadline"] = time.monotonic() + 0.9 * self.diag_timeout
        job = self.workers.device(self.diag_level, d, kw, self._diag_done, host)
        self._diag_threads[d] = _DiagRun(job, time.time(), time.monotonic())

    def _unmatched_allocations(self, allocated: Dict[str, str], entries: Dict[int, Dict[str, Any]],
                               devices: List[int]) -> Optional[str]:
        """Fail safe for device IDs the agent cannot map: the kubelet reports a GPU allocated to a pod whose ID is
        not a PCI address of this node's devices (a device plugin that names partitions by another scheme, a DRA
        claim keyed by driver/pool/device).  That allocation may be any of the GPUs, so none is diagnosed -- even
        when other allocations do map (the reason, else None)."""
        local = {normalize_bdf((entries.get(d) or {}).get("bdf") or self._bdf.get(d, "")) for d in devices}
        local.discard("")
        unmapped = sorted(k for k in allocated if k not in local)
        if not local or not unmapped:
            return None
        sample = ", ".join(unmapped[:3])
        return (f"kubelet reports {len(unmapped)} allocated GPU device(s) ({sample}) matching no local PCI "
                "address: not diagnosing any GPU")

    def hung_diagnostic(self, now: Optional[float] = None) -> Optional[str]:
        """Why /healthz must fail: a diagnostic thread alive for HUNG_RESTART_FACTOR x diag_timeout (its watchdog
        verdict was published at 1x); None when nothing is hung that long."""
        if self.workers.isolated:
            # a child past its watchdog was SIGKILLed and its GPU reported failed; one the kernel cannot end (stuck
            # in the driver) would survive a restart of the agent as well, so it is reported, not restarted for
            return None
        now = time.monotonic() if now is None else now
        limit = HUNG_RESTART_FACTOR * self.diag_timeout
        runs = [(f"gpu{d} diagnostics", r) for d, r in list(self._diag_threads.items())]
        fab = self._fabric_thread
        if fab is not None:
            runs.append(("node-level xGMI/RCCL tests", fab))
        for what, r in runs:
            age = now - r.mono
            if r.is_alive() and age >= limit:
                return f"{what} running for {age:.0f} s (> {HUNG_RESTART_FACTOR:g} x --diag-timeout): restart to free the GPU"
        return None

    def _allocated(self) -> Optional[Dict[str, str]]:
        """Devices the kubelet allocated to pods (normalised BDF -> "ns/pod"), or None when unknown."""
        if not self.pod_resources_socket:
            return None
        from ..kube import podresources
        try:
            got = podresources.allocated_devices(self.pod_resources_socket, self.gpu_resources)
        except podresources.PodResourcesError as e:
            state = f"error: {e}"[:200]
            if state != self.pod_resources_state:
                print(f"kubelet PodResources unavailable, using the amd-smi busy heuristic: {e}", file=sys.stderr,
                      flush=True)
            self.pod_resources_state = state
            return None
        self.pod_resources_state = "absent" if got is None else "ok"
        return None if got is None else {normalize_bdf(k): v for k, v in got.items()}

    def probe_once(self) -> Dict[str, Any]:
        from ..ops.amdsmi_probe import SCHEMA, probe
        try:
            rep = probe(self.node, self.source, self.fixture)
        except Exception as e:  # a probe that cannot run is an unknown verdict, published, not a crash loop
            rep = {"schema": SCHEMA, "node": self.node, "ts": time.time(), "gpus": [],
                   "error": f"probe: {type(e).__name__}: {e}"[:300]}
        self._throttle_windows(rep)
        self._ce_rates(rep)
        drv = rep.get("driver")
        self._driver_version = drv.get("version") if isinstance(drv, dict) else None
        gpus = rep.get("gpus") or []
        diags = self._diagnostics(gpus)
        if diags or self._diag_skipped:
            entries = self._entries_by_device(gpus, sorted(set(diags) | set(self._diag_skipped)))
            for d, g in entries.items():
                if diags.get(d):
                    g["diag"] = diags[d]
                    g["diag_at"] = round(self._diag_ran.get(d, 0.0), 1)  # when it ran (a busy GPU's result ages)
                    if d in self.diag_procs:  # process isolation: the child that measured it (pid, peak RSS)
                        g["diag_proc"] = self.diag_procs[d]
                if d in self._diag_skipped:
                    g["diag_skipped"] = self._diag_skipped[d]
            if self._fabric:
                rep["fabric"] = self._fabric
            if self.diag_findings:
                rep["diag_node"] = {"findings": self.diag_findings}
        if self.fabric_skipped:  # the node-level child was killed from outside the agent: no new result, and why
            rep["fabric_skipped"] = self.fabric_skipped
        if self.pod_resources_state is not None:
            rep["pod_resources"] = self.pod_resources_state
        verdict = self.evaluate(rep)
        rep["state"] = verdict.state
        if self.expected_gpus:
            rep["expected_gpus"] = self.expected_gpus
        with self.lock:
            self.last = rep
            self.last_probe_done = time.monotonic()
        return rep

    def _ce_rates(self, rep: Dict[str, Any], now: Optional[float] = None) -> None:
        """``gpus[i].ecc_ce_per_h``: correctable ECC errors per hour over the agent's probes of the last
        hour (once they span ``CE_MIN_SPAN_S``); a counter that went down (driver reload) restarts it."""
        now = time.monotonic() if now is None else now
        for g in rep.get("gpus") or []:
            ce = g.get("ecc_correctable")
            if not isinstance(ce, int) or isinstance(ce, bool):
                continue
            key = str(g.get("bdf") or g.get("index"))
            hist = self._ce_hist.setdefault(key, [])
            if hist and ce < hist[-1][1]:
                hist.clear()
            hist.append((now, ce))
            while len(hist) > 2 and now - hist[1][0] >= CE_WINDOW_S:
                hist.pop(0)  # keep the newest sample that is at least a window old as the baseline
            span = now - hist[0][0]
            if span >= CE_MIN_SPAN_S:
                g["ecc_ce_per_h"] = round((ce - hist[0][1]) * 3600.0 / span, 1)

    def _throttle_windows(self, rep: Dict[str, Any]) -> None:
        """Turn the firmware's since-boot throttle accumulators into the share of the time since the
        previous probe spent throttled (``gpus[i].throttle``; models/health.throttle_window)."""
        now = time.monotonic()
        for g in rep.get("gpus") or []:
            acc = g.get("throttle_acc")
            if not isinstance(acc, dict):
                continue
            key = str(g.get("bdf") or g.get("index"))
            prev = self._acc_prev.get(key)
            if prev is not None:
                win = throttle_window(prev[1], acc, now - prev[0])
                if win is not None:
                    g["throttle"] = win
            self._acc_prev[key] = (now, acc)

    def annotation(self, rep: Dict[str, Any]) -> Dict[str, str]:
        """The report as the node annotation, minus the raw counters (xGMI traffic, throttle accumulators,
        per-process VRAM, per-GPU probe time): every client that LISTs or watches nodes receives the
        annotation, it is rewritten only when the health content changes, so those would only be stale
        bytes there; they stay on ``/probe`` and ``/metrics``.  The diagnostics' per-XCD/CU maps, burn-in rows
        and wall times stay there too (``models/node.DIAG_AGENT_ONLY``): the checker judges from the rest, and
        at fleet scale parsing them was a third of a report-reading check."""
        gpus = [_annotation_gpu(g) if isinstance(g, dict) else g for g in rep.get("gpus") or []]
        doc = dict(rep, gpus=gpus)
        value = encode_annotation(doc, self.annotation_encoding)
        if len(value) > ANNOTATION_JSON_MAX and self.annotation_encoding == "json":
            # a node's annotations share 256 KiB; a CPX node's 64 processors at level 2 come near that as
            # JSON, so an oversized report goes out gzip-encoded (the checker reads both) instead of being
            # rejected
            if not self._gz_fallback_noted:
                print(f"report annotation is {len(value)} bytes as JSON: writing it gzip-encoded", file=sys.stderr,
                      flush=True)
                self._gz_fallback_noted = True
            value = encode_annotation(doc, "gzip")
        return {HEALTH_ANNOTATION: value}

    def condition(self, rep: Dict[str, Any]) -> Dict[str, Any]:
        v = self.evaluate(rep)
        cond = condition_for(v, previous=self._last_condition)
        self._last_condition = cond
        self._verdict = v
        return cond

    def publish_annotation(self, client: Any, rep: Dict[str, Any]) -> None:
        _OwnNodeClient(client, self.node).patch_node_annotations(self.node, self.annotation(rep))

    def publish(self, client: Any, rep: Dict[str, Any], force: bool = False) -> Dict[str, bool]:
        """Full report as annotation when it changed (or every ``annotation_refresh`` s), verdict as the
        ``AMDGPUHealthy`` NodeCondition when it changed (or every ``heartbeat_interval`` s), and on a
        verdict change an Event and (``taint_unhealthy``) the taint.  Returns what was written."""
        if rep.get("node") is not None and rep.get("node") != self.node:
            # a report of another node (a misrouted or replayed one) must never become this node's verdict
            raise ForeignNodeError(f"report is for node {rep.get('node')!r}; this agent publishes only for "
                                   f"{self.node!r}")
        if not isinstance(client, _OwnNodeClient):
            client = _OwnNodeClient(client, self.node)
        digest = report_digest(rep)
        now = time.monotonic()
        wrote = {"annotation": False, "condition": False, "event": False, "taint": False, "labels": False}
        # each write stands alone: a rejected annotation (e.g. the node's 256 KiB annotation budget) or
        # label/taint PATCH must not stop the condition heartbeat the checker gates on.  A failed write
        # keeps its old state, so it is retried at the next publish; the errors are raised together at
        # the end for the caller to log.
        errors: List[str] = []

        def attempt(what: str, fn: Any) -> None:
            try:
                fn()
            except Exception as e:
                errors.append(f"{what}: {e}")
        if force or digest != self._annotated or now - self._annotated_at >= self.annotation_refresh:
            def annotate() -> None:
                client.patch_node_annotations(self.node, self.annotation(rep))
                self._annotated, self._annotated_at = digest, now
                wrote["annotation"] = True
            attempt("annotation", annotate)
        cond = self.condition(rep)
        key = (cond.get("status"), cond.get("reason"), cond.get("message"))
        if force or key != self._cond_key or now - self._cond_at >= self.heartbeat_interval:
            def heartbeat() -> None:
                self.observe_node(client.patch_node_condition(self.node, cond))  # the response is the Node
                self._cond_key, self._cond_at = key, now
                wrote["condition"] = True
            attempt("condition", heartbeat)
        v = self._verdict
        if v is not None and self.label_node:
            labels = node_labels(rep, v.state)
            if labels != self._labels:
                def relabel() -> None:
                    client.patch_node_labels(self.node, labels)
                    self._labels = labels
                    wrote["labels"] = True
                attempt("labels", relabel)
        if v is not None and self.events and v.state != self._event_state:
            prev, self._event_state = self._event_state, v.state
            if prev is not None or v.state != HEALTHY:  # an agent (re)starting on a healthy node is no news
                wrote["event"] = self._post_event(client, v, prev)
        # UNKNOWN (probe failed) leaves the taint as it is: a flaky probe must not flap scheduling
        if v is not None and self.taint_unhealthy and v.state != UNKNOWN and v.state != self._taint_state:
            def taint() -> None:
                wrote["taint"] = self._sync_taint(client, v.state == UNHEALTHY)
                self._taint_state = v.state
            attempt("taint", taint)
        if errors:
            raise PublishError("; ".join(errors), wrote)
        return wrote

    def _post_event(self, client: Any, verdict: Verdict, previous: Optional[str]) -> bool:
        try:
            client.create_event(self.event_namespace,
                                node_event(self.node, verdict, previous, self.event_namespace))
            return True
        except Exception as e:  # advisory: a missing RBAC rule must not stop the condition heartbeat
            print(f"node event post failed: {e}", file=sys.stderr, flush=True)
            return False

    def _sync_taint(self, client: Any, want: bool) -> bool:
        """Add (``want``) or remove UNHEALTHY_TAINT, keeping every other taint; True if a write happened.
        On the first publish this also clears a taint left behind by a previous agent instance."""
        key = UNHEALTHY_TAINT["key"]

        def edit(taints: List[Dict[str, Any]]) -> Optional[List[Dict[str, Any]]]:
            if any(t.get("key") == key for t in taints) == want:
                return None
            return taints + [dict(UNHEALTHY_TAINT)] if want else [t for t in taints if t.get("key") != key]
        return client.update_node_taints(self.node, edit) is not None


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="k8s-gpu-node-agent", description="MI355X node agent (probe + publish)")
    ap.add_argument("--node", default=os.environ.get("NODE_NAME") or socket.gethostname())
    ap.add_argument("--source", choices=("auto", "native", "python", "fixture"), default="auto")
    ap.add_argument("--fixture", help="recorded probe report (source=fixture)")
    ap.add_argument("--interval", type=float, default=60.0)
    ap.add_argument("--diag-level", type=int, default=0, choices=(0, 1, 2))
    ap.add_argument("--diag-interval", type=float, default=3600.0)
    ap.add_argument("--publish", default="annotation", help="comma list of annotation,http,stdout")
    ap.add_argument("--listen", default="0.0.0.0:9464")
    ap.add_argument("--kubeconfig")
    ap.add_argument("--once", action="store_true")
    ap.add_argument("--annotation-refresh", type=float, default=900.0,
                    help="rewrite an unchanged report annotation at most this often (s)")
    ap.add_argument("--heartbeat-interval", type=float, default=300.0,
                    help="re-send an unchanged AMDGPUHealthy condition this often (s); keep it below the "
                         "checker's --probe-max-age")
    ap.add_argument("--no-events", dest="events", action="store_false",
                    help="do not post a Kubernetes Event on the node when its verdict changes")
    ap.add_argument("--event-namespace", default="default", help="namespace of the node Events (default: default)")
    ap.add_argument("--taint-unhealthy", action="store_true",
                    help=f"keep the taint {UNHEALTHY_TAINT['key']}={UNHEALTHY_TAINT['value']}:"
                         f"{UNHEALTHY_TAINT['effect']} on the node while it is unhealthy (removed on recovery)")
    ap.add_argument("--diag-when", choices=DIAG_WHEN, default="idle",
                    help="idle (default): run the active diagnostics only on GPUs no workload holds (a busy GPU "
                         "keeps its last result and is retried at the next probe); always: on schedule")
    ap.add_argument("--busy-vram-mb", type=int, default=2048,
                    help="a process other than the agent holding this much VRAM makes its GPU busy (default 2048)")
    ap.add_argument("--diag-timeout", type=float, default=300.0,
                    help="a GPU whose diagnostics run longer than this (s) is reported failed (hung); default 300")
    ap.add_argument("--diag-isolation", choices=ISOLATION, default="process",
                    help="process (default): each cycle's HIP diagnostics run in disposable child processes, so the "
                         "agent never initialises HIP, a hung one is SIGKILLed at --diag-timeout and a GPU fault "
                         "ends only its child; thread: in the agent process (a hung HIP call then needs a restart, "
                         "/healthz)")
    ap.add_argument("--diag-parallel", type=int, default=DIAG_PARALLEL, metavar="N",
                    help=f"per-device diagnostic threads at once (default {DIAG_PARALLEL}: an SPX node's GPUs together, "
                         "a CPX node's 64 partitions in waves); tests on shared host resources (the PCIe host link) "
                         "run one device at a time whatever N is")
    ap.add_argument("--ignore-pid", type=int, action="append", default=[], metavar="PID",
                    help="a process whose VRAM never makes a GPU busy (repeatable; e.g. the harness that "
                         "started the agent). The agent's own PID is always ignored")
    ap.add_argument("--expect-gpus", type=int, default=None, metavar="N",
                    help="GPUs amd-smi must see on this node (default: the Node's amd.com/gpu capacity)")
    ap.add_argument("--xgmi-links", type=int, default=XGMI_LINKS_EXPECTED, metavar="N",
                    help=f"xGMI links that must be Up per GPU (default {XGMI_LINKS_EXPECTED}: 8-GPU hive; "
                         "0 disables the check)")
    ap.add_argument("--pod-resources-socket", default=None, metavar="PATH",
                    help="kubelet PodResources socket (e.g. /var/lib/kubelet/pod-resources/kubelet.sock): GPUs "
                         "allocated to pods are never diagnosed; without it (or when absent) only the amd-smi "
                         "busy heuristic applies")
    ap.add_argument("--gpu-resource", action="append", default=None, metavar="NAME",
                    help=f"extended resource whose kubelet allocations mark GPUs busy (repeatable; default "
                         f"{PRIMARY_GPU_KEY})")
    ap.add_argument("--annotation-encoding", choices=("json", "gzip"), default="json",
                    help="report annotation as JSON (readable with kubectl) or gz: + base64(gzip(JSON)), "
                         "~12x smaller in every node LIST and watch event (the checker reads both)")
    ap.add_argument("--tls-cert-file", default=None, metavar="PEM",
                    help="serve the HTTP port over TLS with this certificate (with --tls-key-file)")
    ap.add_argument("--tls-key-file", default=None, metavar="PEM")
    ap.add_argument("--tls-client-ca", default=None, metavar="PEM",
                    help="with TLS: /probe, /metrics and /status need a client certificate signed by this CA "
                         "(the checker's --probe-client-cert, Prometheus' tlsConfig); /healthz stays open for "
                         "the kubelet's probe")
    ap.add_argument("--label-node", action="store_true",
                    help="keep node labels " + ", ".join(NODE_LABELS) + " current (verdict, GPU count, partition "
                         "modes, VBIOS, driver) for nodeSelector / nodeAffinity")
    ap.add_argument("--busy-gfx-activity", type=int, default=10,
                    help="graphics-engine activity (%%) at which a GPU counts as busy (default 10)")
    ap.add_argument("--diag-baseline-file", default=None, metavar="PATH",
                    help="keep each GPU's self-baseline of the diagnostics' rates (its first clean runs) in this "
                         "JSON file across restarts (default: in memory only)")
    ap.add_argument("--no-diag-baseline", dest="diag_baseline", action="store_false",
                    help="do not keep per-GPU self-baselines (no drift warnings)")
    ap.add_argument("--diag-baseline-reset", default=None, metavar="GPUS",
                    help="at start, forget the self-baselines of these GPUs (comma-separated amd-smi UUIDs or PCI "
                         "addresses, or 'all'): they re-form from their next clean runs (after a planned change, "
                         "e.g. a lower power cap; a driver or firmware change re-forms them by itself).  A running "
                         "agent takes POST /baseline/reset[?gpu=...] from inside its pod (kubectl port-forward)")
    return ap


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(argv)
    pubs = set(args.publish.split(","))
    agent = Agent(args.node, args.source, args.fixture, args.diag_level, args.diag_interval,
                  annotation_refresh=args.annotation_refresh, heartbeat_interval=args.heartbeat_interval,
                  events=args.events, event_namespace=args.event_namespace, taint_unhealthy=args.taint_unhealthy,
                  diag_when=args.diag_when, busy_vram_mb=args.busy_vram_mb,
                  busy_gfx_activity=args.busy_gfx_activity, diag_timeout=args.diag_timeout,
                  ignore_pids=args.ignore_pid, expect_gpus=args.expect_gpus,
                  expectations=HealthExpectations(xgmi_links=args.xgmi_links),
                  pod_resources_socket=args.pod_resources_socket,
                  gpu_resources=tuple(args.gpu_resource or (PRIMARY_GPU_KEY,)), label_node=args.label_node,
                  annotation_encoding=args.annotation_encoding, diag_parallel=args.diag_parallel,
                  diag_baseline=args.diag_baseline, baseline_file=args.diag_baseline_file,
                  isolation=args.diag_isolation)
    if args.diag_baseline_reset and agent.baselines is not None:
        spec = args.diag_baseline_reset.strip()
        gone = agent.baselines.drop(None if spec.lower() == "all" else spec.split(","))
        print(f"self-baselines reset: {', '.join(gone) if gone else 'none matched'}", file=sys.stderr, flush=True)
    client = None
    srv = None
    try:
        if "annotation" in pubs:
            from ..kube.client import KubeClient
            from ..kube.config import load_kube_config
            conn = load_kube_config(args.kubeconfig)
            tok = conn.token
            if conn.token_file:
                try:
                    with open(conn.token_file, encoding="utf-8") as f:
                        tok = f.read()
                except OSError:
                    pass
            bound = token_node_name(tok)
            if bound is not None and bound != args.node:
                # deploy/agent-policy.yaml would refuse every write anyway; say why at start-up instead
                print(f"--node {args.node!r} is not the node this pod's ServiceAccount token is bound to ({bound!r}): "
                      "refusing to publish another node's status", file=sys.stderr, flush=True)
                return 2
            client = KubeClient(conn, timeout=10.0)
            try:  # the node's registered GPU count; refreshed from every condition PATCH response after this
                agent.observe_node(client.get_node(args.node))
            except Exception as e:
                print(f"could not read node {args.node}: {e}", file=sys.stderr, flush=True)
        if "http" in pubs:
            host, _, port = args.listen.rpartition(":")
            # a probe cycle may legitimately include diagnostics (up to --diag-timeout per GPU)
            if bool(args.tls_cert_file) != bool(args.tls_key_file) or (args.tls_client_ca and not args.tls_cert_file):
                print("--tls-cert-file and --tls-key-file go together (and --tls-client-ca needs them)", file=sys.stderr,
                      flush=True)
                return 2
            tls = tls_context(args.tls_cert_file, args.tls_key_file, args.tls_client_ca) if args.tls_cert_file else None
            srv = serve(agent, host or "0.0.0.0", int(port),
                        stale_after=max(180.0, 3 * args.interval + args.diag_timeout), tls=tls,
                        require_client_cert=bool(args.tls_client_ca))
        # SIGTERM (pod deletion, rolling update): finish the cycle in flight and leave with 0 instead of dying
        # mid-write; the condition keeps its last heartbeat and ages out at the checker's --probe-max-age
        stop = threading.Event()
        if threading.current_thread() is threading.main_thread():
            import signal
            signal.signal(signal.SIGTERM, lambda *_: stop.set())
        while not stop.is_set():
            started = time.monotonic()
            rep = agent.probe_once()
            if "stdout" in pubs:
                print(json.dumps(rep, separators=(",", ":")), flush=True)
            published = True
            if client is not None:
                try:
                    agent.publish(client, rep)
                except Exception as e:
                    published = False
                    print(f"node status publish failed: {e}", file=sys.stderr, flush=True)
            if args.once:  # a one-shot run (CI, a harness) says whether the node saw its verdict
                return 0 if published else 1
            stop.wait(max(0.0, args.interval - (time.monotonic() - started)))
        print("SIGTERM: agent stopped", file=sys.stderr, flush=True)
        return 0
    finally:
        # --once, SIGTERM or a start-up refusal: the kube connection and the HTTP server do not outlive main
        if client is not None:
            client.close()
        if srv is not None:
            srv.shutdown()
            srv.server_close()


if __name__ == "__main__":
    sys.exit(main())
