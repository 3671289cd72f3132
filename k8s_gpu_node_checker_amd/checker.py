"""Check orchestration: scan -> MI355X health gate -> Slack -> report.

Reference ``one_shot`` (``check-gpu-node.py:252-293``) runs strictly in
sequence: LIST, then Slack (including up to 3 x ``retry_delay`` of sleeps),
then output.  Here the Slack POST runs on a worker thread while the report is
rendered, and the report is written in one ``write`` once Slack has finished,
so the stream order of Appendix A / SURVEY §5.1 is unchanged (the Slack
success line still precedes the summary on stdout).

:func:`run_check` is the library entry point (used by the CLI, the bench and
the node agent's self-test); :func:`one_shot` adds the printing.
"""

from __future__ import annotations

import sys
import time
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Callable, Dict, List, Optional, TextIO, Tuple

from . import report
from .kube.client import KubeClient
from .kube.config import ClusterConnection
from .models import health as H
from .models.node import ScanResult, withdrawn_count
from .models.node import HEALTH_ANNOTATION
from .models.resources import GPU_RESOURCE_KEYS, PRIMARY_GPU_KEY
from .utils.timing import NullTracer, Tracer

#: the node agents' headless Service (deploy/daemonset.yaml): its EndpointSlices fill ``{pod_ip}``
AGENT_SERVICE = "gpu-health/mi355x-node-agent"


class CheckOptions:
    """All knobs of one check; defaults reproduce the reference exactly."""

    def __init__(self, **kw: Any):
        self.json = False
        self.json_extended = False
        self.slack_webhook: Optional[str] = None
        self.slack_username = "k8s-gpu-checker"
        self.slack_only_on_error = False
        self.slack_retry_count = 3
        self.slack_retry_delay = 30
        self.slack_retry_policy = "backoff"
        self.kube_timeout = 30.0
        self.kube_retries = 2
        self.page_size = 500
        self.label_selector: Optional[str] = None
        self.resource_version: Optional[str] = None
        self.gpu_source = "capacity"
        self.health_policy = "auto"
        self.probe_max_age = 900.0
        self.probe_unknown = "allow"
        self.xgmi_links = H.XGMI_LINKS_EXPECTED
        self.probe_endpoint: Optional[str] = None
        self.probe_service = AGENT_SERVICE
        self.probe_concurrency = 64
        self.probe_timeout = 2.0
        self.probe_ca: Optional[str] = None
        self.probe_tls_server_name: Optional[str] = None
        #: ``--watch-events``: a ``parallel.fanout.ProbeCache`` reused across evaluations (``--probe-cache-ttl``)
        self.probe_cache: Optional[Any] = None
        self.probe_cache_ttl = 30.0
        self.probe_client_cert: Optional[str] = None
        self.probe_client_key: Optional[str] = None
        self.health_reeval = False
        self.require_schedulable = False
        self.trace = False
        self.slack_gate: Optional[Callable[["CheckResult"], bool]] = None
        for k, v in kw.items():
            if not hasattr(self, k):
                raise TypeError(f"unknown check option {k!r}")
            setattr(self, k, v)

    @classmethod
    def from_args(cls, args: Any) -> "CheckOptions":
        o = cls()
        for k in list(vars(o)):
            if hasattr(args, k):
                setattr(o, k, getattr(args, k))
        return o

    @property
    def needs_extras(self) -> bool:
        return self.health_policy != "off" or self.json_extended or self.require_schedulable

    @property
    def custom_thresholds(self) -> bool:
        """Checker-side thresholds that differ from the ones the node agent evaluated with."""
        return self.xgmi_links != H.XGMI_LINKS_EXPECTED

    @property
    def reeval(self) -> bool:
        """Re-judge the full report annotation instead of trusting the agent's condition: asked for
        (``--health-reeval``), or implied by non-default thresholds, which the condition cannot honour."""
        return self.health_reeval or self.custom_thresholds


class CheckResult:
    def __init__(self, scan: ScanResult, verdicts: List[Optional[H.Verdict]], tracer: Tracer):
        self.scan = scan
        self.verdicts = verdicts
        self.tracer = tracer
        self.slack_sent: Optional[bool] = None
        #: the fleet-relative diagnostics summary (``models/fleet.judge_fleet``), when reports were judged
        self.fleet_diag: Optional[Dict[str, Any]] = None
        #: operator-facing notes (stderr), e.g. thresholds that could not be applied to a node
        self.warnings: List[str] = []

    @property
    def gpu_nodes(self) -> List[Dict[str, Any]]:
        return self.scan.gpu_nodes

    @property
    def ready_gpu_nodes(self) -> List[Dict[str, Any]]:
        return self.scan.ready_gpu_nodes

    @property
    def exit_code(self) -> int:
        return self.scan.exit_code()

    def extended_fields(self) -> Dict[str, Any]:
        nodes = []
        for i, n in enumerate(self.scan.gpu_nodes):
            ex = self.scan.extras[i] if i < len(self.scan.extras) else None
            v = self.verdicts[i] if i < len(self.verdicts) else None
            entry: Dict[str, Any] = {"name": n["name"], "ready": n["ready"]}
            if ex is not None:
                entry.update(ex.to_dict())
            entry["health"] = v.to_dict() if v is not None else None
            nodes.append(entry)
        return {
            "mi355x": {
                "health_summary": H.summarize(self.verdicts) if self.verdicts else None,
                "fleet": fleet_versions(self.scan.extras),
                "diag_fleet": self.fleet_diag,
                "nodes": nodes,
            },
            "timings_ms": self.tracer.as_ms(),
            "items_seen": self.scan.items_seen,
        }


def fleet_versions(extras: List[Any]) -> Optional[Dict[str, Any]]:
    """Software versions across the MI355X nodes that publish a report (``--json-extended``): amdgpu
    driver, and firmware per image, each as ``{version: node count}``.  More than one key in a row is
    a fleet that was only partly upgraded -- jobs spanning those nodes run on different driver or
    firmware behaviour.  None when no node carries a report."""
    drivers: Dict[str, int] = {}
    firmware: Dict[str, Dict[str, int]] = {}
    n = 0
    for ex in extras:
        rep = ex.report() if ex is not None else None
        if not rep or not isinstance(rep, dict) or rep.get("error"):
            continue
        n += 1
        drv = (rep.get("driver") or {}).get("version") if isinstance(rep.get("driver"), dict) else None
        if drv:
            rel = H.driver_release(drv)
            drivers[rel] = drivers.get(rel, 0) + 1
        raw_fw: Dict[str, set] = {}
        for g in H.report_gpus(rep):
            for name, ver in ((g.get("fw") or {}) if isinstance(g, dict) and isinstance(g.get("fw"), dict)
                              else {}).items():
                try:
                    raw_fw.setdefault(name, set()).add(ver)
                except TypeError:  # an unhashable value: kept as its text
                    raw_fw.setdefault(name, set()).add(str(ver))
        node_fw = {name: {H.fw_version_str(name, v) for v in vers} for name, vers in raw_fw.items()}
        for name, vers in node_fw.items():
            row = firmware.setdefault(name, {})
            for v in vers:  # a node with two versions of one image counts under both
                row[v] = row.get(v, 0) + 1
    if not n:
        return None
    mixed = sorted([k for k, row in firmware.items() if len(row) > 1] + (["driver"] if len(drivers) > 1 else []))
    return {"nodes_reporting": n, "driver": drivers, "firmware": {k: firmware[k] for k in sorted(firmware)},
            "mixed": mixed}


def scan_cluster(cluster: ClusterConnection, opts: CheckOptions, tracer: Tracer) -> ScanResult:
    client = KubeClient(cluster, timeout=opts.kube_timeout, retries=opts.kube_retries, tracer=tracer)
    try:
        with tracer.span("list"):
            return client.scan_nodes(limit=opts.page_size, keys=GPU_RESOURCE_KEYS, gpu_source=opts.gpu_source,
                                     want_extras=opts.needs_extras, label_selector=opts.label_selector,
                                     resource_version=opts.resource_version,
                                     annotation_mode=2 if (opts.reeval or opts.json_extended) else 1)
    finally:
        client.close()


def resolve_agent_endpoints(cluster: Optional[ClusterConnection], opts: CheckOptions,
                            tracer: Tracer) -> Tuple[Optional[Dict[str, str]], Optional[str]]:
    """``{pod_ip}`` in ``--probe-endpoint``: the agent pod's address per node, from the EndpointSlices of
    ``--probe-service`` (one paged GET; RBAC ``endpointslices: list`` in that namespace,
    ``deploy/rbac.yaml``).  Returns ``(addresses, None)`` or ``(None, error)``; an error makes every node
    ``unknown`` with that reason instead of failing the check."""
    from .parallel.fanout import template_fields
    if not opts.probe_endpoint or "pod_ip" not in template_fields(opts.probe_endpoint):
        return None, None
    if cluster is None:
        return None, "no cluster connection to read the agent's EndpointSlices"
    ns, _, svc = (opts.probe_service or AGENT_SERVICE).partition("/")
    if not ns or not svc:
        return None, f"--probe-service {opts.probe_service!r} is not NAMESPACE/NAME"
    cache = opts.probe_cache
    if cache is not None:
        hit = cache.fresh_endpoints(time.monotonic())
        if hit is not None:
            return hit
        res = _list_agent_endpoints(cluster, opts, tracer, ns, svc)
        cache.endpoints = (time.monotonic(), res)
        return res
    return _list_agent_endpoints(cluster, opts, tracer, ns, svc)


def _list_agent_endpoints(cluster: ClusterConnection, opts: CheckOptions, tracer: Tracer, ns: str,
                          svc: str) -> Tuple[Optional[Dict[str, str]], Optional[str]]:
    from .parallel.fanout import agent_addresses
    client = KubeClient(cluster, timeout=opts.kube_timeout, retries=opts.kube_retries, tracer=tracer)
    try:
        with tracer.span("endpoints"):
            return agent_addresses(client.list_endpoint_slices(ns, svc, limit=opts.page_size)), None
    except Exception as e:  # 403 without the Role, 404 without discovery.k8s.io/v1, transport errors
        return None, str(e).strip().splitlines()[0] if str(e).strip() else type(e).__name__
    finally:
        client.close()


def apply_health(scan: ScanResult, opts: CheckOptions, tracer: Tracer,
                 warnings: Optional[List[str]] = None,
                 cluster: Optional[ClusterConnection] = None,
                 fleet_out: Optional[Dict[str, Any]] = None) -> List[Optional[H.Verdict]]:
    """Evaluate MI355X probe reports and gate ``ready`` (no-op when no node carries one).

    With three or more current reports the diagnostics' rates are also judged across the fleet
    (``models/fleet.py``); ``fleet_out``, when given, receives its ``summary`` and the per-node ``views``.

    Every verdict is cross-checked against the node's ``amd.com/gpu`` count from this LIST
    (:func:`models.node.expected_gpu_count`): on the condition path through the ``ok/seen`` counts
    in its message, on the report path through ``evaluate_report``'s ``expected_gpus``.
    """
    if opts.health_policy == "off" or not scan.gpu_nodes:
        return []
    with tracer.span("health"):
        exp = H.HealthExpectations(xgmi_links=opts.xgmi_links, max_age_s=opts.probe_max_age)
        reports: List[Optional[Dict[str, Any]]] = [None] * len(scan.gpu_nodes)
        if opts.probe_endpoint:
            from .parallel.fanout import fetch_probe_reports
            pod_ips, pod_err = resolve_agent_endpoints(cluster, opts, tracer)
            reports = fetch_probe_reports(scan, opts.probe_endpoint, opts.probe_concurrency, opts.probe_timeout,
                                          ca_file=opts.probe_ca, client_cert=opts.probe_client_cert,
                                          client_key=opts.probe_client_key, pod_ips=pod_ips,
                                          pod_ip_error=pod_err, server_name=opts.probe_tls_server_name,
                                          cache=opts.probe_cache)
        verdicts: List[Optional[H.Verdict]] = []
        changed = False
        unknown_ok = opts.probe_unknown == "allow"
        reeval = opts.reeval
        now = time.time()
        unapplied: List[str] = []
        key = PRIMARY_GPU_KEY
        policy = opts.health_policy
        max_age = opts.probe_max_age
        from_condition = H.verdict_from_condition
        gate = H.gate_ready
        # pass 1: which report (if any) judges each node; the condition path needs none
        judged: List[Optional[Dict[str, Any]]] = [None] * len(scan.gpu_nodes)
        pre: List[Optional[H.Verdict]] = [None] * len(scan.gpu_nodes)
        # reports the fleet judgement may compare: the judged ones, plus (when the scan parsed the annotations
        # anyway, --json-extended / --explain / --fleet) those of nodes judged by their condition
        compare: List[Optional[Dict[str, Any]]] = [None] * len(scan.gpu_nodes)
        cached: List[bool] = [False] * len(scan.gpu_nodes)  # compare[i] is ex.report(): its fractions are cached
        parsed = opts.json_extended
        comparable = 0
        for i, (node, ex, rep) in enumerate(zip(scan.gpu_nodes, scan.extras, reports)):
            if rep is None and reeval:
                rep = ex.report()
            if rep is None and ex.health_condition is not None:
                if parsed and ex.health_annotation:
                    r = ex.report()
                    if isinstance(r, dict) and r.get("node") in (None, node["name"]):
                        compare[i] = r
                        cached[i] = True
                        comparable += 1
                continue
            if rep is None and ex.health_annotation:
                rep = ex.report()
            cached[i] = rep is not None and reports[i] is None
            other = rep.get("node") if isinstance(rep, dict) else None
            if other is not None and other != node["name"]:
                # a report names the node it was taken on: one fetched from a reassigned or stale IP (or an
                # annotation copied between nodes) says nothing about this node
                pre[i] = H.Verdict(H.UNKNOWN, [f"report is for node {other}"])
            else:
                judged[i] = compare[i] = rep
                comparable += rep is not None
        # the fleet-relative judgement of the diagnostics' rates (models/fleet.py): only with 3+ reports to compare
        fleet_views: List[Optional[Dict[str, Any]]] = [None] * len(scan.gpu_nodes)
        if comparable >= 3:
            from .models import fleet as F
            current = [r if H.report_gate(r, exp, now) is None else None for r in compare]
            fracs = [ex.fleet_fractions() if cached[i] and current[i] is not None else None
                     for i, ex in enumerate(scan.extras)]
            summary, fleet_views = F.judge_fleet([n["name"] for n in scan.gpu_nodes], current, fracs)
            if summary and fleet_out is not None:
                fleet_out.update(summary=summary, views=fleet_views)
        by_alloc = opts.gpu_source != "capacity"
        for i, (node, ex, rep) in enumerate(zip(scan.gpu_nodes, scan.extras, reports)):
            cap, alloc = ex.capacity.get(key), ex.allocatable.get(key)
            is_amd = alloc is not None or cap is not None or key in node["gpu_breakdown"]
            expected = max(cap or 0, alloc or 0)  # models.node.expected_gpu_count
            # counting allocatable, a node whose device plugin withdrew every GPU is in the set (models.node
            # classify_node) but has nothing to schedule on: never Ready, whatever its agent says
            withdrawn = withdrawn_count(ex.capacity, ex.allocatable) if by_alloc else 0
            v: Optional[H.Verdict] = pre[i]
            rep = judged[i]
            if rep is None and fleet_views[i] is not None:
                # the fleet has something to say about a node judged by its condition: its report carries the
                # rates, the condition's message does not
                rep = compare[i]
            if v is not None:
                pass
            elif rep is None and ex.health_condition is not None:
                # cheap path: the agent's verdict is a NodeCondition already parsed by the scan
                v = from_condition(ex.health_condition, max_age, now, expected)
                if reeval:
                    unapplied.append(node["name"])
            elif rep is not None or policy == "require":
                v = H.evaluate_report(rep, expected, exp, now, fleet_views[i])
            if withdrawn:
                plugin = (f"device plugin allocates {alloc or 0} of {cap} {key}" if cap
                          else f"device plugin allocates 0 of {withdrawn} GPUs")
                if v is None:
                    v = H.Verdict(H.UNHEALTHY, [plugin])
                else:
                    v.reasons.insert(0, plugin)
                    v.state = H.UNHEALTHY
                verdicts.append(v)
                if node["ready"]:  # classify_node already cleared it; kept false against any later gate
                    node["ready"] = False
                    changed = True
                continue
            if v is None:
                verdicts.append(None)
                continue
            if cap and alloc is not None and alloc < cap:
                # SURVEY §5 failure detection: the device plugin withholds GPUs it judged unhealthy
                # (allocatable < capacity); the scheduler already avoids them, so a hint, not a failure
                v.warnings.append(f"device plugin allocates {alloc} of {cap} {key}")
                if v.state == H.HEALTHY:
                    v.state = H.DEGRADED
            verdicts.append(v)
            gated = gate(ex.ready_condition, v, policy, is_amd, unknown_ok)
            if gated != node["ready"]:
                node["ready"] = gated
                changed = True
        if changed:
            scan.recompute_ready()
        if unapplied and warnings is not None:
            shown = ", ".join(unapplied[:5]) + (f" (+{len(unapplied) - 5} more)" if len(unapplied) > 5 else "")
            warnings.append(f"warning: no {HEALTH_ANNOTATION} report on {shown}: checker thresholds "
                            f"(--xgmi-links {opts.xgmi_links}) not applied, the agent's AMDGPUHealthy verdict is used")
        if not any(verdicts):
            return []
        return verdicts


def apply_schedulability(scan: ScanResult, opts: CheckOptions) -> None:
    """``--require-schedulable``: a GPU node that takes no new pods -- cordoned (``spec.unschedulable``)
    or tainted ``amd.com/gpu-unhealthy`` by the node agent -- does not count as Ready.

    Off by default: the reference counts cordoned and tainted nodes as Ready (``check-gpu-node.py:172-178``
    reads conditions only; SURVEY §2.2 "not consumed")."""
    if not opts.require_schedulable:
        return
    changed = False
    for node, ex in zip(scan.gpu_nodes, scan.extras):
        if node["ready"] and (ex.unschedulable or any(t.get("key") == H.UNHEALTHY_TAINT["key"]
                                                      for t in node["taints"])):
            node["ready"] = False
            changed = True
    if changed:
        scan.recompute_ready()


def run_check(cluster: ClusterConnection, opts: CheckOptions, tracer: Optional[Tracer] = None) -> CheckResult:
    tracer = tracer or (Tracer() if (opts.trace or opts.json_extended) else NullTracer())
    scan = scan_cluster(cluster, opts, tracer)
    warnings: List[str] = []
    fleet: Dict[str, Any] = {}
    verdicts = apply_health(scan, opts, tracer, warnings, cluster, fleet)
    apply_schedulability(scan, opts)
    result = CheckResult(scan, verdicts, tracer)
    result.warnings = warnings
    result.fleet_diag = fleet.get("summary")
    return result


def _health_notes(result: CheckResult) -> Optional[List[Optional[str]]]:
    if not result.verdicts:
        return None
    return [v.short() if v is not None else None for v in result.verdicts]


def one_shot(cluster: ClusterConnection, opts: CheckOptions, out: Optional[TextIO] = None,
             err: Optional[TextIO] = None, tracer: Optional[Tracer] = None) -> int:
    """Reference ``one_shot`` (``:252-293``): prints the report, returns the exit code."""
    return check_and_report(cluster, opts, out, err, tracer).exit_code


def check_and_report(cluster: ClusterConnection, opts: CheckOptions, out: Optional[TextIO] = None,
                     err: Optional[TextIO] = None, tracer: Optional[Tracer] = None) -> CheckResult:
    # A check allocates tens of thousands of short-lived, acyclic objects at 1000+ nodes (dicts,
    # labels, strings); refcounting frees them all, so the cyclic collector only adds pauses
    # (observed as 10-70 ms tail latency).  Paused for the check, restored afterwards.
    import gc
    was_enabled = gc.isenabled()
    gc.disable()
    try:
        return _check_and_report(cluster, opts, out, err, tracer)
    finally:
        if was_enabled:
            gc.enable()


def _check_and_report(cluster: ClusterConnection, opts: CheckOptions, out: Optional[TextIO],
                      err: Optional[TextIO], tracer: Optional[Tracer]) -> CheckResult:
    result = run_check(cluster, opts, tracer)
    emit_report(result, opts, out, err)
    return result


def emit_report(result: CheckResult, opts: CheckOptions, out: Optional[TextIO] = None,
                err: Optional[TextIO] = None) -> None:
    """Slack (on a worker thread) + JSON/text report of a finished check, in the reference's stream
    order (``:262-287``); shared by one-shot checks and the event-driven watcher (``kube/watch.py``)."""
    from .notify import slack
    out = out if out is not None else sys.stdout
    err = err if err is not None else sys.stderr
    tr = result.tracer
    gpu_nodes, ready = result.gpu_nodes, result.ready_gpu_nodes

    url = slack.get_slack_webhook_url(opts.slack_webhook)
    worker: "Optional[threading.Thread]" = None
    box: Dict[str, bool] = {}
    if slack.should_send(url, opts.slack_only_on_error, len(ready)) and (
            opts.slack_gate is None or opts.slack_gate(result)):
        text = report.format_slack_message(gpu_nodes, ready, _health_notes(result))
        delay = opts.slack_retry_delay
        if delay < 0:
            print(f"경고: --slack-retry-delay {delay} 는 음수이므로 0으로 처리합니다.", file=err)
            delay = 0

        def _send() -> None:
            with tr.span("slack"):
                box["ok"] = slack.send_slack_message(url, text, opts.slack_username, opts.slack_retry_count,
                                                     delay, policy=opts.slack_retry_policy, err=err)
        import threading  # only when a Slack message goes out
        worker = threading.Thread(target=_send, name="slack", daemon=True)
        worker.start()

    json_mode = opts.json or opts.json_extended
    with tr.span("render"):
        if json_mode:
            extra = None
            if opts.json_extended:
                tr.finish()
                extra = result.extended_fields()
            body = report.render_json(report.json_payload(gpu_nodes, ready, extra))
        else:
            body = report.render_text(gpu_nodes, ready)

    prefix = ""
    if worker is not None:
        worker.join()
        result.slack_sent = box.get("ok", False)
        if not json_mode:
            if result.slack_sent:
                prefix = report.SLACK_SENT + "\n"
            else:
                print(report.SLACK_FAILED, file=err)
    for w in result.warnings:
        print(w, file=err)
    out.write(prefix + body)
    out.flush()
    if opts.trace:
        tr.finish()
        print(f"[trace] {tr.format()} backend={_backend()}", file=err)


def _backend() -> str:
    from .ops import fastpath
    return fastpath.backend()
