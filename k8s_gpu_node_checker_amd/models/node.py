"""Node projection and GPU-node classification.

The reference deserialises every ``V1Node`` through the OpenAPI client and
then projects it (``check-gpu-node.py:172-226``).  Here the raw JSON *is* the
model: a ``NodeList`` page is decoded once (``json.loads`` or the native
scanner in :mod:`k8s_gpu_node_checker_amd.ops.fastpath`) and each item is
projected straight into the report dict, so there is no per-node object
graph to build and no ``isinstance(cond, V1NodeCondition)`` trap (``:176``).

Report dict schema (reference ``:202-212``)::

    {"name": str, "ready": bool, "gpus": int, "gpu_breakdown": {key: int},
     "labels": {str: str}, "taints": [{"key", "value", "effect"}]}
"""

from __future__ import annotations

from _collections_abc import Mapping  # collections.abc.Mapping; loaded by os, unlike collections
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

from .resources import GPU_RESOURCE_KEYS, PRIMARY_GPU_KEY, gpu_breakdown

#: Annotation written by the MI355X node agent (see ``agent/``): the full probe report.
HEALTH_ANNOTATION = "amd.com/mi355x-health"
#: NodeCondition the agent maintains (its verdict; cheap to read from the LIST).
HEALTH_CONDITION = "AMDGPUHealthy"


def _k8s_time(ts: Any) -> Optional[float]:
    if not isinstance(ts, str):
        return None
    from .health import parse_k8s_time
    return parse_k8s_time(ts)


def health_condition(node: Mapping[str, Any]) -> Optional[Tuple[Any, Any, Any, Optional[float]]]:
    conds = _get(_get(node, "status"), "conditions")
    if not isinstance(conds, list):
        return None
    found = None
    for c in conds:
        if isinstance(c, Mapping) and c.get("type") == HEALTH_CONDITION:
            found = (c.get("status"), c.get("reason"), c.get("message"), _k8s_time(c.get("lastHeartbeatTime")))
    return found


def _get(obj: Any, key: str) -> Any:
    return obj.get(key) if isinstance(obj, Mapping) else None


def is_ready(node: Mapping[str, Any]) -> bool:
    """NodeCondition ``Ready`` with status ``"True"`` (reference ``:172-178``)."""
    conds = _get(_get(node, "status"), "conditions")
    if not conds or not isinstance(conds, list):
        return False
    for cond in conds:
        if isinstance(cond, Mapping) and cond.get("type") == "Ready" and cond.get("status") == "True":
            return True
    return False


def _taints(spec: Any) -> List[Dict[str, Any]]:
    taints = _get(spec, "taints")
    if not taints or not isinstance(taints, list):
        return []
    out = []
    for t in taints:
        if isinstance(t, Mapping):
            out.append({"key": t.get("key"), "value": t.get("value"), "effect": t.get("effect")})
    return out


def project_node(node: Mapping[str, Any], keys: Sequence[str] = GPU_RESOURCE_KEYS,
                 gpu_source: str = "capacity") -> Dict[str, Any]:
    """Project one raw ``Node`` into the report dict (reference ``extract_node_info``, ``:199-212``).

    ``gpu_source`` selects which status map the GPU counts come from.  The
    reference reads ``capacity`` only (default, byte parity); the MI355X
    preset reads ``allocatable``, i.e. what the ROCm device plugin reports as
    usable after its own health checks.
    """
    meta = _get(node, "metadata")
    status = _get(node, "status")
    caps = gpu_breakdown(_get(status, gpu_source), keys)
    labels = _get(meta, "labels") if meta else None
    return {
        "name": meta.get("name") if isinstance(meta, Mapping) else "",
        "ready": is_ready(node),
        "gpus": sum(caps.values()) if caps else 0,
        "gpu_breakdown": caps,
        "labels": labels if labels else {},
        "taints": _taints(_get(node, "spec")),
    }


def classify_node(node: Mapping[str, Any], keys: Sequence[str] = GPU_RESOURCE_KEYS,
                  gpu_source: str = "capacity") -> Optional[Dict[str, Any]]:
    """The report dict of a GPU node, ``None`` for any other node (reference ``:220-225``).

    Membership is the reference's -- GPU keys summing above 0 in ``capacity`` (``:181-196``) -- or,
    under ``--gpu-source allocatable``, above 0 in either map: counts come from allocatable, but a
    node whose device plugin withdrew every GPU (allocatable 0, capacity 8: a crashed or wedged
    plugin, the commonest GPU-node failure) stays in the set with ``"ready": false`` instead of
    leaving the report, Slack and metrics.  A fleet entirely in that state exits 3, not 2
    (``:289-293``).  The native scanner (``csrc/fastpath/fastpath.cpp`` ``emit_node``) applies the
    same rule.
    """
    info = project_node(node, keys, gpu_source)
    if info["gpus"] > 0:
        return info
    if gpu_source != "capacity" and withdrawn_count(gpu_breakdown(_get(_get(node, "status"), "capacity"), keys),
                                                    info["gpu_breakdown"]):
        info["ready"] = False
        return info
    return None


def withdrawn_count(capacity: Mapping[str, int], allocatable: Mapping[str, int]) -> int:
    """GPUs registered (capacity) on a node whose allocatable GPU keys sum to 0 or less: the device
    plugin withdrew all of them.  0 for any node with an allocatable GPU or no registered one."""
    cap = sum(capacity.values()) if capacity else 0
    if cap <= 0 or (sum(allocatable.values()) if allocatable else 0) > 0:
        return 0
    return cap


_UNPARSED = object()


class NodeExtras:
    """Side information the default report does not show but the health gate uses."""

    __slots__ = ("ready_condition", "capacity", "allocatable", "unschedulable", "health_annotation", "internal_ip",
                 "health_condition", "_report", "_fleet")

    def __init__(self, ready_condition: bool, capacity: Dict[str, int], allocatable: Dict[str, int],
                 unschedulable: bool, health_annotation: Optional[str], internal_ip: Optional[str] = None,
                 health_condition: Optional[Tuple[Any, Any, Any, Optional[float]]] = None):
        self.ready_condition = ready_condition
        self.capacity = capacity
        self.allocatable = allocatable
        self.unschedulable = unschedulable
        self.health_annotation = health_annotation
        self.internal_ip = internal_ip
        #: ``(status, reason, message, lastHeartbeatTime epoch)`` of the AMDGPUHealthy condition
        self.health_condition = health_condition
        self._report: Any = _UNPARSED
        self._fleet: Any = None

    def report(self) -> Optional[Dict[str, Any]]:
        """The report annotation parsed (``models.health.parse_annotation``), once per node object: the
        health gate, ``--json-extended``'s fleet view and ``--explain`` share it, and the watcher keeps the
        object until the node changes."""
        try:
            r = self._report
        except AttributeError:  # built by the native scanner, which sets only __init__'s slots
            r = _UNPARSED
        if r is _UNPARSED:
            from .health import parse_annotation
            r = self._report = slim_report(parse_annotation(self.health_annotation))
        return r

    def fleet_fractions(self) -> Dict[Any, float]:
        """``models/fleet.node_fractions`` of :meth:`report`, once per node object: the watcher re-judges the
        fleet on every event, and only the nodes that changed are new objects."""
        try:
            f = self._fleet
        except AttributeError:  # built by the native scanner
            f = None
        if f is None:
            from .fleet import node_fractions
            f = self._fleet = node_fractions(self.report())
        return f

    def to_dict(self) -> Dict[str, Any]:
        return {
            "ready_condition": self.ready_condition,
            "capacity": self.capacity,
            "allocatable": self.allocatable,
            "unschedulable": self.unschedulable,
            "internal_ip": self.internal_ip,
            "health_condition": list(self.health_condition) if self.health_condition else None,
        }


# per-test fields of a diagnostic result that only the agent's own views read (per-XCD/CU maps, per-kind burn-in
# rows, wall time): the agent leaves them out of the node annotation, and the checker drops them from reports
# fetched from /probe too -- it keeps every node's parsed report (the watcher, across checks)
DIAG_AGENT_ONLY = ("map", "kinds", "wall_s")


def slim_report(report: Any) -> Any:
    """``report`` without the agent-only fields of its diagnostic results (:data:`DIAG_AGENT_ONLY`), in place."""
    gpus = report.get("gpus") if isinstance(report, dict) else None
    for g in gpus if isinstance(gpus, list) else ():
        diag = g.get("diag") if isinstance(g, dict) else None
        for res in diag.values() if isinstance(diag, dict) else ():
            if isinstance(res, dict):
                for k in DIAG_AGENT_ONLY:
                    res.pop(k, None)
    return report


def node_extras(node: Mapping[str, Any], keys: Sequence[str] = GPU_RESOURCE_KEYS,
                annotation_mode: int = 2) -> NodeExtras:
    """``annotation_mode``: 2 = always keep the probe-report annotation, 1 = only for nodes
    without the ``AMDGPUHealthy`` condition (the checker's default: the condition is the verdict)."""
    meta = _get(node, "metadata")
    status = _get(node, "status")
    ann = _get(meta, "annotations")
    raw = ann.get(HEALTH_ANNOTATION) if isinstance(ann, Mapping) else None
    ip = None
    addrs = _get(status, "addresses")
    if isinstance(addrs, list):
        for a in addrs:
            if isinstance(a, Mapping) and a.get("type") == "InternalIP" and isinstance(a.get("address"), str):
                ip = a["address"]
                break
    hc = health_condition(node)
    if annotation_mode == 0 or (annotation_mode == 1 and hc is not None):
        raw = None
    return NodeExtras(
        ready_condition=is_ready(node),
        capacity=gpu_breakdown(_get(status, "capacity"), keys),
        allocatable=gpu_breakdown(_get(status, "allocatable"), keys),
        unschedulable=bool(_get(_get(node, "spec"), "unschedulable")),
        health_annotation=raw if isinstance(raw, str) else None,
        internal_ip=ip,
        health_condition=hc,
    )


class ScanResult:
    """Outcome of one cluster scan (reference ``list_gpu_nodes`` return value, ``:215-226``).

    ``gpu_nodes`` keeps API order; ``ready_gpu_nodes`` is the Ready subset.
    ``extras`` is parallel to ``gpu_nodes`` and only filled when a consumer
    (health gate, extended JSON) asked for it.
    """

    __slots__ = ("gpu_nodes", "ready_gpu_nodes", "extras", "items_seen")

    def __init__(self) -> None:
        self.gpu_nodes: List[Dict[str, Any]] = []
        self.ready_gpu_nodes: List[Dict[str, Any]] = []
        self.extras: List[NodeExtras] = []
        self.items_seen = 0

    def add(self, info: Optional[Dict[str, Any]], extras: Optional[NodeExtras] = None) -> None:
        """One scanned item: ``info`` is :func:`classify_node`'s (``None``: not a GPU node)."""
        self.items_seen += 1
        if info is not None:
            self.gpu_nodes.append(info)
            if extras is not None:
                self.extras.append(extras)
            if info["ready"]:
                self.ready_gpu_nodes.append(info)

    def recompute_ready(self) -> None:
        self.ready_gpu_nodes = [n for n in self.gpu_nodes if n["ready"]]

    def exit_code(self) -> int:
        """Reference exit-code contract (``:289-293``): 0 ready, 3 none ready, 2 no GPU nodes."""
        if self.ready_gpu_nodes:
            return 0
        if self.gpu_nodes:
            return 3
        return 2


def scan_items(items: Iterable[Mapping[str, Any]], result: Optional[ScanResult] = None,
               keys: Sequence[str] = GPU_RESOURCE_KEYS, gpu_source: str = "capacity",
               want_extras: bool = False, annotation_mode: int = 2) -> ScanResult:
    """Pure-Python scan of decoded ``NodeList.items`` (reference ``:217-225``)."""
    res = result if result is not None else ScanResult()
    for n in items or ():
        info = classify_node(n, keys, gpu_source)
        res.add(info, node_extras(n, keys, annotation_mode) if want_extras and info is not None else None)
    return res


def primary_gpu_count(extras: NodeExtras, source: str = "capacity") -> int:
    table = extras.capacity if source == "capacity" else extras.allocatable
    return table.get(PRIMARY_GPU_KEY, 0)


def expected_gpu_count(extras: NodeExtras) -> int:
    """How many ``amd.com/gpu`` the node's agent must see: the larger of capacity and allocatable.

    Capacity is what the ROCm device plugin registered (the reference's GPU-node definition,
    ``check-gpu-node.py:181-201``); allocatable can only be lower (the plugin marked a GPU
    unhealthy), and a GPU the plugin still counts but amd-smi no longer sees is missing either way.
    Independent of ``--gpu-source``, which decides what the report *shows*."""
    return max(extras.capacity.get(PRIMARY_GPU_KEY, 0), extras.allocatable.get(PRIMARY_GPU_KEY, 0))

