"""Event-driven GPU-node monitoring: one LIST, then the apiserver's watch stream.

The reference is a one-shot check meant for cron every 10 minutes
(``README.md:188-189``), so a node that drops out of Ready is noticed up to
10 minutes late, and every run re-lists the whole cluster.  ``--watch-events``
keeps the GPU-node view current from ``GET /api/v1/nodes?watch=1``:

* initial state from a paginated LIST (its ``metadata.resourceVersion`` is
  where the watch starts);
* ADDED / MODIFIED / DELETED events update the per-node projection (the same
  :func:`models.node.project_node` / :func:`node_extras` as a LIST), BOOKMARK
  events advance the resourceVersion, a 410 ``ERROR`` (history compacted)
  triggers a re-LIST, a dropped stream is re-opened from the last
  resourceVersion with backoff;
* events arriving within ``debounce`` seconds are folded into one
  evaluation; the MI355X health gate runs on the new state (and again every
  ``recheck`` seconds without events: an agent that stopped publishing sends
  no event, its condition only goes stale with time) and a report
  (identical in format to a one-shot check) is emitted only when the
  outcome changed: exit code, or any node's name / Ready / GPU count /
  health verdict.

Slack follows the one-shot policy per report, de-duplicated like
``--state-file --slack-on-change`` (a report is itself a change; with
``--slack-only-on-error`` a recovery is announced once).
"""

from __future__ import annotations

import json
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..models.node import NodeExtras, ScanResult, classify_node, node_extras, project_node
from ..models.resources import GPU_RESOURCE_KEYS
from ..utils.backoff import Backoff
from ..utils.http import HTTPError, LineStream
from .client import KubeClient
from .config import ClusterConnection
from .errors import ApiException


class NodeView:
    """GPU-node projection of the cluster keyed by node name (API order = name order).

    A LIST is scanned natively (``ops/fastpath``, as the one-shot check scans it): that yields the GPU nodes and
    the number of items, not the other nodes' names -- ``unnamed`` counts those, and a watch event about a node
    the view has no name for is one of them (MODIFIED, DELETED) or a new node (ADDED)."""

    def __init__(self, gpu_source: str = "capacity", annotation_mode: int = 1):
        self.gpu_source = gpu_source
        self.annotation_mode = annotation_mode
        self.gpu: Dict[str, Tuple[Dict[str, Any], NodeExtras]] = {}
        self.all_names: set = set()
        self.unnamed = 0  # non-GPU nodes of the last LIST that no event has named yet

    def load(self, scan: ScanResult, items: int) -> None:
        """The view of one (natively scanned) LIST: its GPU nodes, and ``items`` nodes in all."""
        self.reset()
        for info, ex in zip(scan.gpu_nodes, scan.extras):
            self.gpu[info["name"]] = (info, ex)
        self.all_names.update(self.gpu)
        self.unnamed = max(0, items - len(self.gpu))

    def upsert(self, node: Dict[str, Any], kind: str = "MODIFIED") -> None:
        info = classify_node(node, GPU_RESOURCE_KEYS, self.gpu_source)
        name = info["name"] if info is not None else project_node(node, GPU_RESOURCE_KEYS, self.gpu_source)["name"]
        if name not in self.all_names and kind != "ADDED" and self.unnamed > 0:
            self.unnamed -= 1  # a node of the LIST we only counted, named now
        self.all_names.add(name)
        if info is not None:
            self.gpu[name] = (info, node_extras(node, GPU_RESOURCE_KEYS, self.annotation_mode))
        else:
            self.gpu.pop(name, None)

    def delete(self, node: Dict[str, Any]) -> None:
        name = project_node(node, GPU_RESOURCE_KEYS, self.gpu_source)["name"]
        if name in self.all_names:
            self.all_names.discard(name)
        elif self.unnamed > 0:
            self.unnamed -= 1  # a counted, unnamed node of the LIST
        self.gpu.pop(name, None)

    def reset(self) -> None:
        self.gpu.clear()
        self.all_names.clear()
        self.unnamed = 0

    def scan_result(self) -> ScanResult:
        """A fresh :class:`ScanResult` (copies: the health gate rewrites ``ready`` in place)."""
        res = ScanResult()
        for name in sorted(self.gpu):
            info, ex = self.gpu[name]
            res.gpu_nodes.append(dict(info))
            res.extras.append(ex)
        res.recompute_ready()
        res.items_seen = len(self.all_names) + self.unnamed
        return res


def list_resource_version(body: bytes) -> Optional[str]:
    """``metadata.resourceVersion`` of a NodeList: from the ``metadata`` object apiservers put before ``items``
    (decoded alone), else from the whole body."""
    head = body[:4096]
    i = head.find(b'"metadata"')
    items = head.find(b'"items"')
    if i >= 0 and (items < 0 or i < items):
        j = head.find(b"{", i)
        k = head.find(b"}", j)
        if 0 <= j < k:
            try:
                meta = json.loads(head[j:k + 1])
                return str(meta.get("resourceVersion") or "") or None
            except ValueError:
                pass
    doc = json.loads(body)
    meta = (doc.get("metadata") if isinstance(doc, dict) else None) or {}
    return str(meta.get("resourceVersion") or "") or None


def outcome_signature(result: Any) -> Tuple[Any, ...]:
    verdicts = result.verdicts or []
    sig: List[Any] = [result.exit_code]
    for i, n in enumerate(result.gpu_nodes):
        v = verdicts[i] if i < len(verdicts) else None
        sig.append((n["name"], n["ready"], n["gpus"], tuple(n["gpu_breakdown"].items()), v.state if v else None))
    return tuple(sig)


STOP_POLL_S = 0.25  # how often a quiet watch stream checks run()'s should_stop


class NodeWatcher:
    def __init__(self, cluster: ClusterConnection, opts: Any, watch_timeout: int = 300, debounce: float = 0.2,
                 page_size: Optional[int] = None, sleep: Callable[[float], None] = time.sleep,
                 recheck: float = 30.0):
        self.cluster = cluster
        self.opts = opts
        self.watch_timeout = max(1, int(watch_timeout))
        self.debounce = max(0.0, debounce)
        # re-evaluate a quiet cluster this often (0: only on events): the health gate ages heartbeats
        self.recheck = max(0.0, recheck)
        self.page_size = opts.page_size if page_size is None else page_size
        self.sleep = sleep
        self.view = NodeView(opts.gpu_source, 2 if (opts.reeval or opts.json_extended) else 1)
        self.rv: Optional[str] = None
        self.backoff = Backoff(base=0.5, cap=30.0)
        self.relists = 0
        self.events = 0

    # -- state ------------------------------------------------------------------
    def relist(self, client: KubeClient) -> None:
        """Paginated LIST into a fresh view, each page scanned natively (the one-shot check's scanner: 5,000 nodes
        in milliseconds, not the ~1.5 s of decoding and classifying every object in Python); remembers the list's
        resourceVersion, read off each page's leading ``metadata``."""
        from urllib.parse import quote
        from ..ops import fastpath
        scan = ScanResult()
        items = 0
        cont: Optional[str] = None
        while True:
            path = "/api/v1/nodes"
            q = []
            if self.page_size > 0:
                q.append(f"limit={self.page_size}")
            if cont:
                q.append("continue=" + quote(cont, safe=""))
            if self.opts.label_selector:
                q.append("labelSelector=" + quote(self.opts.label_selector, safe=""))
            body = client.request("GET", path + ("?" + "&".join(q) if q else "")).body
            cont, n = fastpath.scan_page(body, scan, GPU_RESOURCE_KEYS, self.view.gpu_source, True,
                                         self.view.annotation_mode)
            items += n
            if not cont or self.page_size <= 0:
                self.rv = list_resource_version(body)
                break
        self.view.load(scan, items)
        self.relists += 1

    def apply(self, ev: Dict[str, Any]) -> bool:
        """Apply one watch event; returns False when the stream must be abandoned for a re-LIST."""
        kind = ev.get("type")
        obj = ev.get("object") or {}
        rv = ((obj.get("metadata") or {}) if isinstance(obj, dict) else {}).get("resourceVersion")
        if kind == "ERROR":
            self.rv = None  # 410 Gone (or any watch error): history is gone, re-LIST
            return False
        if kind == "BOOKMARK":
            if rv:
                self.rv = str(rv)
            return True
        if not isinstance(obj, dict):
            return True
        self.events += 1
        if kind in ("ADDED", "MODIFIED"):
            self.view.upsert(obj, kind)
        elif kind == "DELETED":
            self.view.delete(obj)
        if rv:
            self.rv = str(rv)
        return True

    # -- loop -------------------------------------------------------------------
    def _open(self, client: KubeClient) -> LineStream:
        from urllib.parse import quote
        q = ["watch=1", "allowWatchBookmarks=true", f"timeoutSeconds={self.watch_timeout}"]
        if self.rv:
            q.append("resourceVersion=" + quote(self.rv, safe=""))
        if self.opts.label_selector:
            q.append("labelSelector=" + quote(self.opts.label_selector, safe=""))
        path = "/api/v1/nodes?" + "&".join(q)
        conn = client._connection()
        resp = conn.open_stream("GET", path, client._headers(), read_timeout=self.debounce or None)
        if not isinstance(resp, LineStream):
            client.close()
            if resp.status == 401:
                self.cluster.invalidate_credentials()
            if resp.status == 410:
                self.rv = None
                raise _Relist()
            raise ApiException(resp.status, resp.reason, resp.header_dict(), resp.text)
        return resp

    def run(self, evaluate: Callable[[ScanResult], Any], report: Callable[[Any], None], max_reports: int = 0,
            duration: float = 0.0, should_stop: Optional[Callable[[], bool]] = None) -> int:
        """Follow the cluster until ``max_reports`` reports were emitted, ``duration`` seconds passed or
        ``should_stop()`` turns true (checked at least every ``STOP_POLL_S``, and before every report: a
        replica that lost its leader Lease never reports after it).

        ``evaluate(scan)`` turns a state into a result (health gate applied); ``report(result)`` is
        called for the first result and for every result whose :func:`outcome_signature` differs
        from the previous report's.  Returns the number of reports.
        """
        deadline = time.monotonic() + duration if duration > 0 else None
        reports = 0
        last_sig: Optional[Tuple[Any, ...]] = None
        failures = 0
        last_eval = time.monotonic()

        def consider() -> None:
            nonlocal reports, last_sig, last_eval
            last_eval = time.monotonic()
            result = evaluate(self.view.scan_result())
            sig = outcome_signature(result)
            if sig != last_sig and not (should_stop is not None and should_stop()):
                last_sig = sig
                report(result)
                reports += 1

        def done() -> bool:
            return (max_reports > 0 and reports >= max_reports) or (
                deadline is not None and time.monotonic() >= deadline) or (should_stop is not None and should_stop())

        while not done():
            client = KubeClient(self.cluster, timeout=self.opts.kube_timeout, retries=self.opts.kube_retries)
            try:
                if self.rv is None:
                    self.relist(client)
                    consider()
                    if done():
                        break
                stream = self._open(client)
                failures = 0
                pending = False
                while not done():
                    wait = self.debounce if pending else self.watch_timeout + 30
                    if self.recheck > 0:
                        wait = min(wait, max(0.01, last_eval + self.recheck - time.monotonic()))
                    if should_stop is not None:
                        wait = min(wait, STOP_POLL_S)
                    if deadline is not None:
                        remaining = deadline - time.monotonic()
                        if remaining <= 0:
                            break
                        wait = min(wait, remaining)
                    client._connection().sock.settimeout(wait)
                    try:
                        line = stream.next_line()
                    except EOFError:
                        break  # server ended the watch (timeoutSeconds): re-open from self.rv
                    if line is None:  # quiet for `debounce` s: evaluate the batch; or time for a recheck
                        if pending or (self.recheck > 0 and time.monotonic() - last_eval >= self.recheck):
                            consider()
                            pending = False
                        continue
                    try:
                        ev = json.loads(line)
                    except ValueError:
                        continue
                    if not self.apply(ev):
                        break
                    pending = pending or ev.get("type") != "BOOKMARK"
                if pending:
                    consider()
            except _Relist:
                pass
            except (HTTPError, ApiException, OSError, ValueError) as e:
                failures += 1
                if failures > 3:
                    self.rv = None  # persistent trouble: start over from a LIST
                if isinstance(e, ApiException) and (e.status == 403 or (e.status == 401 and failures > 3)):
                    raise  # RBAC denies it / credentials stay rejected after re-reads: not transient
                self.sleep(self.backoff.delay(min(failures, 6)))
            finally:
                client.close()
        return reports


class _Relist(Exception):
    pass
