"""kube-apiserver client: paginated node LIST, node GET/PATCH (SURVEY §7.2 layer 2).

Replaces ``CoreV1Api().list_node()`` (reference ``check-gpu-node.py:217``),
which is one unpaginated GET with no timeout and no retry.  Here:

* ``GET /api/v1/nodes?limit=<page>`` then ``&continue=<token>`` on one
  keep-alive connection; pages are scanned as they arrive (the native scanner
  never holds more than one page), so memory is bounded by the page size.
* an expired ``continue`` token (HTTP 410) falls back to one full LIST, as
  client-go's pager does.
* every request has a timeout; idempotent requests are retried on connection
  errors, 429 and 5xx with jittered exponential backoff honouring
  ``Retry-After``.
* ``Accept-Encoding: gzip`` is sent to non-loopback servers (a 1000-node
  NodeList shrinks ~15x on the wire); loopback skips the inflate cost.
* failures raise :class:`ApiException` / :class:`TransportError` whose
  ``str()`` matches what the reference would have printed.
"""

from __future__ import annotations

import time
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

from ..models.node import ScanResult
from ..models.resources import GPU_RESOURCE_KEYS
from ..utils.backoff import Backoff
from ..utils.http import Connection, HTTPError, Response
from ..utils.urls import quote
from .config import ClusterConnection
from .errors import ApiException, TransportError

USER_AGENT = "k8s-gpu-node-checker-amd/0.1 (MI355X)"


def _continue_from_prefix(prefix: bytes) -> Optional[str]:
    """``metadata.continue`` from the head of a NodeList body, if it precedes ``items``.

    Only the unescaped form apiservers emit is accepted (opaque base64 tokens);
    anything else returns ``None`` and pagination simply is not pipelined.
    """
    i = prefix.find(b'"continue"')
    if i < 0:
        return None
    items = prefix.find(b'"items"')
    if 0 <= items < i:
        return None
    j = prefix.find(b'"', prefix.find(b":", i + 10) + 1)
    if j < 0:
        return None
    k = prefix.find(b'"', j + 1)
    if k < 0 or b"\\" in prefix[j:k]:
        return None
    tok = prefix[j + 1:k]
    return tok.decode("ascii", "strict") if tok and tok.isascii() else None
_RETRY_STATUS = frozenset((429, 500, 502, 503, 504))
_LOOPBACK = ("127.", "localhost", "::1", "[::1]")


class _PageReader:
    """Receives one pipelined LIST page on its own thread.

    Socket reads release the GIL, and so does pass 1 of the native NodeList
    scan, so page k+1 streams in while page k is being scanned.  Once the page
    is in, this thread also runs page k+1's pass 1 (``fastpath.prescan``), which
    leaves only pass 2 for the main thread.
    """

    def __init__(self, conn: Connection, path: str, keys: Optional[Sequence[str]] = None):
        import threading
        self.conn = conn
        self.path = path
        self.keys = keys
        self.resp: Optional[Response] = None
        self.pre: Any = None
        self.thread = threading.Thread(target=self._run, name="list-prefetch", daemon=True)
        self.thread.start()

    def _run(self) -> None:
        try:
            self.resp = self.conn.read_pending("GET", self.path)
        except Exception:  # transport trouble: the caller re-requests the page normally
            self.resp = None
            return
        if self.keys is not None and 200 <= self.resp.status < 300:
            try:
                from ..ops import fastpath
                self.pre = fastpath.prescan(self.resp.body, self.keys)
            except Exception:  # the main thread scans the page itself
                self.pre = None

    def join(self) -> Optional[Response]:
        self.thread.join()
        return self.resp


class KubeClient:
    def __init__(self, cluster: ClusterConnection, timeout: float = 30.0, retries: int = 2,
                 backoff: Optional[Backoff] = None, gzip: Optional[bool] = None,
                 sleep=time.sleep, tracer=None, pipeline: bool = True):
        self.cluster = cluster
        self.timeout = timeout
        self.retries = max(0, retries)
        self.backoff = backoff or Backoff(base=0.2, cap=5.0)
        self.sleep = sleep
        self.tracer = tracer
        self._conn: Optional[Connection] = None
        self._conn2: Optional[Connection] = None
        self.pipeline = pipeline
        host = cluster.server.split("://", 1)[-1]
        self.gzip = (not host.startswith(_LOOPBACK)) if gzip is None else gzip
        self.requests_made = 0

    # -- plumbing -------------------------------------------------------------
    def _connection(self) -> Connection:
        if self._conn is None:
            ctx = self.cluster.ssl_context() if self.cluster.server.startswith("https") else None
            self._conn = Connection(self.cluster.server, timeout=self.timeout, ssl_context=ctx,
                                    server_hostname=self.cluster.tls_server_name,
                                    proxy_url=self.cluster.proxy_url,
                                    tracer=self.tracer if getattr(self.tracer, "live", False) else None)
        return self._conn

    def close(self) -> None:
        for c in (self._conn, self._conn2):
            if c is not None:
                c.close()
        self._conn = self._conn2 = None

    def __enter__(self) -> "KubeClient":
        return self

    def __exit__(self, *exc: Any) -> None:
        self.close()

    def _headers(self, content_type: Optional[str] = None) -> Dict[str, str]:
        headers = {"Accept": "application/json", "User-Agent": USER_AGENT}
        headers.update(self.cluster.auth_headers())
        if self.gzip:
            headers["Accept-Encoding"] = "gzip"
        if content_type:
            headers["Content-Type"] = content_type
        return headers

    def request(self, method: str, path: str, body: Optional[bytes] = None,
                content_type: Optional[str] = None, idempotent: bool = True, peek=None) -> Response:
        headers = self._headers(content_type)
        attempt = 0
        reauth = False
        while True:
            conn = self._connection()
            self.requests_made += 1
            try:
                resp = conn.request(method, path, headers, body, peek)
            except HTTPError as e:
                if idempotent and attempt < self.retries and e.kind != "tls":
                    self.sleep(self.backoff.delay(attempt))
                    attempt += 1
                    continue
                raise TransportError(conn.scheme, conn.host, conn.port, path, e) from e
            if 200 <= resp.status < 300:
                return resp
            if resp.status == 401 and not reauth and self.cluster.invalidate_credentials():
                # rotated service-account token / expired exec credential: fetch fresh ones once
                reauth = True
                headers = self._headers(content_type)
                continue
            if idempotent and resp.status in _RETRY_STATUS and attempt < self.retries:
                self.sleep(self.backoff.delay(attempt, resp.header("Retry-After")))
                attempt += 1
                continue
            raise ApiException(resp.status, resp.reason, resp.header_dict(), resp.text)

    # -- nodes ----------------------------------------------------------------
    def _list_path(self, limit: int, cont: Optional[str], label_selector: Optional[str],
                   resource_version: Optional[str]) -> str:
        q = []
        if limit > 0:
            q.append(f"limit={limit}")
        if cont:
            q.append("continue=" + quote(cont))
        if label_selector:
            q.append("labelSelector=" + quote(label_selector))
        if resource_version is not None and not cont:
            q.append("resourceVersion=" + quote(resource_version))
        return "/api/v1/nodes" + ("?" + "&".join(q) if q else "")

    def scan_nodes(self, limit: int = 500, keys: Sequence[str] = GPU_RESOURCE_KEYS,
                   gpu_source: str = "capacity", want_extras: bool = False,
                   label_selector: Optional[str] = None,
                   resource_version: Optional[str] = None, annotation_mode: int = 2) -> ScanResult:
        """LIST all nodes (paginated) and classify them (reference ``list_gpu_nodes``, ``:215-226``)."""
        from ..ops import fastpath
        result = ScanResult()
        cont: Optional[str] = None
        prefetched: Dict[str, _PageReader] = {}  # next-page path -> reader of the request already sent

        def peek(prefix: bytes) -> None:
            # NodeList JSON carries metadata.continue *before* items: as soon as the head of page k
            # arrives, request page k+1 on a second connection, so the server produces (and the
            # kernel buffers) it while page k is still being received and scanned
            if not self.pipeline or prefetched:
                return
            token = _continue_from_prefix(prefix)
            if token is None:
                return
            nxt = self._list_path(limit, token, label_selector, resource_version)
            conn2 = self._spare_connection()
            try:
                conn2.send_only("GET", nxt, self._headers())
            except HTTPError:
                return
            prefetched[nxt] = _PageReader(conn2, nxt, keys)

        seen_tokens = set()
        while True:
            if cont is not None:
                if cont in seen_tokens:
                    # a continue token handed out twice (a misbehaving proxy or aggregator) would page forever,
                    # collecting the same nodes again: take one consistent full LIST instead, as on a 410
                    result = ScanResult()
                    resp = self.request("GET", self._list_path(0, None, label_selector, None))
                    fastpath.scan_page(resp.body, result, keys, gpu_source, want_extras, annotation_mode)
                    return result
                seen_tokens.add(cont)
            path = self._list_path(limit, cont, label_selector, resource_version)
            pre = None
            try:
                resp, pre = self._take_prefetched(prefetched, path)
                if resp is None:
                    resp = self.request("GET", path, peek=peek if limit > 0 else None)
            except ApiException as e:
                if e.status == 410 and cont:
                    # continue token expired mid-list: restart as one consistent full LIST
                    result = ScanResult()
                    resp = self.request("GET", self._list_path(0, None, label_selector, None))
                    fastpath.scan_page(resp.body, result, keys, gpu_source, want_extras, annotation_mode)
                    return result
                raise
            t0 = time.perf_counter()
            cont, _ = fastpath.scan_page(resp.body, result, keys, gpu_source, want_extras, annotation_mode, pre)
            if self.tracer is not None:
                self.tracer.add("parse", time.perf_counter() - t0)
            if not cont or limit <= 0:
                return result

    # -- pipelined pagination helpers ------------------------------------------
    def _spare_connection(self) -> Connection:
        if self._conn2 is None:
            ctx = self.cluster.ssl_context() if self.cluster.server.startswith("https") else None
            self._conn2 = Connection(self.cluster.server, timeout=self.timeout, ssl_context=ctx,
                                     server_hostname=self.cluster.tls_server_name, proxy_url=self.cluster.proxy_url)
        return self._conn2

    def _take_prefetched(self, prefetched: Dict[str, "_PageReader"],
                         path: str) -> Tuple[Optional[Response], Any]:
        """Collect the already-sent request for ``path`` (and its pass-1 prescan); swap its
        connection in as the primary."""
        reader = prefetched.pop(path, None)
        for other in prefetched.values():
            other.join()
        prefetched.clear()
        if reader is None:
            return None, None
        self.requests_made += 1
        conn2 = reader.conn
        resp = reader.join()
        if resp is None:
            return None, None  # fall back to a normal (retried) request
        # alternate: the connection that just answered becomes primary, the old primary the spare
        self._conn, self._conn2 = conn2, self._conn
        if 200 <= resp.status < 300:
            return resp, reader.pre
        if resp.status in _RETRY_STATUS:
            return None, None  # retried through request() with backoff
        raise ApiException(resp.status, resp.reason, resp.header_dict(), resp.text)

    def get_node(self, name: str) -> Dict[str, Any]:
        import json
        return json.loads(self.request("GET", "/api/v1/nodes/" + quote(name)).body)

    # -- discovery ------------------------------------------------------------
    def list_endpoint_slices(self, namespace: str, service: str, limit: int = 500) -> List[Dict[str, Any]]:
        """Every ``discovery.k8s.io/v1`` EndpointSlice of one Service (label ``kubernetes.io/service-name``),
        paged like the node LIST.  Needs RBAC ``endpointslices: list`` in ``namespace`` only."""
        import json
        base = (f"/apis/discovery.k8s.io/v1/namespaces/{quote(namespace)}/endpointslices"
                f"?labelSelector={quote('kubernetes.io/service-name=' + service)}&limit={int(limit)}")
        items: List[Dict[str, Any]] = []
        cont: Optional[str] = None
        seen = set()
        while True:
            doc = json.loads(self.request("GET", base + (f"&continue={quote(cont)}" if cont else "")).body)
            items.extend(x for x in doc.get("items") or [] if isinstance(x, dict))
            cont = (doc.get("metadata") or {}).get("continue") or None
            if not cont or cont in seen:
                return items
            seen.add(cont)

    def patch_node_condition(self, name: str, condition: Dict[str, Any]) -> Dict[str, Any]:
        """Upsert one ``status.conditions`` entry (strategic merge by ``type``; RBAC ``nodes/status: patch``).

        This is how node-problem-detector publishes custom node conditions; the
        kubelet preserves condition types it does not own.
        """
        import json
        body = json.dumps({"status": {"conditions": [condition]}}).encode()
        resp = self.request("PATCH", "/api/v1/nodes/" + quote(name) + "/status", body,
                            content_type="application/strategic-merge-patch+json", idempotent=True)
        return json.loads(resp.body) if resp.body else {}

    def patch_node_annotations(self, name: str, annotations: Dict[str, Optional[str]]) -> Dict[str, Any]:
        """JSON merge-patch ``metadata.annotations`` (needs RBAC ``nodes: patch``)."""
        import json
        body = json.dumps({"metadata": {"annotations": annotations}}).encode()
        resp = self.request("PATCH", "/api/v1/nodes/" + quote(name), body,
                            content_type="application/merge-patch+json", idempotent=True)
        return json.loads(resp.body) if resp.body else {}

    def patch_node_labels(self, name: str, labels: Dict[str, Optional[str]]) -> Dict[str, Any]:
        """JSON merge-patch ``metadata.labels`` (``None`` removes a label; RBAC ``nodes: patch``)."""
        import json
        body = json.dumps({"metadata": {"labels": labels}}).encode()
        resp = self.request("PATCH", "/api/v1/nodes/" + quote(name), body,
                            content_type="application/merge-patch+json", idempotent=True)
        return json.loads(resp.body) if resp.body else {}

    def update_node_taints(self, name: str,
                           edit: Callable[[List[Dict[str, Any]]], Optional[List[Dict[str, Any]]]],
                           attempts: int = 5) -> Optional[List[Dict[str, Any]]]:
        """Read-modify-write of ``spec.taints`` under optimistic concurrency (client-go ``RetryOnConflict``).

        ``edit(taints)`` returns the new list, or ``None`` when nothing has to change.  A merge-patch
        replaces the whole list, so it carries the ``resourceVersion`` that was read: if anyone wrote the
        node in between (kubelet, node controller, an operator's ``kubectl taint``) the apiserver answers
        409 Conflict instead of dropping their change, and the cycle is redone on a fresh read.
        Returns the list written, or ``None`` if no write was needed.
        """
        import json
        path = "/api/v1/nodes/" + quote(name)
        attempts = max(1, attempts)
        for attempt in range(attempts):
            node = self.get_node(name)
            new = edit(list((node.get("spec") or {}).get("taints") or []))
            if new is None:
                return None
            patch: Dict[str, Any] = {"spec": {"taints": new}}
            rv = (node.get("metadata") or {}).get("resourceVersion")
            if rv:
                patch["metadata"] = {"resourceVersion": rv}
            try:
                self.request("PATCH", path, json.dumps(patch).encode(), content_type="application/merge-patch+json")
                return new
            except ApiException as e:
                if e.status != 409 or attempt + 1 >= attempts:
                    raise
                self.sleep(self.backoff.delay(attempt))
        return None

    def create_event(self, namespace: str, event: Dict[str, Any]) -> Dict[str, Any]:
        """``POST /api/v1/namespaces/{ns}/events`` (RBAC ``events: create``).  Not retried: a retry after
        a lost response would post the event twice."""
        import json
        resp = self.request("POST", f"/api/v1/namespaces/{quote(namespace)}/events",
                            json.dumps(event).encode(), content_type="application/json", idempotent=False)
        return json.loads(resp.body) if resp.body else {}
