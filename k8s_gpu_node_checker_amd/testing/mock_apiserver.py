"""Mock kube-apiserver: ``GET/PATCH /api/v1/nodes`` over HTTP/1.1.

The single ``list_node()`` call is the reference's only cluster seam
(``check-gpu-node.py:217``); anything that serves a ``NodeList`` at
``/api/v1/nodes`` is a complete fake cluster.  Features:

* ``limit`` / ``continue`` pagination (pages pre-serialised and cached, so
  the server's own JSON encoding does not pollute client-side timings)
* ``GET /api/v1/nodes/{name}``, JSON merge-``PATCH`` of a node (the node
  agent's annotation write) with ``metadata.resourceVersion`` preconditions
  (409 Conflict on a stale version, ``conflict_first`` injected conflicts),
  ``POST /api/v1/namespaces/{ns}/events`` (kept in ``k8s_events``)
* bearer-token auth (401 on mismatch), TLS (given a cert/key)
* fault injection: fixed status (``403``/``500``), ``fail_first`` transient
  errors with ``Retry-After``, an expired-``continue`` 410, response delay,
  connection reset
* ``?watch=1`` event streams (chunked, one JSON event per line): ADDED /
  MODIFIED / DELETED from every change (``set_nodes``, PATCH, ``add_node``,
  ``delete_node``), BOOKMARKs with ``allowWatchBookmarks``, ``timeoutSeconds``,
  and the 410 ``ERROR`` event for a ``resourceVersion`` older than the log
* request log for assertions

Run standalone (used by ``bench.py`` in its own process, so the client under
test does not share a GIL with the server)::

    python -m k8s_gpu_node_checker_amd.testing.mock_apiserver --nodes 8 --kind amd --port 0
"""

from __future__ import annotations

import argparse
import copy
import json
import os
import socket
import struct
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional
from urllib.parse import parse_qs, unquote, urlsplit

from . import fixtures


def _name(node: Dict[str, Any]) -> Optional[str]:
    return (node.get("metadata") or {}).get("name")


class ClusterState:
    EVENT_LOG = 10000  # events kept for watchers; older resourceVersions get 410 Gone

    def __init__(self, nodes: List[Dict[str, Any]]):
        self.lock = threading.Lock()
        self.changed = threading.Condition(self.lock)
        self.nodes = nodes
        self.rv = 1000
        self._cache: Dict[Any, bytes] = {}
        self.events: List[Any] = []  # (rv, type, node snapshot)
        self.closed = False

    def _event(self, kind: str, node: Dict[str, Any]) -> None:
        """Record one change (lock held): bump the resourceVersion, stamp it on the node, wake watchers."""
        self.rv += 1
        if isinstance(node.get("metadata"), dict):
            node["metadata"]["resourceVersion"] = str(self.rv)
        self.events.append((self.rv, kind, copy.deepcopy(node)))
        if len(self.events) > self.EVENT_LOG:
            del self.events[:len(self.events) - self.EVENT_LOG]
        self._cache.clear()
        self.changed.notify_all()

    def set_nodes(self, nodes: List[Dict[str, Any]]) -> None:
        """Replace the cluster; watchers see the difference as DELETED / ADDED / MODIFIED events."""
        with self.lock:
            old = {_name(n): n for n in self.nodes}
            new = {_name(n): n for n in nodes}
            for name, n in old.items():
                if name not in new:
                    self._event("DELETED", n)
            for name, n in new.items():
                if name not in old:
                    self._event("ADDED", n)
                elif json.dumps(n, sort_keys=True) != json.dumps(old[name], sort_keys=True):
                    self._event("MODIFIED", n)
            self.nodes = nodes
            self.rv += 1
            self._cache.clear()

    def add_node(self, node: Dict[str, Any]) -> None:
        with self.lock:
            self.nodes.append(node)
            self._event("ADDED", node)

    def delete_node(self, name: str) -> bool:
        with self.lock:
            for i, n in enumerate(self.nodes):
                if _name(n) == name:
                    del self.nodes[i]
                    self._event("DELETED", n)
                    return True
            return False

    def events_after(self, rv: int) -> Optional[List[Any]]:
        """Events newer than ``rv`` (lock held); ``None`` if ``rv`` is older than the log."""
        if self.events and rv < self.events[0][0] - 1:
            return None
        return [e for e in self.events if e[0] > rv]

    def close(self) -> None:
        with self.lock:
            self.closed = True
            self.changed.notify_all()

    def page(self, limit: int, start: int) -> bytes:
        key = (limit, start, self.rv)
        with self.lock:
            body = self._cache.get(key)
            if body is None:
                items = self.nodes[start:start + limit] if limit > 0 else self.nodes[start:]
                nxt = start + len(items)
                cont = f"c{nxt}.{self.rv}" if (limit > 0 and nxt < len(self.nodes)) else None
                body = json.dumps(fixtures.node_list(items, cont, str(self.rv)), separators=(",", ":")).encode()
                self._cache[key] = body
            return body

    def find(self, name: str) -> Optional[Dict[str, Any]]:
        for n in self.nodes:
            if (n.get("metadata") or {}).get("name") == name:
                return n
        return None

    def patch(self, name: str, patch: Dict[str, Any], strategic: bool = False) -> Optional[Dict[str, Any]]:
        with self.lock:
            node = self.find(name)
            if node is None:
                return None
            conds = (patch.get("status") or {}).get("conditions") if strategic else None
            if conds is not None:
                # strategic merge: status.conditions is a list merged by its `type` key
                patch = copy.deepcopy(patch)
                patch["status"].pop("conditions")
                have = node.setdefault("status", {}).setdefault("conditions", [])
                for c in conds:
                    for i, old in enumerate(have):
                        if old.get("type") == c.get("type"):
                            have[i] = dict(old, **c)
                            break
                    else:
                        have.append(c)
            _merge_patch(node, patch)
            self._event("MODIFIED", node)
            return copy.deepcopy(node)


def _merge_patch(target: Dict[str, Any], patch: Dict[str, Any]) -> None:
    for k, v in patch.items():
        if v is None:
            target.pop(k, None)
        elif isinstance(v, dict) and isinstance(target.get(k), dict):
            _merge_patch(target[k], v)
        else:
            target[k] = copy.deepcopy(v)


LEASES = "/apis/coordination.k8s.io/v1/namespaces/"
SLICES = "/apis/discovery.k8s.io/v1/namespaces/"


def _selector_matches(selector: str, labels: Dict[str, Any]) -> bool:
    """Equality-based label selectors (``k=v,k2==v2,k3!=v3``): what the clients here send."""
    for term in filter(None, (t.strip() for t in selector.split(","))):
        if "!=" in term:
            k, v = term.split("!=", 1)
            if labels.get(k.strip()) == v.strip():
                return False
        else:
            k, v = term.replace("==", "=").split("=", 1)
            if labels.get(k.strip()) != v.strip():
                return False
    return True


def endpoint_slice(namespace: str, service: str, endpoints: List[Dict[str, Any]], port: int = 9464,
                   name: Optional[str] = None) -> Dict[str, Any]:
    """A ``discovery.k8s.io/v1`` EndpointSlice of ``service``; each endpoint dict has ``node`` and ``ip`` and
    optionally ``ready`` / ``terminating`` (omitted conditions are left out, as the apiserver does)."""
    eps = []
    for e in endpoints:
        cond = {k: e[k] for k in ("ready", "serving", "terminating") if k in e}
        ep: Dict[str, Any] = {"addresses": [e["ip"]], "nodeName": e["node"], "conditions": cond,
                              "targetRef": {"kind": "Pod", "namespace": namespace, "name": f"{service}-{e['node']}"}}
        eps.append(ep)
    return {"kind": "EndpointSlice", "apiVersion": "discovery.k8s.io/v1", "addressType": "IPv4",
            "metadata": {"name": name or f"{service}-{len(eps)}", "namespace": namespace,
                         "labels": {"kubernetes.io/service-name": service,
                                    "endpointslice.kubernetes.io/managed-by": "endpointslice-controller.k8s.io"}},
            "endpoints": eps, "ports": [{"name": "probe", "port": port, "protocol": "TCP"}]}


class MockConfig:
    def __init__(self, token: Optional[str] = None, status: Optional[int] = None, fail_first: int = 0,
                 fail_status: int = 503, retry_after: Optional[str] = None, delay: float = 0.0,
                 expire_continue: bool = False, reset: bool = False, gzip: bool = False,
                 chunked: bool = False, bookmark_interval: float = 1.0, conflict_first: int = 0):
        self.token = token
        self.status = status
        self.fail_first = fail_first
        self.fail_status = fail_status
        self.retry_after = retry_after
        self.delay = delay
        self.expire_continue = expire_continue
        self.reset = reset
        self.gzip = gzip
        self.chunked = chunked
        self.bookmark_interval = bookmark_interval
        self.conflict_first = conflict_first  # 409 for the first N PATCHes that carry a resourceVersion


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"
    server: "MockApiServer"  # type: ignore[assignment]

    def log_message(self, fmt: str, *args: Any) -> None:  # quiet
        pass

    def setup(self) -> None:
        super().setup()
        # a response's segments go out as written: with Nagle on, the body's write waited for the client's ACK of the
        # head, which a keep-alive client past its first exchanges delays by up to 40 ms (40 ms per agent PATCH)
        self.connection.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    def _send(self, status: int, body: bytes, extra: Optional[Dict[str, str]] = None,
              reason: Optional[str] = None) -> None:
        if self.server.cfg.gzip and "gzip" in (self.headers.get("Accept-Encoding") or ""):
            import gzip
            body = gzip.compress(body, compresslevel=1)
            extra = dict(extra or {}, **{"Content-Encoding": "gzip"})
        self.send_response(status, reason)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.send_header("Audit-Id", "00000000-0000-0000-0000-000000000000")
        for k, v in (extra or {}).items():
            self.send_header(k, v)
        self.end_headers()
        self.wfile.write(body)  # a second segment: TCP_NODELAY (setup) sends it without waiting for an ACK

    def _status_body(self, code: int, reason: str, message: str) -> bytes:
        return json.dumps({"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
                           "message": message, "reason": reason, "code": code}).encode()

    def _pre(self) -> bool:
        srv = self.server
        cfg = srv.cfg
        srv.log.append({"method": self.command, "path": self.path,
                        "auth": self.headers.get("Authorization"), "ts": time.time()})
        if cfg.delay:
            time.sleep(cfg.delay)
        if cfg.reset:
            self.connection.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
            self.close_connection = True
            self.connection.close()
            return False
        if cfg.token is not None and self.headers.get("Authorization") != f"Bearer {cfg.token}":
            self._send(401, self._status_body(401, "Unauthorized", "Unauthorized"), reason="Unauthorized")
            return False
        if cfg.status is not None:
            msg = 'nodes is forbidden: User "system:anonymous" cannot list resource "nodes" in API group "" at the cluster scope' \
                if cfg.status == 403 else "internal error"
            reason = {403: "Forbidden", 500: "Internal Server Error", 404: "Not Found"}.get(cfg.status, "Error")
            self._send(cfg.status, self._status_body(cfg.status, reason.replace(" ", ""), msg), reason=reason)
            return False
        with srv.lock:
            failing = srv.failures_left > 0
            if failing:
                srv.failures_left -= 1
        if failing:
            extra = {"Retry-After": cfg.retry_after} if cfg.retry_after else None
            self._send(cfg.fail_status, self._status_body(cfg.fail_status, "ServiceUnavailable", "try again"), extra)
            return False
        return True

    def do_GET(self) -> None:  # noqa: N802
        if not self._pre():
            return
        parts = urlsplit(self.path)
        path = parts.path
        if path == "/api/v1/nodes":
            q = parse_qs(parts.query)
            if q.get("watch", ["0"])[0] in ("1", "true"):
                self._watch(q)
                return
            limit = int(q.get("limit", ["0"])[0] or 0)
            cont = q.get("continue", [None])[0]
            start = 0
            if cont:
                if self.server.cfg.expire_continue:
                    self._send(410, self._status_body(410, "Expired", "The provided continue parameter is too old"),
                               reason="Gone")
                    return
                try:
                    start = int(cont[1:].split(".")[0])
                except ValueError:
                    self._send(400, self._status_body(400, "BadRequest", "invalid continue token"))
                    return
            body = self.server.state.page(limit, start)
            if self.server.cfg.chunked:
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Transfer-Encoding", "chunked")
                self.end_headers()
                for i in range(0, len(body), 4096):
                    piece = body[i:i + 4096]
                    self.wfile.write(b"%x\r\n" % len(piece) + piece + b"\r\n")
                self.wfile.write(b"0\r\n\r\n")
                return
            self._send(200, body)
            return
        if path.startswith("/api/v1/nodes/"):
            node = self.server.state.find(unquote(path[len("/api/v1/nodes/"):]))
            if node is None:
                self._send(404, self._status_body(404, "NotFound", "node not found"), reason="Not Found")
            else:
                self._send(200, json.dumps(node).encode())
            return
        if path in ("/healthz", "/readyz", "/livez"):
            self._send(200, b"ok")
            return
        if path.startswith(LEASES):
            self._lease("GET", path, b"")
            return
        if path.startswith(SLICES) and path.endswith("/endpointslices"):
            self._endpoint_slices(unquote(path[len(SLICES):-len("/endpointslices")]), parse_qs(parts.query))
            return
        self._send(404, self._status_body(404, "NotFound", "not found"), reason="Not Found")

    def _endpoint_slices(self, namespace: str, q: Dict[str, List[str]]) -> None:
        """``GET .../namespaces/{ns}/endpointslices?labelSelector=&limit=&continue=`` over
        ``server.endpoint_slices``; ``server.endpoint_slices_status`` fails it (e.g. 403 without the Role)."""
        srv = self.server
        if srv.endpoint_slices_status is not None:
            code = srv.endpoint_slices_status
            reason = {403: "Forbidden", 404: "NotFound"}.get(code, "InternalError")
            msg = (f'endpointslices.discovery.k8s.io is forbidden: User "system:anonymous" cannot list resource '
                   f'"endpointslices" in API group "discovery.k8s.io" in the namespace "{namespace}"'
                   if code == 403 else "not available")
            self._send(code, self._status_body(code, reason, msg), reason=reason)
            return
        sel = q.get("labelSelector", [""])[0]
        items = [sl for sl in srv.endpoint_slices if (sl.get("metadata") or {}).get("namespace") == namespace
                 and _selector_matches(sel, (sl.get("metadata") or {}).get("labels") or {})]
        limit = int(q.get("limit", ["0"])[0] or 0)
        start = int(q.get("continue", ["0"])[0] or 0)
        page = items[start:start + limit] if limit else items[start:]
        meta: Dict[str, Any] = {"resourceVersion": "1"}
        if limit and start + limit < len(items):
            meta["continue"] = str(start + limit)
        self._send(200, json.dumps({"kind": "EndpointSliceList", "apiVersion": "discovery.k8s.io/v1",
                                    "metadata": meta, "items": page}).encode())

    def _lease(self, method: str, path: str, body: bytes) -> None:
        """``coordination.k8s.io/v1`` Leases: GET / POST (create, 409 if it exists) / PUT (update, 409 unless the
        body carries the current ``resourceVersion``).  ``server.lease_status`` fails every lease call with that
        status (a replica that lost the apiserver)."""
        srv = self.server
        parts = path[len(LEASES):].strip("/").split("/")
        if srv.lease_status is not None:
            self._send(srv.lease_status, self._status_body(srv.lease_status, "InternalError", "lease store unavailable"))
            return
        if len(parts) < 2 or parts[1] != "leases" or len(parts) > 3 or (method == "POST") != (len(parts) == 2):
            self._send(404, self._status_body(404, "NotFound", "not found"), reason="Not Found")
            return
        ns = unquote(parts[0])
        try:
            obj = json.loads(body) if body else None
        except ValueError:
            obj = None
        with srv.lock:
            if method == "GET":
                cur = srv.leases.get((ns, unquote(parts[2])))
                if cur is None:
                    self._send(404, self._status_body(404, "NotFound", "leases not found"), reason="Not Found")
                else:
                    self._send(200, json.dumps(cur).encode())
                return
            if not isinstance(obj, dict) or not isinstance(obj.get("metadata"), dict):
                self._send(400, self._status_body(400, "BadRequest", "invalid lease"))
                return
            name = obj["metadata"].get("name") if method == "POST" else unquote(parts[2])
            cur = srv.leases.get((ns, name))
            if method == "POST" and cur is not None:
                self._send(409, self._status_body(409, "AlreadyExists", f'leases "{name}" already exists'),
                           reason="Conflict")
                return
            if method == "PUT":
                if cur is None:
                    self._send(404, self._status_body(404, "NotFound", "leases not found"), reason="Not Found")
                    return
                if obj["metadata"].get("resourceVersion") != cur["metadata"]["resourceVersion"]:
                    self._send(409, self._status_body(409, "Conflict", "the object has been modified"),
                               reason="Conflict")
                    return
            srv.lease_rv += 1
            obj["metadata"].update(name=name, namespace=ns, resourceVersion=str(srv.lease_rv))
            srv.leases[(ns, name)] = obj
            srv.lease_writes.append((method, name, (obj.get("spec") or {}).get("holderIdentity")))
        self._send(201 if method == "POST" else 200, json.dumps(obj).encode(),
                   reason="Created" if method == "POST" else None)

    def do_PUT(self) -> None:  # noqa: N802
        length = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(length) if length else b""
        if not self._pre():
            return
        path = urlsplit(self.path).path
        if path.startswith(LEASES):
            self._lease("PUT", path, body)
            return
        self._send(405, self._status_body(405, "MethodNotAllowed", "PUT is served for leases only"))

    def _watch(self, q: Dict[str, List[str]]) -> None:
        """Stream node events (chunked, one JSON object per line) like the apiserver's watch."""
        st = self.server.state
        timeout = float(q.get("timeoutSeconds", ["30"])[0] or 30)
        bookmarks = q.get("allowWatchBookmarks", ["false"])[0] in ("1", "true")
        rv_param = q.get("resourceVersion", [""])[0]
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Transfer-Encoding", "chunked")
        self.end_headers()

        def send(ev: Dict[str, Any]) -> None:
            line = json.dumps(ev, separators=(",", ":")).encode() + b"\n"
            self.wfile.write(b"%x\r\n" % len(line) + line + b"\r\n")
            self.wfile.flush()

        with st.lock:
            if rv_param in ("", "0"):  # "any": synthetic ADDED for the current state, then follow
                initial = [("ADDED", copy.deepcopy(n)) for n in st.nodes]
                last = st.rv
            else:
                initial = []
                last = int(rv_param)
                if st.events_after(last) is None:
                    initial = None
        try:
            if initial is None:
                send({"type": "ERROR", "object": {"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                                  "message": f"too old resource version: {rv_param}",
                                                  "reason": "Expired", "code": 410}})
            else:
                for kind, node in initial:
                    send({"type": kind, "object": node})
                deadline = time.monotonic() + timeout
                next_bookmark = time.monotonic() + self.server.cfg.bookmark_interval
                while True:
                    now = time.monotonic()
                    if now >= deadline:
                        break
                    with st.lock:
                        evs = st.events_after(last)
                        if evs == [] and not st.closed:
                            st.changed.wait(min(deadline, next_bookmark if bookmarks else deadline) - now)
                            evs = st.events_after(last)
                        closed = st.closed
                        cur = st.rv
                    if closed:
                        break
                    if evs is None:
                        send({"type": "ERROR", "object": {"kind": "Status", "apiVersion": "v1", "status": "Failure",
                                                          "message": "too old resource version", "reason": "Expired",
                                                          "code": 410}})
                        break
                    for rv, kind, node in evs:
                        send({"type": kind, "object": node})
                        last = rv
                    if bookmarks and time.monotonic() >= next_bookmark:
                        send({"type": "BOOKMARK", "object": {"kind": "Node", "apiVersion": "v1",
                                                             "metadata": {"resourceVersion": str(max(cur, last))}}})
                        last = max(cur, last)
                        next_bookmark = time.monotonic() + self.server.cfg.bookmark_interval
            self.wfile.write(b"0\r\n\r\n")
            self.wfile.flush()
        except OSError:
            pass
        self.close_connection = True

    def do_PATCH(self) -> None:  # noqa: N802
        length = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(length) if length else b""
        if not self._pre():
            return
        path = urlsplit(self.path).path
        if not path.startswith("/api/v1/nodes/"):
            self._send(404, self._status_body(404, "NotFound", "not found"), reason="Not Found")
            return
        try:
            patch = json.loads(body or b"{}")
        except ValueError:
            self._send(400, self._status_body(400, "BadRequest", "invalid patch"))
            return
        name = unquote(path[len("/api/v1/nodes/"):])
        meta = patch.get("metadata") if isinstance(patch, dict) else None
        want_rv = meta.pop("resourceVersion", None) if isinstance(meta, dict) else None
        if want_rv is not None:
            # optimistic concurrency: the write only applies to the object version it was computed from
            srv = self.server
            with srv.lock:
                inject = srv.conflicts_left > 0
                if inject:
                    srv.conflicts_left -= 1
            cur = srv.state.find(name[:-len("/status")] if name.endswith("/status") else name)
            have = ((cur or {}).get("metadata") or {}).get("resourceVersion")
            if inject or (have is not None and str(want_rv) != str(have)):
                self._send(409, self._status_body(
                    409, "Conflict", f'Operation cannot be fulfilled on nodes "{name}": the object has been '
                    "modified; please apply your changes to the latest version and try again"), reason="Conflict")
                return
        strategic = "strategic-merge-patch" in (self.headers.get("Content-Type") or "")
        if name.endswith("/status"):
            name = name[:-len("/status")]
            patch = {"status": patch.get("status") or {}}  # the status subresource ignores other fields
        node = self.server.state.patch(name, patch, strategic)
        if node is None:
            self._send(404, self._status_body(404, "NotFound", "node not found"), reason="Not Found")
        else:
            self._send(200, json.dumps(node).encode())

    def do_POST(self) -> None:  # noqa: N802
        """``POST /api/v1/namespaces/{ns}/events``: stored in ``server.k8s_events`` (``generateName`` honoured)."""
        length = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(length) if length else b""
        if not self._pre():
            return
        if urlsplit(self.path).path.startswith(LEASES):
            self._lease("POST", urlsplit(self.path).path, body)
            return
        parts = urlsplit(self.path).path.strip("/").split("/")
        if len(parts) != 5 or parts[:3] != ["api", "v1", "namespaces"] or parts[4] != "events":
            self._send(404, self._status_body(404, "NotFound", "not found"), reason="Not Found")
            return
        try:
            ev = json.loads(body or b"{}")
        except ValueError:
            ev = None
        if not isinstance(ev, dict):
            self._send(400, self._status_body(400, "BadRequest", "invalid event"))
            return
        srv = self.server
        with srv.lock:
            srv.event_seq += 1
            meta = ev.get("metadata") if isinstance(ev.get("metadata"), dict) else {}
            ev["metadata"] = meta
            meta["namespace"] = unquote(parts[3])
            if not meta.get("name"):
                meta["name"] = (meta.get("generateName") or "event.") + f"{srv.event_seq:08x}"
            srv.k8s_events.append(ev)
        self._send(201, json.dumps(ev).encode(), reason="Created")


class MockApiServer(ThreadingHTTPServer):
    daemon_threads = True
    allow_reuse_address = True
    request_queue_size = 256

    def __init__(self, nodes: List[Dict[str, Any]], host: str = "127.0.0.1", port: int = 0,
                 cfg: Optional[MockConfig] = None, certfile: Optional[str] = None, keyfile: Optional[str] = None):
        super().__init__((host, port), _Handler)
        self.state = ClusterState(nodes)
        self.cfg = cfg or MockConfig()
        self.lock = threading.Lock()
        self.failures_left = self.cfg.fail_first
        self.conflicts_left = self.cfg.conflict_first
        self.log: List[Dict[str, Any]] = []
        self.k8s_events: List[Dict[str, Any]] = []  # core/v1 Events POSTed by clients
        self.event_seq = 0
        self.leases: Dict[Any, Dict[str, Any]] = {}  # (namespace, name) -> coordination.k8s.io/v1 Lease
        self.lease_rv = 0
        self.lease_writes: List[Any] = []  # (method, name, holderIdentity) of every accepted write
        self.lease_status: Optional[int] = None
        self.endpoint_slices: List[Dict[str, Any]] = []  # discovery.k8s.io/v1 EndpointSlices (any namespace)
        self.endpoint_slices_status: Optional[int] = None
        self.scheme = "http"
        if certfile:
            import ssl
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(certfile, keyfile)
            self.socket = ctx.wrap_socket(self.socket, server_side=True)
            self.scheme = "https"
        self._thread: Optional[threading.Thread] = None

    @property
    def url(self) -> str:
        host, port = self.server_address[:2]
        return f"{self.scheme}://{host}:{port}"

    def start(self) -> "MockApiServer":
        self._thread = threading.Thread(target=self.serve_forever, kwargs={"poll_interval": 0.05}, daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self.state.close()  # end open watch streams
        self.shutdown()
        self.server_close()

    def __enter__(self) -> "MockApiServer":
        return self.start()

    def __exit__(self, *exc: Any) -> None:
        self.stop()

    def kubeconfig(self, path: str, token: Optional[str] = None, extra_cluster: Optional[Dict[str, Any]] = None) -> str:
        return write_kubeconfig(path, self.url, token if token is not None else self.cfg.token, extra_cluster)


def write_kubeconfig(path: str, server: str, token: Optional[str] = None,
                     extra_cluster: Optional[Dict[str, Any]] = None, fmt: str = "yaml") -> str:
    cluster: Dict[str, Any] = {"server": server}
    if extra_cluster:
        cluster.update(extra_cluster)
    user: Dict[str, Any] = {"token": token} if token else {}
    cfg = {"apiVersion": "v1", "kind": "Config", "current-context": "mock",
           "clusters": [{"name": "mock", "cluster": cluster}],
           "contexts": [{"name": "mock", "context": {"cluster": "mock", "user": "mock-user"}}],
           "users": [{"name": "mock-user", "user": user}]}
    with open(path, "w", encoding="utf-8") as f:
        if fmt == "json":
            json.dump(cfg, f)
        else:
            import yaml
            yaml.safe_dump(cfg, f)
    return path


def build_nodes(n: int, kind: str, not_ready: int = 0, with_health: bool = False,
                gpus_per_node: int = 8, annotation_encoding: str = "json") -> List[Dict[str, Any]]:
    return fixtures.cluster(n, kind, not_ready=range(not_ready), with_health=with_health, gpus_per_node=gpus_per_node,
                            annotation_encoding=annotation_encoding)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="mock kube-apiserver for k8s-gpu-node-checker-amd")
    ap.add_argument("--nodes", type=int, default=8)
    ap.add_argument("--kind", default="amd", choices=("amd", "nvidia", "mixed", "cpu"))
    ap.add_argument("--not-ready", type=int, default=0)
    ap.add_argument("--gpus-per-node", type=int, default=8)
    ap.add_argument("--with-health", action="store_true")
    ap.add_argument("--annotation-encoding", choices=("json", "gzip"), default="json",
                    help="how the --with-health report annotations are written (the agent's flag of that name)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--token")
    ap.add_argument("--golden", help="serve a golden fixture instead of a generated cluster")
    ap.add_argument("--cpu", type=int, help="run on this CPU only (bench.py: the server beside the checking process)")
    args = ap.parse_args(argv)
    if args.cpu is not None:
        try:
            os.sched_setaffinity(0, {args.cpu})  # before any thread: the request threads inherit it
        except (OSError, AttributeError):
            pass
    nodes = fixtures.golden(args.golden) if args.golden else build_nodes(
        args.nodes, args.kind, args.not_ready, args.with_health, args.gpus_per_node, args.annotation_encoding)
    srv = MockApiServer(nodes, args.host, args.port, MockConfig(token=args.token))
    print(json.dumps({"url": srv.url, "port": srv.server_address[1], "nodes": len(nodes)}), flush=True)
    try:
        srv.serve_forever(poll_interval=0.2)
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
