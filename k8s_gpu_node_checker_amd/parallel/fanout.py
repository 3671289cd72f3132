"""Async per-node probe fan-out (SURVEY §7.2 layer 5 source (b), §6 takeaway 3).

When node agents serve their report over HTTP instead of (or besides) the
annotation, the checker fetches every GPU node's ``/probe`` concurrently:
one ``asyncio`` protocol per connection that parses the response as it
arrives (no aiohttp: 310 ms import; 3 % / 11 % less checker CPU than
``asyncio`` streams at 1,000 nodes, min / median of 12 interleaved runs:
no per-read coroutine resumptions, no ``wait_for`` task per request), an
``asyncio.Semaphore`` bounding
in-flight requests, a per-node timeout and one retry on connection errors.  Wall clock is ~max(node latency) instead of the sum, so it stays flat
as the cluster grows.

URL template placeholders: ``{name}`` (node name), ``{ip}`` (the node's
``InternalIP`` from ``status.addresses``) and ``{pod_ip}`` (the address of the
node agent pod on that node, from the EndpointSlices of the agent's Service,
``--probe-service``, default ``gpu-health/mi355x-node-agent``).  The shipped
agent listens on the pod network (``deploy/daemonset.yaml``: no
``hostNetwork``, no ``hostPort``), so ``{pod_ip}`` is the placeholder that
reaches it; ``{ip}`` suits agents run with ``hostNetwork``.  IPv6 addresses
are filled in bracketed (``[fd00::7]``), ready for the host part of a URL.
Each report stays keyed to the node it was fetched for (the reference keys its
verdict to the node it read, ``/root/reference/check-gpu-node.py:199-212``):
the endpoint's ``nodeName`` picks the address, and a node with no agent
endpoint is ``unknown`` ("no agent endpoint") rather than a fetch from
another host.

Every endpoint is untrusted input: a body is read up to ``MAX_BODY`` bytes (``Content-Length``, chunked or
read-to-close; one over the cap fails the node instead of filling the checker's memory), the whole request
runs under ``--probe-timeout``, ``https`` endpoints verify against ``--probe-ca`` (or the system CAs), and
the caller binds each report to the node it was fetched for (``checker.apply_health``: a report whose
``node`` is another node's is ``unknown``).
"""

from __future__ import annotations

import asyncio
import json
import time
from typing import Any, Dict, List, Optional, Sequence
from urllib.parse import urlsplit

from ..models.health import SCHEMA


# an 8-GPU level-2 report is ~25 KB as JSON, a 64-partition CPX one under 256 KB: 1 MiB is far above any
# real report and far below what would hurt the checker
MAX_BODY = 1 << 20


class BodyTooLarge(ValueError):
    pass


def _error_report(node: str, msg: str) -> Dict[str, Any]:
    return {"schema": SCHEMA, "node": node, "ts": time.time(), "error": msg, "gpus": []}


_SSL_CACHE: Dict[Any, Any] = {}


def _ssl_context(ca_file: Optional[str], client_cert: Optional[str] = None, client_key: Optional[str] = None) -> Any:
    """Client TLS for agent endpoints (one context per configuration for the whole fan-out): verified against
    ``ca_file`` or the system roots, presenting ``client_cert`` when the agents require one (their
    ``--tls-client-ca``)."""
    key = (ca_file, client_cert, client_key)
    ctx = _SSL_CACHE.get(key)
    if ctx is None:
        import ssl
        ctx = ssl.create_default_context(cafile=ca_file) if ca_file else ssl.create_default_context()
        if client_cert:
            ctx.load_cert_chain(client_cert, client_key or None)
        _SSL_CACHE[key] = ctx
    return ctx


class _GetProtocol(asyncio.Protocol):
    """One ``GET`` over one connection, parsed as the bytes arrive (no StreamReader, no per-read coroutine
    resumptions): the response body, or the error, lands in ``done``."""

    def __init__(self, request: bytes, cap: int, done: "asyncio.Future[bytes]"):
        self.request, self.cap, self.done = request, cap, done
        self.buf = bytearray()
        self.pos = 0                      # parse offset into buf (after the head: the body / chunk cursor)
        self.status = 0
        self.length: Optional[int] = None  # Content-Length
        self.chunked = False
        self.headed = False
        self.body = bytearray()           # decoded chunked payload
        self.transport: Any = None

    def connection_made(self, transport: Any) -> None:
        self.transport = transport
        transport.write(self.request)

    def _finish(self, body: Optional[bytes] = None, exc: Optional[BaseException] = None) -> None:
        if not self.done.done():
            if exc is not None:
                self.done.set_exception(exc)
            else:
                self.done.set_result(body if body is not None else b"")
        if self.transport is not None:
            self.transport.close()

    def _head(self) -> bool:
        end = self.buf.find(b"\r\n\r\n")
        if end < 0:
            if len(self.buf) > 65536:
                raise ValueError("response head exceeds 64 KiB")
            return False
        lines = bytes(self.buf[:end]).decode("latin-1").split("\r\n")
        status = lines[0].split(None, 2)
        if len(status) < 2 or not status[0].startswith("HTTP/") or not status[1].isdigit():
            raise ValueError(f"malformed status line {lines[0][:80]!r}")
        self.status = int(status[1])
        for line in lines[1:]:
            k, _, v = line.partition(":")
            k = k.strip().lower()
            if k == "transfer-encoding" and "chunked" in v.lower():
                self.chunked = True
            elif k == "content-length":
                if not v.strip().isdigit():
                    raise ValueError(f"malformed Content-Length {v.strip()[:40]!r}")
                self.length = int(v.strip())
        if not self.chunked and self.length is not None and self.length > self.cap:
            raise BodyTooLarge(f"body of {self.length} bytes exceeds {self.cap}")
        self.pos = end + 4
        self.headed = True
        return True

    def _chunks(self) -> Optional[bytes]:
        """Decode whole chunks from ``pos``; the payload once the last chunk and its trailer are in."""
        buf = self.buf
        while True:
            eol = buf.find(b"\r\n", self.pos)
            if eol < 0:
                return None
            line = bytes(buf[self.pos:eol])
            size = int(line.split(b";", 1)[0].strip() or b"x", 16)
            if size == 0:
                end = buf.find(b"\r\n\r\n", eol) if buf[eol + 2:eol + 4] != b"\r\n" else eol
                if end < 0:
                    return None  # trailer fields still arriving
                return bytes(self.body)
            if len(self.body) + size > self.cap:
                raise BodyTooLarge(f"body exceeds {self.cap} bytes")
            if len(buf) < eol + 2 + size + 2:
                return None
            if buf[eol + 2 + size:eol + 4 + size] != b"\r\n":
                raise ValueError("malformed chunk")
            self.body += buf[eol + 2:eol + 2 + size]
            self.pos = eol + 4 + size

    def data_received(self, data: bytes) -> None:
        if self.done.done():
            return
        self.buf += data
        try:
            if not self.headed and not self._head():
                return
            if self.chunked:
                body = self._chunks()
                if body is not None:
                    self._finish(body)
            elif self.length is not None:
                if len(self.buf) - self.pos >= self.length:
                    self._finish(bytes(self.buf[self.pos:self.pos + self.length]))
            elif len(self.buf) - self.pos > self.cap:
                raise BodyTooLarge(f"body exceeds {self.cap} bytes")
        except Exception as e:  # malformed or oversized: the node's fetch fails, nothing propagates
            self._finish(exc=e if isinstance(e, ValueError) else ValueError(f"malformed response: {e!r}"))

    def eof_received(self) -> Optional[bool]:
        if self.headed and not self.chunked and self.length is None:
            self._finish(bytes(self.buf[self.pos:]))  # read-to-close body
        else:
            self._finish(exc=asyncio.IncompleteReadError(bytes(self.buf), None))
        return None

    def connection_lost(self, exc: Optional[BaseException]) -> None:
        if not self.done.done():
            self.done.set_exception(exc or asyncio.IncompleteReadError(bytes(self.buf), None))


async def _http_get_json(url: str, timeout: float, ca_file: Optional[str] = None, max_body: int = MAX_BODY,
                         client_cert: Optional[str] = None, client_key: Optional[str] = None,
                         server_name: Optional[str] = None) -> Any:
    """GET ``url`` and parse its JSON body.  ``server_name``: verify an https peer's certificate against this
    name instead of the URL's host (agents reached by pod IP present the Service's name)."""
    parts = urlsplit(url)
    host = parts.hostname or "localhost"
    port = parts.port or (443 if parts.scheme == "https" else 80)
    ssl_ctx = _ssl_context(ca_file, client_cert, client_key) if parts.scheme == "https" else None
    path = (parts.path or "/") + (("?" + parts.query) if parts.query else "")
    loop = asyncio.get_running_loop()
    done: "asyncio.Future[bytes]" = loop.create_future()
    req = (f"GET {path} HTTP/1.1\r\nHost: {f'[{host}]' if ':' in host else host}:{port}\r\n"
           f"Accept: application/json\r\n"
           f"Connection: close\r\n\r\n").encode()
    proto = _GetProtocol(req, max_body, done)
    # the deadline cancels this task (what asyncio.timeout does from 3.11): no wrapper task per request
    task = asyncio.current_task()
    expired: List[bool] = []

    def expire() -> None:
        expired.append(True)
        if task is not None:
            task.cancel()
    timer = loop.call_later(timeout, expire)
    try:
        if ssl_ctx is not None and server_name:
            await loop.create_connection(lambda: proto, host, port, ssl=ssl_ctx, server_hostname=server_name)
        else:
            await loop.create_connection(lambda: proto, host, port, ssl=ssl_ctx)
        body = await done
    except asyncio.CancelledError:
        if expired:
            raise asyncio.TimeoutError() from None
        raise
    finally:
        timer.cancel()
        if proto.transport is not None:
            proto.transport.close()
    if proto.status != 200:
        raise RuntimeError(f"HTTP {proto.status}")
    # the agent-only per-test fields (per-XCD/CU maps, burn-in rows, wall time) go before the report is judged or
    # cached: a --watch-events checker keeps every node's report (ProbeCache), as it keeps parsed annotations
    from ..models.node import slim_report
    return slim_report(json.loads(body))


async def fetch_all(targets: Sequence[Dict[str, str]], concurrency: int = 64, timeout: float = 2.0,
                    retries: int = 1, ca_file: Optional[str] = None, client_cert: Optional[str] = None,
                    client_key: Optional[str] = None, server_name: Optional[str] = None) -> List[Dict[str, Any]]:
    sem = asyncio.Semaphore(max(1, concurrency))

    async def one(t: Dict[str, str]) -> Dict[str, Any]:
        if t.get("error"):
            return _error_report(t["name"], t["error"])
        async with sem:
            last = "unreachable"
            for attempt in range(retries + 1):
                try:
                    doc = await _http_get_json(t["url"], timeout, ca_file, client_cert=client_cert,
                                               client_key=client_key, server_name=server_name)
                    if not isinstance(doc, dict):
                        return _error_report(t["name"], "probe endpoint returned non-object JSON")
                    return doc
                except asyncio.TimeoutError:
                    last = f"timeout after {timeout:g}s"
                    break  # a slow agent will not get faster; don't double the wait
                except BodyTooLarge as e:
                    last = f"probe response too large: {e}"
                    break
                except (OSError, asyncio.IncompleteReadError, RuntimeError, ValueError) as e:
                    last = f"{type(e).__name__}: {e}"
                    if attempt < retries:
                        await asyncio.sleep(0.05 * (attempt + 1))
                except Exception as e:  # anything else one endpoint provokes fails that node, not the check
                    last = f"{type(e).__name__}: {e}"
                    break
            return _error_report(t["name"], last)

    return list(await asyncio.gather(*(one(t) for t in targets)))


def _url_host(addr: str) -> str:
    return f"[{addr}]" if ":" in addr and not addr.startswith("[") else addr


def agent_addresses(slices: Sequence[Dict[str, Any]]) -> Dict[str, str]:
    """``nodeName -> address`` of the agent pod on each node, from a Service's EndpointSlices.

    Per node the best endpoint wins: ready (``conditions.ready`` true, or absent, which Kubernetes reads as
    ready) before not ready, not terminating before terminating (a rolling update briefly has two agent
    pods on a node), then the lowest address for a stable choice.  Endpoints without ``nodeName`` or
    address are skipped."""
    best: Dict[str, Any] = {}
    for sl in slices:
        if not isinstance(sl, dict):
            continue
        eps = sl.get("endpoints")
        for ep in eps if isinstance(eps, list) else []:
            if not isinstance(ep, dict):
                continue
            node = ep.get("nodeName")
            raw = ep.get("addresses")
            addrs = [a for a in raw if isinstance(a, str) and a] if isinstance(raw, list) else []
            if not isinstance(node, str) or not node or not addrs:
                continue
            cond = ep.get("conditions") if isinstance(ep.get("conditions"), dict) else {}
            rank = (cond.get("ready") is False, cond.get("terminating") is True, addrs[0])
            if node not in best or rank < best[node][0]:
                best[node] = (rank, addrs[0])
    return {node: addr for node, (_, addr) in best.items()}


def template_fields(template: str) -> set:
    import string
    try:
        fields = {f for _, f, _, _ in string.Formatter().parse(template) if f is not None}
    except ValueError as e:
        raise ValueError(f"--probe-endpoint {template!r}: {e}") from None
    allowed = {"name", "ip", "pod_ip"}
    if not fields <= allowed:
        raise ValueError(f"--probe-endpoint {template!r}: only {{name}}, {{ip}} and {{pod_ip}} can be filled in, "
                         f"not {', '.join(sorted('{' + f + '}' for f in fields - allowed))}")
    return fields


def build_targets(scan: Any, template: str, pod_ips: Optional[Dict[str, str]] = None,
                  pod_ip_error: Optional[str] = None) -> List[Dict[str, str]]:
    """One ``{"name", "url"}`` per GPU node; a node the template cannot address carries an ``error``
    instead: ``{ip}`` with no InternalIP (the URL would name no host, and the client would fall back to
    localhost), ``{pod_ip}`` with no agent endpoint on the node, or with the EndpointSlices unreadable
    (``pod_ip_error``)."""
    fields = template_fields(template)
    out = []
    needs_ip = "ip" in fields
    needs_pod = "pod_ip" in fields
    pod_ips = pod_ips or {}
    for node, ex in zip(scan.gpu_nodes, scan.extras):
        name = node["name"] or ""
        ip = getattr(ex, "internal_ip", None) or ""
        if needs_ip and not ip:
            out.append({"name": name, "url": "", "error": "node has no InternalIP for the probe endpoint"})
            continue
        pod_ip = ""
        if needs_pod:
            if pod_ip_error:
                out.append({"name": name, "url": "", "error": f"agent endpoints unavailable: {pod_ip_error}"})
                continue
            pod_ip = pod_ips.get(name, "")
            if not pod_ip:
                out.append({"name": name, "url": "", "error": "no agent endpoint on this node"})
                continue
        out.append({"name": name, "url": template.format(name=name, ip=_url_host(ip), pod_ip=_url_host(pod_ip))})
    return out


def run_coroutine(coro: Any) -> Any:
    """``asyncio.run`` that also works when the caller already runs an event loop (a notebook, an async
    embedding): then the coroutine gets its own loop on a helper thread."""
    try:
        asyncio.get_running_loop()
    except RuntimeError:
        return asyncio.run(coro)
    import threading
    box: Dict[str, Any] = {}

    def target() -> None:
        try:
            box["value"] = asyncio.run(coro)
        except BaseException as e:  # re-raised in the caller's thread
            box["error"] = e
    t = threading.Thread(target=target, name="probe-fanout", daemon=True)
    t.start()
    t.join()
    if "error" in box:
        raise box["error"]
    return box["value"]


class ProbeCache:
    """Fan-out results kept for ``ttl`` seconds, for the event watcher (``--watch-events``), which re-evaluates the
    whole fleet on every batch of node events: the agents probe once a minute, so fetching every agent's report
    on every event only loads them (1000 nodes heartbeating every 5 minutes are ~3 events a second).  A report is
    reused per (node, URL) while younger than ``ttl``; a failed fetch is not kept (the next evaluation retries
    it).  The agents' EndpointSlices are kept the same way (``endpoints``)."""

    def __init__(self, ttl: float = 30.0):
        self.ttl = ttl
        self._reports: Dict[Any, Any] = {}
        self.endpoints: Optional[Any] = None  # (monotonic time, (addresses, error))
        self.fetched = 0
        self.reused = 0

    def get(self, target: Dict[str, str], now: float) -> Optional[Dict[str, Any]]:
        hit = self._reports.get((target["name"], target["url"]))
        if hit is not None and now - hit[0] < self.ttl:
            self.reused += 1
            return hit[1]
        return None

    def put(self, target: Dict[str, str], report: Any, now: float) -> None:
        self.fetched += 1
        if isinstance(report, dict) and not report.get("error"):
            self._reports[(target["name"], target["url"])] = (now, report)

    def prune(self, now: float) -> None:
        """Forget reports well past the TTL: a rescheduled agent pod has a new address, so its old entry would
        otherwise stay for the life of the watcher."""
        old = [k for k, (t, _) in self._reports.items() if now - t >= 4 * self.ttl]
        for k in old:
            del self._reports[k]

    def fresh_endpoints(self, now: float) -> Optional[Any]:
        e = self.endpoints
        return e[1] if e is not None and now - e[0] < self.ttl and e[1][1] is None else None


def fetch_probe_reports(scan: Any, template: str, concurrency: int = 64, timeout: float = 2.0,
                        ca_file: Optional[str] = None, client_cert: Optional[str] = None,
                        client_key: Optional[str] = None, pod_ips: Optional[Dict[str, str]] = None,
                        pod_ip_error: Optional[str] = None,
                        server_name: Optional[str] = None,
                        cache: Optional[ProbeCache] = None) -> List[Optional[Dict[str, Any]]]:
    """Fetch one probe report per GPU node (parallel to ``scan.gpu_nodes``); with a ``cache``, reports it holds
    fresh are reused and only the rest are fetched."""
    import time
    targets = build_targets(scan, template, pod_ips, pod_ip_error)
    if not targets:
        return []
    now = time.monotonic()
    if cache is not None:
        cache.prune(now)
    out: List[Optional[Dict[str, Any]]] = [None] * len(targets)
    todo = []
    for i, t in enumerate(targets):
        hit = cache.get(t, now) if cache is not None and not t.get("error") else None
        if hit is not None:
            out[i] = hit
        else:
            todo.append(i)
    if todo:
        got = run_coroutine(fetch_all([targets[i] for i in todo], concurrency, timeout, ca_file=ca_file,
                                      client_cert=client_cert, client_key=client_key, server_name=server_name))
        for i, rep in zip(todo, got):
            out[i] = rep
            if cache is not None and not targets[i].get("error"):
                cache.put(targets[i], rep, now)
    return out
