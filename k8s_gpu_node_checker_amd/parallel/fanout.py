"""Async per-node probe fan-out (SURVEY §7.2 layer 5 source (b), §6 takeaway 3).

When node agents serve their report over HTTP instead of (or besides) the
annotation, the checker fetches every GPU node's ``/probe`` concurrently:
``asyncio`` streams (no aiohttp: 310 ms import), an ``asyncio.Semaphore``
bounding in-flight requests, a per-node timeout and one retry on connection
errors.  Wall clock is ~max(node latency) instead of the sum, so it stays flat
as the cluster grows.

URL template placeholders: ``{name}`` (node name) and ``{ip}`` (the node's
``InternalIP`` from ``status.addresses``).

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


async def _read_capped(reader: asyncio.StreamReader, n: Optional[int], cap: int) -> bytes:
    """``n`` bytes (Content-Length) or everything to EOF (``n`` None), refusing more than ``cap``."""
    if n is not None:
        if n > cap:
            raise BodyTooLarge(f"body of {n} bytes exceeds {cap}")
        return await reader.readexactly(n)
    buf = bytearray()
    while True:
        chunk = await reader.read(65536)
        if not chunk:
            return bytes(buf)
        buf += chunk
        if len(buf) > cap:
            raise BodyTooLarge(f"body exceeds {cap} bytes")


async def _read_chunked(reader: asyncio.StreamReader, cap: int) -> bytes:
    """A ``Transfer-Encoding: chunked`` body (RFC 9112 section 7.1), at most ``cap`` bytes of payload."""
    buf = bytearray()
    while True:
        line = await reader.readuntil(b"\r\n")
        size = int(line.split(b";", 1)[0].strip() or b"x", 16)
        if size == 0:
            while (await reader.readuntil(b"\r\n")) != b"\r\n":  # trailer fields
                pass
            return bytes(buf)
        if len(buf) + size > cap:
            raise BodyTooLarge(f"body exceeds {cap} bytes")
        buf += await reader.readexactly(size)
        if await reader.readexactly(2) != b"\r\n":
            raise ValueError("malformed chunk")


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


async def _http_get_json(url: str, timeout: float, ca_file: Optional[str] = None, max_body: int = MAX_BODY,
                         client_cert: Optional[str] = None, client_key: Optional[str] = None) -> Any:
    parts = urlsplit(url)
    host = parts.hostname or "localhost"
    port = parts.port or (443 if parts.scheme == "https" else 80)
    ssl_ctx = _ssl_context(ca_file, client_cert, client_key) if parts.scheme == "https" else None
    path = (parts.path or "/") + (("?" + parts.query) if parts.query else "")

    async def run() -> Any:
        reader, writer = await asyncio.open_connection(host, port, ssl=ssl_ctx)
        try:
            writer.write(f"GET {path} HTTP/1.1\r\nHost: {host}:{port}\r\nAccept: application/json\r\n"
                         f"Connection: close\r\n\r\n".encode())
            await writer.drain()
            head = await reader.readuntil(b"\r\n\r\n")
            lines = head.decode("latin-1").split("\r\n")
            status = int(lines[0].split()[1])
            headers = {}
            for line in lines[1:]:
                k, _, v = line.partition(":")
                headers[k.strip().lower()] = v.strip()
            if "chunked" in headers.get("transfer-encoding", "").lower():
                body = await _read_chunked(reader, max_body)
            elif "content-length" in headers:
                body = await _read_capped(reader, int(headers["content-length"]), max_body)
            else:
                body = await _read_capped(reader, None, max_body)
            if status != 200:
                raise RuntimeError(f"HTTP {status}")
            return json.loads(body)
        finally:
            writer.close()

    return await asyncio.wait_for(run(), timeout)


async def fetch_all(targets: Sequence[Dict[str, str]], concurrency: int = 64, timeout: float = 2.0,
                    retries: int = 1, ca_file: Optional[str] = None, client_cert: Optional[str] = None,
                    client_key: Optional[str] = None) -> List[Dict[str, Any]]:
    sem = asyncio.Semaphore(max(1, concurrency))

    async def one(t: Dict[str, str]) -> Dict[str, Any]:
        async with sem:
            last = "unreachable"
            for attempt in range(retries + 1):
                try:
                    doc = await _http_get_json(t["url"], timeout, ca_file, client_cert=client_cert,
                                               client_key=client_key)
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
            return _error_report(t["name"], last)

    return list(await asyncio.gather(*(one(t) for t in targets)))


def build_targets(scan: Any, template: str) -> List[Dict[str, str]]:
    out = []
    for node, ex in zip(scan.gpu_nodes, scan.extras):
        ip = getattr(ex, "internal_ip", None) or ""
        out.append({"name": node["name"] or "", "url": template.format(name=node["name"] or "", ip=ip)})
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


def fetch_probe_reports(scan: Any, template: str, concurrency: int = 64, timeout: float = 2.0,
                        ca_file: Optional[str] = None, client_cert: Optional[str] = None,
                        client_key: Optional[str] = None) -> List[Optional[Dict[str, Any]]]:
    """Fetch one probe report per GPU node (parallel to ``scan.gpu_nodes``)."""
    targets = build_targets(scan, template)
    if not targets:
        return []
    return list(run_coroutine(fetch_all(targets, concurrency, timeout, ca_file=ca_file, client_cert=client_cert,
                                        client_key=client_key)))
