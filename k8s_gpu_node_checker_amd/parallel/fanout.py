"""Async per-node probe fan-out (SURVEY §7.2 layer 5 source (b), §6 takeaway 3).

When node agents serve their report over HTTP instead of (or besides) the
annotation, the checker fetches every GPU node's ``/probe`` concurrently:
``asyncio`` streams (no aiohttp: 310 ms import), an ``asyncio.Semaphore``
bounding in-flight requests, a per-node timeout and one retry on connection
errors.  Wall clock is ~max(node latency) instead of the sum, so it stays flat
as the cluster grows.

URL template placeholders: ``{name}`` (node name) and ``{ip}`` (the node's
``InternalIP`` from ``status.addresses``).
"""

from __future__ import annotations

import asyncio
import json
import time
from typing import Any, Dict, List, Optional, Sequence
from urllib.parse import urlsplit

from ..models.health import SCHEMA


def _error_report(node: str, msg: str) -> Dict[str, Any]:
    return {"schema": SCHEMA, "node": node, "ts": time.time(), "error": msg, "gpus": []}


async def _http_get_json(url: str, timeout: float) -> Any:
    parts = urlsplit(url)
    host = parts.hostname or "localhost"
    port = parts.port or (443 if parts.scheme == "https" else 80)
    ssl_ctx = None
    if parts.scheme == "https":
        import ssl
        ssl_ctx = ssl.create_default_context()
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
            if "content-length" in headers:
                body = await reader.readexactly(int(headers["content-length"]))
            else:
                body = await reader.read()
            if status != 200:
                raise RuntimeError(f"HTTP {status}")
            return json.loads(body)
        finally:
            writer.close()

    return await asyncio.wait_for(run(), timeout)


async def fetch_all(targets: Sequence[Dict[str, str]], concurrency: int = 64, timeout: float = 2.0,
                    retries: int = 1) -> List[Dict[str, Any]]:
    sem = asyncio.Semaphore(max(1, concurrency))

    async def one(t: Dict[str, str]) -> Dict[str, Any]:
        async with sem:
            last = "unreachable"
            for attempt in range(retries + 1):
                try:
                    doc = await _http_get_json(t["url"], timeout)
                    if not isinstance(doc, dict):
                        return _error_report(t["name"], "probe endpoint returned non-object JSON")
                    return doc
                except asyncio.TimeoutError:
                    last = f"timeout after {timeout:g}s"
                    break  # a slow agent will not get faster; don't double the wait
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


def fetch_probe_reports(scan: Any, template: str, concurrency: int = 64,
                        timeout: float = 2.0) -> List[Optional[Dict[str, Any]]]:
    """Fetch one probe report per GPU node (parallel to ``scan.gpu_nodes``)."""
    targets = build_targets(scan, template)
    if not targets:
        return []
    return list(asyncio.run(fetch_all(targets, concurrency, timeout)))
