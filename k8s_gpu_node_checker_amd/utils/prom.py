"""Prometheus metrics of the checker (SURVEY §5 "Metrics": the reference has bare prints only).

Two outputs of the same exposition text (:func:`render`):

* a node-exporter textfile (``--prometheus-textfile``), written atomically (temp file + ``rename``) so the
  textfile collector never reads a half-written file -- for the CronJob, whose pod is gone between runs;
* an HTTP ``/metrics`` endpoint (``--metrics-listen``, :class:`MetricsServer`) for the long-running event
  watcher (``--watch-events``, ``deploy/watcher.yaml``), scraped through its Service by a ServiceMonitor
  (``deploy/monitoring/monitoring.yaml``).  With ``--leader-elect`` every replica serves
  ``k8s_gpu_checker_leader`` (1 on the holder) and only the holder the cluster's gauges.

No ``prometheus_client`` import: the exposition format is a few lines of text.
"""

from __future__ import annotations

import os
import tempfile
import time
from typing import Any, List

from .http import nodelay


def _esc(v: Any) -> str:
    return str(v).replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def _write(path: str, lines: List[str]) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".k8sgpu-", suffix=".prom", dir=d)
    with os.fdopen(fd, "w", encoding="utf-8") as f:
        f.write("\n".join(lines) + "\n")
    os.chmod(tmp, 0o644)
    os.replace(tmp, path)


def render(result: Any) -> List[str]:
    now = time.time()
    lines = [
        "# HELP k8s_gpu_checker_gpu_nodes GPU nodes seen in the cluster.",
        "# TYPE k8s_gpu_checker_gpu_nodes gauge",
        f"k8s_gpu_checker_gpu_nodes {len(result.gpu_nodes)}",
        "# HELP k8s_gpu_checker_ready_gpu_nodes GPU nodes that are Ready (and MI355X-healthy when gated).",
        "# TYPE k8s_gpu_checker_ready_gpu_nodes gauge",
        f"k8s_gpu_checker_ready_gpu_nodes {len(result.ready_gpu_nodes)}",
        "# HELP k8s_gpu_checker_exit_code Exit code of the last check (0 ok, 1 error, 2 no GPU, 3 none ready).",
        "# TYPE k8s_gpu_checker_exit_code gauge",
        f"k8s_gpu_checker_exit_code {result.exit_code}",
        "# HELP k8s_gpu_checker_last_run_timestamp_seconds Unix time of the last check.",
        "# TYPE k8s_gpu_checker_last_run_timestamp_seconds gauge",
        f"k8s_gpu_checker_last_run_timestamp_seconds {now:.3f}",
        "# HELP k8s_gpu_checker_node_ready Per-node Ready verdict.",
        "# TYPE k8s_gpu_checker_node_ready gauge",
    ]
    for n in result.gpu_nodes:
        lines.append(f'k8s_gpu_checker_node_ready{{node="{_esc(n["name"])}"}} {1 if n["ready"] else 0}')
    lines += ["# HELP k8s_gpu_checker_node_gpus Per-node GPU count by resource key.",
              "# TYPE k8s_gpu_checker_node_gpus gauge"]
    for n in result.gpu_nodes:
        for k, v in n["gpu_breakdown"].items():
            lines.append(f'k8s_gpu_checker_node_gpus{{node="{_esc(n["name"])}",resource="{_esc(k)}"}} {v}')
    if result.verdicts:
        lines += ["# HELP k8s_gpu_checker_mi355x_health MI355X probe verdict (1 for the current state).",
                  "# TYPE k8s_gpu_checker_mi355x_health gauge"]
        for n, v in zip(result.gpu_nodes, result.verdicts):
            if v is not None:
                lines.append(f'k8s_gpu_checker_mi355x_health{{node="{_esc(n["name"])}",state="{v.state}"}} 1')
    fleet = getattr(result, "fleet_diag", None)
    if fleet:
        # models/fleet.py: per test, the fleet's median node as a fraction of the MI355X reference, and how many
        # nodes fall under 85 % of the others
        lines += ["# HELP k8s_gpu_checker_diag_fleet_median_fraction The median node's diagnostic rate as a "
                  "fraction of the MI355X reference, per test.",
                  "# TYPE k8s_gpu_checker_diag_fleet_median_fraction gauge"]
        lines += [f'k8s_gpu_checker_diag_fleet_median_fraction{{test="{_esc(t)}"}} {row["median_fraction"]}'
                  for t, row in fleet.items() if row.get("unit", "fraction") == "fraction"]
        lines += ["# HELP k8s_gpu_checker_diag_fleet_outlier_nodes Nodes under 85 % of the other nodes' median, per "
                  "test.",
                  "# TYPE k8s_gpu_checker_diag_fleet_outlier_nodes gauge"]
        lines += [f'k8s_gpu_checker_diag_fleet_outlier_nodes{{test="{_esc(t)}"}} {len(row["outliers"])}'
                  for t, row in fleet.items()]
    spans = result.tracer.as_ms() if result.tracer is not None else {}
    if spans:
        lines += ["# HELP k8s_gpu_checker_phase_seconds Wall time per check phase.",
                  "# TYPE k8s_gpu_checker_phase_seconds gauge"]
        for k, ms in spans.items():
            lines.append(f'k8s_gpu_checker_phase_seconds{{phase="{_esc(k)}"}} {ms / 1e3:.6f}')
    return lines


def write_textfile(path: str, result: Any) -> None:
    _write(path, render(result))


def write_error_textfile(path: str, message: str) -> None:
    _write(path, [
        "# HELP k8s_gpu_checker_exit_code Exit code of the last check (0 ok, 1 error, 2 no GPU, 3 none ready).",
        "# TYPE k8s_gpu_checker_exit_code gauge",
        "k8s_gpu_checker_exit_code 1",
        "# HELP k8s_gpu_checker_error Last check failed before a report was produced.",
        "# TYPE k8s_gpu_checker_error gauge",
        f'k8s_gpu_checker_error{{message="{_esc(message[:200])}"}} 1',
        f"k8s_gpu_checker_last_run_timestamp_seconds {time.time():.3f}",
    ])


LEADER_HELP = ["# HELP k8s_gpu_checker_leader 1 on the watcher replica that holds the leader Lease (it reports).",
               "# TYPE k8s_gpu_checker_leader gauge"]


class MetricsServer:
    """``GET /metrics`` (the last rendered report, plus the leader gauge) and ``GET /healthz`` on a thread.

    ``update(result)`` swaps in a new report's lines; ``set_leader(bool)`` the replica's role.  Before the first
    report (or on a follower) only the leader gauge is served, so a scrape never shows a stale cluster."""

    def __init__(self, host: str, port: int):
        import threading
        from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
        self._lock = threading.Lock()
        self._lines: List[str] = []
        self._leader: Any = None
        outer = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"
            timeout = 30

            def log_message(self, *a: Any) -> None:
                pass

            def setup(self) -> None:
                super().setup()
                nodelay(self.connection)

            def do_GET(self) -> None:  # noqa: N802
                if self.path.split("?")[0] == "/metrics":
                    body, ctype, code = outer.text().encode(), "text/plain; version=0.0.4; charset=utf-8", 200
                elif self.path.split("?")[0] == "/healthz":
                    body, ctype, code = b"ok\n", "text/plain", 200
                else:
                    body, ctype, code = b"not found\n", "text/plain", 404
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        server_cls = ThreadingHTTPServer
        if ":" in host:  # an IPv6 address ("::" for every interface)
            import socket

            class V6(ThreadingHTTPServer):
                address_family = socket.AF_INET6
            server_cls = V6
        self.httpd = server_cls((host, port), Handler)
        self.httpd.daemon_threads = True
        self._thread = threading.Thread(target=self.httpd.serve_forever, kwargs={"poll_interval": 0.2},
                                        name="metrics", daemon=True)

    @property
    def port(self) -> int:
        return self.httpd.server_address[1]

    def start(self) -> "MetricsServer":
        self._thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()

    def update(self, result: Any) -> None:
        lines = render(result)
        with self._lock:
            self._lines = lines

    def set_leader(self, leading: bool) -> None:
        with self._lock:
            self._leader = bool(leading)
            if not leading:
                self._lines = []  # a follower serves no cluster gauges (the leader does)

    def text(self) -> str:
        with self._lock:
            lines = list(self._lines)
            if self._leader is not None:
                lines += LEADER_HELP + [f"k8s_gpu_checker_leader {1 if self._leader else 0}"]
        return "\n".join(lines) + "\n" if lines else "\n"


def parse_listen(spec: str) -> "tuple[str, int]":
    """``HOST:PORT`` / ``:PORT`` / ``[v6]:PORT`` -> (host, port); host defaults to all interfaces."""
    host, sep, port = spec.rpartition(":")
    if not sep or not port.isdigit():
        raise ValueError(f"--metrics-listen {spec!r}: expected HOST:PORT")
    return (host.strip("[]") or "0.0.0.0"), int(port)
