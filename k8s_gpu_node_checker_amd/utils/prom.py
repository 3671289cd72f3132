"""Prometheus node-exporter textfile output (SURVEY §5 "Metrics": the reference has bare prints only).

Written atomically (temp file + ``rename``) so the textfile collector never
reads a half-written file.  No ``prometheus_client`` import: the exposition
format is a few lines of text.
"""

from __future__ import annotations

import os
import tempfile
import time
from typing import Any, List


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
