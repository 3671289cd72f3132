"""``check-gpu-node --explain NODE``: why a GPU node counts (or does not count) as Ready.

One node, in the checker's own terms: the reference's Ready rule (``check-gpu-node.py:172-178``), the
GPU count it sees (``:181-196``), then the MI355X gate -- the agent's ``AMDGPUHealthy`` condition, the
full report annotation re-judged with the checker's thresholds, and one row per GPU with the fields
the verdict rests on.  Exit code: 0 the node counts as Ready, 3 it does not, 2 no such GPU node,
1 an error (the reference's codes, applied to one node).
"""

from __future__ import annotations

import time
from typing import Any, Dict, List, Optional, TextIO

from .checker import CheckOptions, apply_health, apply_schedulability, scan_cluster
from .kube.config import ClusterConnection
from .models import health as H
from .models.node import HEALTH_CONDITION
from .utils.timing import NullTracer


def _age(seconds: Optional[float]) -> str:
    if seconds is None:
        return "?"
    if seconds < 120:
        return f"{seconds:.0f} s"
    if seconds < 7200:
        return f"{seconds / 60:.0f} min"
    return f"{seconds / 3600:.1f} h"


def _gpu_row(g: Dict[str, Any], verdict_lines: List[str]) -> List[str]:
    idx = g.get("index", "?")
    diag = g.get("diag") if isinstance(g.get("diag"), dict) else {}
    bad_diag = sorted(t for t, r in diag.items() if isinstance(r, dict) and r.get("pass") is False)
    slow_diag = sorted(t for t, r in diag.items() if isinstance(r, dict) and r.get("degraded"))
    dstate = ("fail: " + ",".join(bad_diag)) if bad_diag else ("slow: " + ",".join(slow_diag)) if slow_diag else \
        ("pass" if diag else "-")
    fw = g.get("fw") if isinstance(g.get("fw"), dict) else {}
    mine = [ln for ln in verdict_lines if ln.startswith(f"gpu{idx}:")]
    return [str(idx), str(g.get("bdf", "")), str(g.get("gfx", "")), str(g.get("cus", "")),
            f"{g.get('vram_mb', '')}", f"{g.get('ecc_uncorrectable', '-')}/{g.get('ecc_correctable', '-')}",
            str(g.get("xgmi", "")), H.fw_version_str("pm", fw["pm"]) if "pm" in fw else "-", dstate,
            "ok" if not mine else "; ".join(m.split(": ", 1)[1] for m in mine)]


def explain(cluster: ClusterConnection, node_name: str, opts: CheckOptions, out: TextIO) -> int:
    opts.json_extended = True  # the full report annotation is read (annotation mode 2)
    scan = scan_cluster(cluster, opts, NullTracer())
    names = [n["name"] for n in scan.gpu_nodes]
    if node_name not in names:
        out.write(f"{node_name}: not a GPU node in this cluster (no {', '.join(opts_keys())} capacity)\n"
                  if scan.items_seen else f"{node_name}: no nodes listed\n")
        return 2
    i = names.index(node_name)
    node, ex = scan.gpu_nodes[i], scan.extras[i]
    ready_cond = ex.ready_condition
    verdicts = apply_health(scan, opts, NullTracer(), [])
    apply_schedulability(scan, opts)
    v = verdicts[i] if i < len(verdicts) else None
    breakdown = ", ".join(f"{k}:{c}" for k, c in node["gpu_breakdown"].items())
    out.write(f"node {node_name}: Ready={ready_cond}  GPUs {node['gpus']} ({breakdown})"
              f"  allocatable {ex.allocatable or '-'}{'  cordoned' if ex.unschedulable else ''}\n")
    now = time.time()
    if ex.health_condition is not None:
        status, reason, message, hb = ex.health_condition
        out.write(f"{HEALTH_CONDITION}={status} ({reason}, heartbeat {_age(now - hb if hb else None)} ago): "
                  f"{message}\n")
    else:
        out.write(f"{HEALTH_CONDITION}: not published (no node agent)\n")
    if v is None:
        out.write(f"MI355X verdict: none (policy {opts.health_policy}: the reference's Ready rule applies)\n")
    else:
        out.write(f"MI355X verdict: {v.state}, {v.gpus_ok}/{v.gpus_seen} GPUs ok"
                  + (f", report {_age(v.age_s)} old" if v.age_s is not None else "") + "\n")
        for title, items in (("reasons", v.reasons), ("warnings", v.warnings)):
            for r in items:
                out.write(f"  {title[:-1]}: {r}\n")
    rep = H.parse_annotation(ex.health_annotation)
    if rep and not rep.get("error"):
        drv = rep.get("driver") if isinstance(rep.get("driver"), dict) else {}
        out.write(f"report: probe {rep.get('probe', '?')}, amd-smi {rep.get('amdsmi', '?')}, driver "
                  f"{H.driver_release(drv.get('version')) or '?'}, {len(rep.get('gpus') or [])} GPUs\n")
        re_v = H.evaluate_report(rep, max(ex.capacity.get("amd.com/gpu", 0), ex.allocatable.get("amd.com/gpu", 0)),
                                 H.HealthExpectations(xgmi_links=opts.xgmi_links, max_age_s=opts.probe_max_age), now)
        lines = re_v.reasons + re_v.warnings
        head = ["GPU", "BDF", "gfx", "CUs", "VRAM MB", "ECC ue/ce", "xGMI", "PM fw", "diag", "findings"]
        rows = [head] + [_gpu_row(g, lines) for g in rep.get("gpus") or [] if isinstance(g, dict)]
        widths = [max(len(r[c]) for r in rows) for c in range(len(head) - 1)]
        for r in rows:
            out.write("  " + "  ".join(r[c].ljust(widths[c]) for c in range(len(head) - 1)) + "  " + r[-1] + "\n")
        shown = {f"gpu{g.get('index')}:" for g in rep.get("gpus") or [] if isinstance(g, dict)}
        node_level = [ln for ln in lines if ln.split(" ", 1)[0] not in shown]  # incl. spans ("gpu6-7: ...")
        for ln in node_level:
            out.write(f"  node: {ln}\n")
    elif rep and rep.get("error"):
        out.write(f"report: unreadable ({rep['error']})\n")
    counts = node["ready"]
    out.write(f"=> counts as Ready: {'yes' if counts else 'no'}\n")
    return 0 if counts else 3


def opts_keys() -> List[str]:
    from .models.resources import GPU_RESOURCE_KEYS
    return list(GPU_RESOURCE_KEYS)
