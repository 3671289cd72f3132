"""``check-gpu-node --explain NODE``: why a GPU node counts (or does not count) as Ready.

One node, in the checker's own terms: the reference's Ready rule (``check-gpu-node.py:172-178``), the
GPU count it sees (``:181-196``), then the MI355X gate -- the agent's ``AMDGPUHealthy`` condition, the
full report annotation re-judged with the checker's thresholds, and one row per GPU with the fields
the verdict rests on.  Exit code: 0 the node counts as Ready, 3 it does not, 2 no such GPU node,
1 an error (the reference's codes, applied to one node).
"""

from __future__ import annotations

import json
import time
from typing import Any, Dict, List, Optional, TextIO

from .checker import CheckOptions, apply_health, apply_schedulability, fleet_versions, run_check, scan_cluster
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


_COLUMNS = ("GPU", "BDF", "gfx", "CUs", "VRAM MB", "ECC ue/ce", "xGMI", "PM fw", "diag", "vs peers", "vs own",
            "findings")


def _min_ratio(diag: Dict[str, Any], key: str) -> Any:
    """The lowest rate ratio of a GPU's diagnostics against its node's other GPUs (``peers``) or its own
    baseline (``baseline``), None when no test was judged that way."""
    vals = [v for r in diag.values() if isinstance(r, dict) and isinstance(r.get(key), dict)
            for v in ((r[key].get("ratio") or {}) if isinstance(r[key].get("ratio"), dict) else {}).values()
            if isinstance(v, (int, float)) and not isinstance(v, bool)]
    return round(min(vals), 3) if vals else None


def _gpu_entry(g: Dict[str, Any], verdict_lines: List[str]) -> Dict[str, Any]:
    """One GPU of the report, reduced to the fields its verdict rests on, with its findings."""
    idx = g.get("index", "?")
    diag = g.get("diag") if isinstance(g.get("diag"), dict) else {}
    fw = g.get("fw") if isinstance(g.get("fw"), dict) else {}
    return {"index": idx, "bdf": g.get("bdf"), "gfx": g.get("gfx"), "cus": g.get("cus"), "vram_mb": g.get("vram_mb"),
            "ecc_uncorrectable": g.get("ecc_uncorrectable"), "ecc_correctable": g.get("ecc_correctable"),
            "xgmi": g.get("xgmi"), "pm_fw": H.fw_version_str("pm", fw["pm"]) if "pm" in fw else None,
            "diag_failed": sorted(t for t, r in diag.items() if isinstance(r, dict) and r.get("pass") is False),
            "diag_slow": sorted(t for t, r in diag.items() if isinstance(r, dict) and r.get("degraded")),
            "diag_ran": bool(diag),
            "peer_ratio_min": _min_ratio(diag, "peers"), "baseline_ratio_min": _min_ratio(diag, "baseline"),
            "findings": [ln.split(": ", 1)[1] for ln in verdict_lines if ln.startswith(f"gpu{idx}:")]}


def _gpu_row(e: Dict[str, Any]) -> List[str]:
    def txt(v: Any, none: str = "") -> str:
        return none if v is None else str(v)
    dstate = ("fail: " + ",".join(e["diag_failed"])) if e["diag_failed"] else \
        ("slow: " + ",".join(e["diag_slow"])) if e["diag_slow"] else ("pass" if e["diag_ran"] else "-")
    return [txt(e["index"]), txt(e["bdf"]), txt(e["gfx"]), txt(e["cus"]), txt(e["vram_mb"]),
            f"{txt(e['ecc_uncorrectable'], '-')}/{txt(e['ecc_correctable'], '-')}", txt(e["xgmi"]),
            txt(e["pm_fw"], "-"), dstate,
            f"x{e['peer_ratio_min']:.2f}" if isinstance(e.get("peer_ratio_min"), (int, float)) else "-",
            f"x{e['baseline_ratio_min']:.2f}" if isinstance(e.get("baseline_ratio_min"), (int, float)) else "-",
            "; ".join(e["findings"]) or "ok"]


def gpu_table(entries: List[Dict[str, Any]]) -> List[str]:
    """The per-GPU table (one line per :func:`_gpu_entry`, header first), as ``--explain`` and the agent's
    ``/status`` print it."""
    rows = [list(_COLUMNS)] + [_gpu_row(e) for e in entries]
    widths = [max(len(r[c]) for r in rows) for c in range(len(_COLUMNS) - 1)]
    return ["  ".join(r[c].ljust(widths[c]) for c in range(len(_COLUMNS) - 1)) + "  " + r[-1] for r in rows]


def report_text(rep: Dict[str, Any], verdict: Any) -> str:
    """One report and its verdict as text (the agent's ``/status``): verdict, reasons and warnings, the
    per-GPU table, node-level findings, GPUs whose diagnostics were skipped and why."""
    drv = rep.get("driver") if isinstance(rep.get("driver"), dict) else {}
    lines = [f"node {rep.get('node', '?')}: MI355X verdict {verdict.state}, {verdict.gpus_ok}/{verdict.gpus_seen} GPUs "
             f"ok (probe {rep.get('probe', '?')}, amd-smi {rep.get('amdsmi', '?')}, driver "
             f"{H.driver_release(drv.get('version')) if drv.get('version') else '?'})"]
    if rep.get("error"):
        lines.append(f"  probe error: {rep['error']}")
    for title in ("reasons", "warnings"):
        for r in getattr(verdict, title):
            lines.append(f"  {title[:-1]}: {r}")
    found = verdict.reasons + verdict.warnings
    entries = [_gpu_entry(g, found) for g in H.report_gpus(rep) if isinstance(g, dict)]
    if entries:
        lines += ["  " + ln for ln in gpu_table(entries)]
    for g in H.report_gpus(rep):
        if isinstance(g, dict) and g.get("diag_skipped"):
            lines.append(f"  gpu{g.get('index', '?')} diagnostics skipped: {g['diag_skipped']}")
    return "\n".join(lines) + "\n"


def diagnose(cluster: ClusterConnection, node_name: str, opts: CheckOptions) -> Dict[str, Any]:
    """Everything ``--explain`` says about one node, as data (``--explain NODE --json`` prints it)."""
    opts.json_extended = True  # the full report annotation is read (annotation mode 2)
    scan = scan_cluster(cluster, opts, NullTracer())
    names = [n["name"] for n in scan.gpu_nodes]
    if node_name not in names:
        return {"node": node_name, "gpu_node": False, "nodes_listed": scan.items_seen}
    i = names.index(node_name)
    node, ex = scan.gpu_nodes[i], scan.extras[i]
    fleet: Dict[str, Any] = {}
    verdicts = apply_health(scan, opts, NullTracer(), [], cluster, fleet)
    view = (fleet.get("views") or [None] * len(names))[i]
    apply_schedulability(scan, opts)
    v = verdicts[i] if i < len(verdicts) else None
    now = time.time()
    doc: Dict[str, Any] = {"node": node_name, "gpu_node": True, "ready_condition": ex.ready_condition,
                           "gpus": node["gpus"], "gpu_breakdown": node["gpu_breakdown"],
                           "allocatable": ex.allocatable, "unschedulable": ex.unschedulable,
                           "health_policy": opts.health_policy, "health_condition": None,
                           "amd_labels": {k: v for k, v in sorted((node.get("labels") or {}).items())
                                          if k.startswith("amd.com/")},
                           "verdict": v.to_dict() if v is not None else None, "report": None}
    if ex.health_condition is not None:
        status, reason, message, hb = ex.health_condition
        doc["health_condition"] = {"status": status, "reason": reason, "message": message,
                                   "heartbeat_age_s": round(now - hb, 1) if hb else None}
    rep = ex.report()
    if rep and not isinstance(rep, dict):
        rep = {"error": f"malformed report (a JSON {type(rep).__name__}, not an object)"}
    if rep and rep.get("error"):
        doc["report"] = {"error": rep["error"]}
    elif rep:
        drv = rep.get("driver") if isinstance(rep.get("driver"), dict) else {}
        re_v = H.evaluate_report(rep, max(ex.capacity.get("amd.com/gpu", 0), ex.allocatable.get("amd.com/gpu", 0)),
                                 H.HealthExpectations(xgmi_links=opts.xgmi_links, max_age_s=opts.probe_max_age), now,
                                 view)
        lines = re_v.reasons + re_v.warnings
        gpus = [_gpu_entry(g, lines) for g in H.report_gpus(rep) if isinstance(g, dict)]
        shown = {f"gpu{e['index']}:" for e in gpus}
        doc["report"] = {"probe": rep.get("probe"), "amdsmi": rep.get("amdsmi"),
                         "driver": H.driver_release(drv.get("version")) if drv.get("version") else None,
                         "gpus": gpus,
                         # findings not about one GPU of the table, incl. spans ("... gpu0-2,4-7 ...")
                         "node_findings": [ln for ln in lines if ln.split(" ", 1)[0] not in shown]}
    if fleet.get("summary"):
        # this node's place in the fleet (models/fleet.py): per test, the fleet's median and this node's ratio to it
        from .models.fleet import explained_text, summary_key
        mine = {summary_key(k): v for k, v in ex.fleet_fractions().items()}
        ratios = {k: round(mine[k] / row["median_fraction"], 3) for k, row in fleet["summary"].items()
                  if k in mine and row.get("median_fraction")}
        doc["fleet_diag"] = {"summary": fleet["summary"], "explained": explained_text(view) if view else [],
                             "node_ratio": ratios}
    doc["counts_as_ready"] = bool(node["ready"])
    return doc


def render(doc: Dict[str, Any], out: TextIO) -> None:
    name = doc["node"]
    if not doc["gpu_node"]:
        out.write(f"{name}: not a GPU node in this cluster (no {', '.join(opts_keys())} capacity)\n"
                  if doc["nodes_listed"] else f"{name}: no nodes listed\n")
        return
    breakdown = ", ".join(f"{k}:{c}" for k, c in doc["gpu_breakdown"].items())
    out.write(f"node {name}: Ready={doc['ready_condition']}  GPUs {doc['gpus']} ({breakdown})"
              f"  allocatable {doc['allocatable'] or '-'}{'  cordoned' if doc['unschedulable'] else ''}\n")
    if doc.get("amd_labels"):
        out.write("labels: " + ", ".join(f"{k}={v}" for k, v in doc["amd_labels"].items()) + "\n")
    hc = doc["health_condition"]
    if hc is not None:
        out.write(f"{HEALTH_CONDITION}={hc['status']} ({hc['reason']}, heartbeat {_age(hc['heartbeat_age_s'])} ago): "
                  f"{hc['message']}\n")
    else:
        out.write(f"{HEALTH_CONDITION}: not published (no node agent)\n")
    v = doc["verdict"]
    if v is None:
        out.write(f"MI355X verdict: none (policy {doc['health_policy']}: the reference's Ready rule applies)\n")
    else:
        out.write(f"MI355X verdict: {v['state']}, {v['gpus_ok']}/{v['gpus_seen']} GPUs ok"
                  + (f", published {_age(v['age_s'])} ago" if v.get("age_s") is not None else "") + "\n")
        for title in ("reasons", "warnings"):
            for r in v.get(title) or []:
                out.write(f"  {title[:-1]}: {r}\n")
    rep = doc["report"]
    if rep and rep.get("error"):
        out.write(f"report: unreadable ({rep['error']})\n")
    elif rep:
        out.write(f"report: probe {rep['probe'] or '?'}, amd-smi {rep['amdsmi'] or '?'}, driver "
                  f"{rep['driver'] or '?'}, {len(rep['gpus'])} GPUs\n")
        for ln in gpu_table(rep["gpus"]):
            out.write("  " + ln + "\n")
        for ln in rep["node_findings"]:
            out.write(f"  node: {ln}\n")
    fd = doc.get("fleet_diag")
    if fd:
        low = sorted(fd.get("node_ratio", {}).items(), key=lambda kv: kv[1])[:3]
        if low:
            out.write("  fleet: lowest against the fleet's median node: "
                      + ", ".join(f"{k} x{r:.2f}" for k, r in low) + "\n")
        for ln in fd["explained"]:
            out.write(f"  fleet: {ln}\n")
    out.write(f"=> counts as Ready: {'yes' if doc['counts_as_ready'] else 'no'}\n")


def explain(cluster: ClusterConnection, node_name: str, opts: CheckOptions, out: TextIO) -> int:
    as_json = opts.json
    doc = diagnose(cluster, node_name, opts)
    if as_json:
        out.write(json.dumps(doc, indent=2, ensure_ascii=False) + "\n")
    else:
        render(doc, out)
    return 2 if not doc["gpu_node"] else 0 if doc["counts_as_ready"] else 3


def opts_keys() -> List[str]:
    from .models.resources import GPU_RESOURCE_KEYS
    return list(GPU_RESOURCE_KEYS)


def fleet(cluster: ClusterConnection, opts: CheckOptions, out: TextIO) -> int:
    """``check-gpu-node --fleet``: the cluster's MI355X nodes at a glance -- how many count as Ready, the
    verdicts by state, every node that is not healthy with its first reason, and the driver / firmware
    versions across the nodes that publish a report (two versions of one image = a partial upgrade).
    Exit code as the plain check (0 / 2 / 3)."""
    as_json = opts.json
    opts.json_extended = True  # every report annotation is read (fleet versions)
    res = run_check(cluster, opts)
    nodes = res.gpu_nodes
    verdicts = res.verdicts or []
    by_state: Dict[str, int] = {}
    for v in verdicts:
        if v is not None:
            by_state[v.state] = by_state.get(v.state, 0) + 1
    unjudged = len(nodes) - sum(by_state.values())
    if as_json:
        attention = []
        for i, n in enumerate(nodes):
            v = verdicts[i] if i < len(verdicts) else None
            if (v is not None and v.state != "healthy") or not n["ready"]:
                attention.append({"name": n["name"], "ready": n["ready"], "state": v.state if v else None,
                                  "reasons": v.reasons if v else [], "warnings": v.warnings if v else []})
        out.write(json.dumps({"total_nodes": len(nodes), "ready_nodes": len(res.ready_gpu_nodes),
                              "verdicts": by_state, "without_verdict": unjudged, "attention": attention,
                              "fleet": fleet_versions(res.scan.extras), "diag_fleet": res.fleet_diag},
                             indent=2, ensure_ascii=False) + "\n")
        return res.exit_code
    out.write(f"GPU nodes: {len(nodes)}, counting as Ready: {len(res.ready_gpu_nodes)}\n")
    parts = [f"{n} {s}" for s, n in sorted(by_state.items(), key=lambda kv: ("healthy", "degraded", "unhealthy",
                                                                              "unknown").index(kv[0])
                                                  if kv[0] in ("healthy", "degraded", "unhealthy", "unknown") else 9)]
    out.write("MI355X verdicts: " + (", ".join(parts) if parts else "none") +
              (f"; {unjudged} without a verdict" if unjudged and parts else "") + "\n")
    for i, n in enumerate(nodes):
        v = verdicts[i] if i < len(verdicts) else None
        if v is not None and v.state != "healthy":
            why = (v.reasons or v.warnings or [""])[0]
            more = len(v.reasons) + len(v.warnings) - 1
            out.write(f"  {n['name']}: {v.state}{' (not Ready)' if not n['ready'] else ''}  {why}"
                      + (f"  (+{more} more)" if more > 0 else "") + "\n")
        elif not n["ready"]:
            out.write(f"  {n['name']}: not Ready\n")
    fv = fleet_versions(res.scan.extras)
    if fv:
        out.write(f"versions across {fv['nodes_reporting']} reporting nodes"
                  + (f" (mixed: {', '.join(fv['mixed'])})" if fv["mixed"] else "") + ":\n")
        if fv["driver"]:
            out.write("  driver: " + ", ".join(f"{k} x{c}" for k, c in sorted(fv["driver"].items())) + "\n")
        for image, row in fv["firmware"].items():
            out.write(f"  {image}: " + ", ".join(f"{k} x{c}" for k, c in sorted(row.items())) + "\n")
    if res.fleet_diag:
        out.write("diagnostics across the fleet (node medians, fraction of the MI355X reference; fabric in GB/s):\n")
        for test, row in res.fleet_diag.items():
            def fmt(x, unit=row.get("unit")):
                return f"{x:.0f} GB/s" if unit == "GB/s" else f"{x:.0%}"
            out.write(f"  {test}: {row['nodes']} nodes, median {fmt(row['median_fraction'])} "
                      f"({fmt(row['min_fraction'])}-{fmt(row['max_fraction'])})"
                      + ("  platform shortfall: nodes in line with it are not degraded for it"
                         if row["platform_shortfall"] else "")
                      + ("  outliers: " + ", ".join(f"{o['node']} x{o['ratio']:.2f}" for o in row["outliers"])
                         if row["outliers"] else "")
                      + ("  behind at the reference: " + ", ".join(f"{o['node']} x{o['ratio']:.2f}"
                                                                   for o in row["behind_at_reference"])
                         if row.get("behind_at_reference") else "")
                      + ("  slowest: " + ", ".join(f"{x['node']} {fmt(x['fraction'])}" for x in row.get("slowest", []))
                         if not row["outliers"] else "") + "\n")
    return res.exit_code
