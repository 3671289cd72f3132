"""Fleet-relative judgement of the active diagnostics' rates: each MI355X node against the other nodes of the
same check.

The node agent judges a GPU against the other GPUs of its node (``models/peers.py``) and against its own history
(``models/baseline.py``); what it cannot see is the rest of the fleet.  Two verdicts need that view, and the
checker has it -- one LIST carries every node's report:

* **platform-wide shortfall** -- when the fleet's median node sits below the degraded line for a test and metric
  (the whole fleet is a slower platform than the single boxes the references were measured on: its cooling,
  power limits, firmware), a node in line with that median (within ``FLEET_UNIFORM_SPREAD``) is not degraded
  for it: its node-wide finding and its GPUs' slow-only results (lone GPUs judged against the references) are
  the platform's normal, not warnings.  The absolute failure floor stays: a GPU under ``FAIL_FRACTION`` of its
  reference still fails, as the agent judged it;
* **node outlier** -- a node whose median GPU is below ``FLEET_FAIL_RATIO`` of the median of the *other* nodes
  gets a ``degraded`` finding naming the fleet median: all of its GPUs are slow alike (else the agent would
  have singled one out), which is the node's condition -- cooling, power delivery, a BIOS setting -- and a
  warning, never a failure.  A node at or above the degraded line of the references gets no finding and is no
  outlier (the rest of the fleet is fast, not it slow); the summary lists it under ``behind_at_reference``.

It needs at least ``FLEET_MIN_NODES`` nodes with results for the same test, shape and metric, and it needs the
reports themselves (``--health-reeval``, ``--probe-endpoint``, or nodes that publish no condition): on the
condition-only path the checker trusts the agents' verdicts as they are.  Reference analogue: the reference's
verdict is a stable binary read off each node (``/root/reference/check-gpu-node.py:172-178``); this keeps the
MI355X gate equally stable on a fleet whose platform differs from the reference boxes.
"""

from __future__ import annotations

import statistics
from typing import Any, Dict, List, Optional, Tuple

from .peers import DEGRADED_FRACTION, FAIL_FRACTION, _rate_fractions

FLEET_MIN_NODES = 3
# the MI355X's identifiers (models/health.MI35X_DEVICE_IDS, amd-smi product name): results keyed without a model
MI355X_IDS = ("0x75a3", "amd instinct mi355 oam")
# a node below this share of the other nodes' median is an outlier (the per-GPU peer ratio, one level up)
FLEET_FAIL_RATIO = 0.85
# a node within this ratio of the fleet's median shares the fleet's condition
FLEET_UNIFORM_SPREAD = 1.10

Key = Tuple[str, str, str]  # (test, shape, metric)


def _size(res: Dict[str, Any]) -> str:
    for k in ("shape", "gib", "slice_mib"):
        if k in res:
            return repr(res[k])
    return ""


def _shape(res: Dict[str, Any], gpu: Any = None) -> str:
    """What makes two results comparable besides the test: its size, and the GPU model (an MI350X is compared
    with MI350Xs -- its rates sit under an MI355X's at the same fraction of the MI355X references)."""
    model = (gpu.get("device_id") or gpu.get("product_name")) if isinstance(gpu, dict) else None
    suffix = f" on {model}" if isinstance(model, str) and model and model.lower() not in MI355X_IDS else ""
    return _size(res) + suffix


# node-level fabric results (level 2, ``report["fabric"]``) compared across nodes as raw rates: no reference
# to be short of, so outliers only (a node whose xGMI pairs or RCCL collectives run well under the others')
RAW_TESTS = ("xgmi_p2p", "rccl")


def _num(v: Any) -> bool:
    return isinstance(v, (int, float)) and not isinstance(v, bool) and v > 0


def node_fractions(report: Any) -> Dict[Key, float]:
    """``(test, shape, metric) -> the node's median GPU`` (rate as a fraction of its scaled reference), plus the
    node-level fabric rates (``RAW_TESTS``, GB/s, keyed by how many GPUs took part)."""
    # the checker runs this over every node of a report-reading LIST (1000 nodes x 8 GPUs x 7 tests): one flat
    # pass, the GPU model resolved once per GPU, numbers tested by exact type (a bool is not a rate)
    per: Dict[Key, List[float]] = {}
    gpus = report.get("gpus") if isinstance(report, dict) else None
    for g in gpus if isinstance(gpus, list) else ():
        diag = g.get("diag") if isinstance(g, dict) else None
        if not isinstance(diag, dict):
            continue
        suffix = _shape({}, g)  # " on <model>" for other GPU models, "" for the MI355X
        for test, res in diag.items():
            if type(res) is not dict:
                continue
            rates, expect = res.get("rates"), res.get("expect")
            if type(rates) is not dict or type(expect) is not dict:
                continue
            shape = None
            for m, v in rates.items():
                e = expect.get(m)
                tv, te = type(v), type(e)
                if (tv is float or tv is int) and (te is float or te is int) and v >= 0 and e > 0:
                    if shape is None:
                        shape = _size(res) + suffix
                    key = (test, shape, m)
                    lst = per.get(key)
                    if lst is None:
                        per[key] = [v / e]
                    else:
                        lst.append(v / e)
    out = {k: (v[0] if len(v) == 1 else statistics.median(v)) for k, v in per.items()}
    fab = report.get("fabric") if isinstance(report, dict) else None
    if isinstance(fab, dict):
        p2p, rccl = fab.get("p2p"), fab.get("rccl")
        if isinstance(p2p, dict) and _num(p2p.get("median_gbps")) and isinstance(p2p.get("pairs"), list):
            out[("xgmi_p2p", f"pairs={len(p2p['pairs'])}", "median_gbps")] = float(p2p["median_gbps"])
        if isinstance(rccl, dict) and _num(rccl.get("best_busbw_gbps")) and isinstance(rccl.get("world"), int):
            out[("rccl", f"world={rccl['world']}", "busbw_gbps")] = float(rccl["best_busbw_gbps"])
    return out


def summary_key(key: Key) -> str:
    """``test@shape/metric``: a key of ``judge_fleet``'s summary."""
    return f"{key[0]}{('@' + key[1]) if key[1] else ''}/{key[2]}"


def _loo_medians(vals: Dict[int, float]) -> Dict[int, float]:
    """Each member's leave-one-out median (the median of the *other* members' values), O(n log n) for the
    whole set: one sort, then the median of the sorted list with one position skipped."""
    order = sorted(vals, key=lambda i: vals[i])
    s = [vals[i] for i in order]
    n = len(s)
    if n < 2:
        return {}  # nobody else to compare with
    L = n - 1

    def at(j: int, k: int) -> float:  # element j of s with position k removed
        return s[j] if j < k else s[j + 1]
    out = {}
    for k, i in enumerate(order):
        out[i] = at(L // 2, k) if L % 2 else (at(L // 2 - 1, k) + at(L // 2, k)) / 2.0
    return out


def judge_fleet(names: List[str], reports: List[Optional[Dict[str, Any]]],
                fractions: Optional[List[Optional[Dict[Key, float]]]] = None
                ) -> Tuple[Dict[str, Any], List[Optional[Dict[str, Any]]]]:
    """Judge every report's rate tests against the fleet.  The reports are not changed (the watcher keeps them
    across checks); the judgement comes back as one view per node, which ``models/health.evaluate_report``
    takes as ``fleet=``:

    * ``findings`` -- this node is an outlier for a test and metric (a warning each);
    * ``explained`` -- ``(test, shape, metric) -> {"fleet_fraction", "nodes"}``: the fleet is short alike there
      and this node is in line with it, so its node-wide finding and its GPUs' slow-only results for it are
      not warnings.

    ``reports`` is parallel to ``names`` (None where a node has no report to judge); a node with nothing to say
    gets None.  The summary, per test: node count, median, min and max fraction, the outliers, the three slowest
    nodes and whether the fleet is short alike.  ``fractions`` (parallel, optional): reports' ``node_fractions``
    already computed (``NodeExtras.fleet_fractions`` caches them per node object)."""
    values: Dict[Key, Dict[int, float]] = {}
    for i, rep in enumerate(reports):
        if not isinstance(rep, dict):
            continue
        fr = fractions[i] if fractions is not None and fractions[i] is not None else node_fractions(rep)
        for key, v in fr.items():
            values.setdefault(key, {})[i] = v
    views: List[Optional[Dict[str, Any]]] = [None] * len(reports)

    def view(i: int) -> Dict[str, Any]:
        if views[i] is None:
            views[i] = {"findings": [], "explained": {}}
        return views[i]  # type: ignore[return-value]
    summary: Dict[str, Any] = {}
    for key in sorted(values):
        vals = values[key]
        if len(vals) < FLEET_MIN_NODES:
            continue
        med = statistics.median(vals.values())
        raw = key[0] in RAW_TESTS
        platform_short = not raw and med < DEGRADED_FRACTION
        row: Dict[str, Any] = {"nodes": len(vals), "unit": "GB/s" if raw else "fraction",
                               "median_fraction": round(med, 3),
                               "min_fraction": round(min(vals.values()), 3),
                               "max_fraction": round(max(vals.values()), 3), "platform_shortfall": platform_short,
                               "outliers": [],
                               "slowest": [{"node": names[i], "fraction": round(v, 3)}
                                           for i, v in sorted(vals.items(), key=lambda kv: (kv[1], kv[0]))[:3]]}
        loo = _loo_medians(vals)
        for i, v in vals.items():
            others = loo[i]
            ratio = v / others if others > 0 else 1.0
            if ratio < FLEET_FAIL_RATIO:
                if not raw and v >= DEGRADED_FRACTION:
                    # at the MI355X reference itself: the rest of the fleet is fast, this node is not slow
                    # (healthy devices differ by up to ~14 %, profiles/diag_box_spread_r05_mi355x.jsonl)
                    row.setdefault("behind_at_reference", []).append({"node": names[i], "ratio": round(ratio, 3)})
                    continue
                row["outliers"].append({"node": names[i], "ratio": round(ratio, 3)})
                f = {"test": key[0], "metric": key[2], "ratio": round(ratio, 3), "nodes": len(vals) - 1}
                if raw:
                    f.update(node_value=round(v, 1), fleet_value=round(others, 1))
                else:
                    f.update(node_fraction=round(v, 3), fleet_fraction=round(others, 3))
                view(i)["findings"].append(f)
            elif platform_short and max(v, med) <= FLEET_UNIFORM_SPREAD * min(v, med):
                view(i)["explained"][key] = {"fleet_fraction": round(med, 3), "nodes": len(vals)}
        summary[summary_key(key)] = row
    return summary, views


def explains_node_finding(fleet: Optional[Dict[str, Any]], f: Dict[str, Any]) -> bool:
    """A node-wide finding (``models/peers``) the fleet's own shortfall accounts for (not one below the floor)."""
    if not fleet or not fleet.get("explained") or f.get("below_floor"):
        return False
    return any(k[0] == f.get("test") and k[2] == f.get("metric") for k in fleet["explained"])


def explains_gpu_result(fleet: Optional[Dict[str, Any]], test: str, res: Dict[str, Any], gpu: Any = None) -> bool:
    """A GPU's degraded result that is only slow -- no failure, lag or drift -- on metrics the fleet is short
    alike on, with the GPU itself in line with the fleet's median."""
    if not fleet or not fleet.get("explained"):
        return False
    if res.get("pass") is not True or not res.get("degraded") or res.get("lag") or res.get("drift"):
        return False  # failures, and lag / drift notes, are the GPU's own whatever the fleet does
    fr = _rate_fractions(res)
    if not fr or min(fr.values()) < FAIL_FRACTION:
        return False
    shape = _shape(res, gpu)
    for m, v in fr.items():
        if v >= DEGRADED_FRACTION:
            continue
        ex = fleet["explained"].get((test, shape, m))
        if not ex:
            return False
        med = ex["fleet_fraction"]
        if max(v, med) > FLEET_UNIFORM_SPREAD * min(v, med):
            return False
    return True


def explained_text(fleet: Dict[str, Any]) -> List[str]:
    """What the fleet explained on this node, for ``--explain`` / ``--json-extended`` notes."""
    return [f"diag {t} {m}: the fleet's median node is at {ex['fleet_fraction']:.0%} of the MI355X reference "
            f"({ex['nodes']} nodes alike): the platform's normal, not this node's"
            for (t, _s, m), ex in sorted(fleet.get("explained", {}).items())]


def finding_text(f: Dict[str, Any]) -> str:
    """One fleet outlier finding as a verdict warning."""
    if "node_value" in f:
        return (f"fleet: {f.get('test')} {f.get('metric')} at {f.get('ratio', 0):.0%} of the other {f.get('nodes')} "
                f"nodes' median ({f.get('node_value')} vs {f.get('fleet_value')}): this node's xGMI fabric")
    return (f"fleet: diag {f.get('test')} {f.get('metric')} at {f.get('ratio', 0):.0%} of the other "
            f"{f.get('nodes')} nodes' median ({f.get('node_fraction', 0):.0%} vs {f.get('fleet_fraction', 0):.0%} of "
            f"the MI355X reference): this node's cooling, power or firmware")
