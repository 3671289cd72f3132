"""Peer-relative judgement of the active diagnostics' rates across the GPUs of one node.

A GPU's rates (GEMM TFLOP/s, HBM TB/s, ...) were judged against absolute references measured on single
healthy MI355X boxes (``ops/diag.REFERENCE_RATES``).  Those references move with what a node is -- its
cooling, power delivery, firmware, BIOS -- so a whole healthy fleet of a slower platform would sit under
them and be reported ``degraded`` or ``unhealthy`` for what is the platform's normal.  The reference
checker's verdict is a stable binary read off the node itself (``/root/reference/check-gpu-node.py:172-178``);
this module gives the MI355X gate the same stability.  On a node whose GPUs were measured together, each
GPU is judged against the other GPUs of the same node, which share every one of those conditions:

* **outlier** -- a GPU below ``PEER_FAIL_RATIO`` of the median of the *other* GPUs (leave-one-out, so with two
  GPUs the slower is judged against the faster) fails, and the failure names it -- unless the GPU itself is at
  or above the absolute degraded line: then its peers are fast, not it slow, and it is ``degraded`` with the
  ratio in the detail.  Healthy MI355X devices differ by up to ~14 % on MFMA-bound tests under the same code
  (two devices of one pool, profiles/diag_box_spread_r05_mi355x.jsonl: GEMM 1,280 vs 1,484 TFLOP/s, MX-fp4
  7,028 vs 8,171), so a slow-but-healthy GPU next to fast ones sits near 0.85 of them;
* **node-wide shortfall** -- when the remaining GPUs agree within ``NODE_UNIFORM_SPREAD`` and their median is
  below the degraded line, the node gets one node-level ``degraded`` finding: every GPU is slow alike, which
  is the node's condition, not a GPU's.  Only down to the absolute failure line: when the shared median is
  under ``FAIL_FRACTION`` the finding is still recorded (``below_floor``) but each GPU is also judged against
  the references, so a node whose GPUs all run at 30 % fails;
* otherwise (the GPUs disagree without a clear outlier, e.g. half of them slow) each GPU falls back to the
  absolute references, as does a lone GPU (fewer than ``MIN_PEERS`` measured).

Numerics (wrong results, checksums), lagging XCDs/CUs and drift from the GPU's own baseline
(``models/baseline.py``) are per-GPU findings whatever the peers say.

Rates are compared as fractions of each GPU's own scaled reference (``rates[k] / expect[k]``), so GPUs of
different partition modes or power caps on one node still compare like for like.  The judgement is a pure
function of the raw fields ``ops/diag._rated`` records (``rates``, ``expect``, ``unit``, ``numerics``,
``lag``, ``drift``): re-judging a result gives the same answer, so the agent re-judges every cycle.
"""

from __future__ import annotations

import statistics
from typing import Any, Dict, Hashable, List, Optional

# a GPU below this share of the median of its node's other GPUs fails (the absolute floor's 0.85, applied to
# peers: healthy MI355X spread box to box ~10 % on DVFS, but GPUs of one node share the box)
PEER_FAIL_RATIO = 0.85
# GPUs whose rates agree within this ratio (max / min) are "alike": any shortfall they share is node-wide
NODE_UNIFORM_SPREAD = 1.10
MIN_PEERS = 2
# the absolute lines (ops/diag.py), repeated so this module needs no ctypes import
FAIL_FRACTION = 0.85
DEGRADED_FRACTION = 0.95


def _rate_fractions(res: Dict[str, Any]) -> Dict[str, float]:
    rates, expect = res.get("rates"), res.get("expect")
    if not isinstance(rates, dict) or not isinstance(expect, dict):
        return {}
    out = {}
    for k, v in rates.items():
        e = expect.get(k)
        if isinstance(v, (int, float)) and isinstance(e, (int, float)) and e > 0:
            out[k] = float(v) / float(e)
    return out


def _absolute(res: Dict[str, Any]) -> Dict[str, Any]:
    from ..ops.diag import judge_absolute  # ctypes-free at import: ops.diag loads its library lazily
    return judge_absolute(res)


def judge_node(results: Dict[Hashable, Dict[str, Any]], label: Optional[Dict[Hashable, str]] = None) -> List[Dict[str, Any]]:
    """Re-judge every rate test of ``results`` (device -> {test: result}) against the node's other GPUs, in
    place; returns the node-level findings (one per test and metric with a node-wide shortfall).

    ``label`` names devices in the details (default ``gpu{device}``)."""
    label = label or {}
    tests = sorted({t for r in results.values() if isinstance(r, dict)
                    for t, x in r.items() if isinstance(x, dict) and _rate_fractions(x)})
    findings: List[Dict[str, Any]] = []
    for test in tests:
        members = {d: r[test] for d, r in results.items()
                   if isinstance(r, dict) and isinstance(r.get(test), dict) and _rate_fractions(r[test])}
        if len(members) < MIN_PEERS:
            for res in members.values():
                _absolute(res)
            continue
        fr = {d: _rate_fractions(res) for d, res in members.items()}
        metrics = sorted(set.intersection(*(set(f) for f in fr.values())))
        problems: Dict[Hashable, List[str]] = {d: [] for d in members}
        slow: Dict[Hashable, List[str]] = {d: [] for d in members}
        peer_ratio: Dict[Hashable, Dict[str, float]] = {d: {} for d in members}
        for m in metrics:
            vals = {d: fr[d][m] for d in members}
            peer_fail = set()
            for d, v in vals.items():
                others = statistics.median([x for j, x in vals.items() if j != d])
                ratio = v / others if others > 0 else 1.0
                peer_ratio[d][m] = round(ratio, 3)
                if ratio < PEER_FAIL_RATIO:
                    peer_fail.add(d)
                    res = members[d]
                    unit = res.get("unit", "")
                    rate = res["rates"][m]
                    peers = statistics.median([members[j]["rates"][m] for j in members if j != d])
                    txt = f"{m} {rate:.3g} {unit} = {ratio:.0%} of the node's other GPUs' median {peers:.3g}"
                    if v >= DEGRADED_FRACTION:  # at the MI355X reference itself: its peers are the fast ones
                        slow[d].append(f"{txt} (itself at {v:.0%} of the MI355X reference)")
                    else:
                        problems[d].append(txt)
            alike = [d for d in vals if d not in peer_fail]
            span = [vals[d] for d in alike]
            uniform = len(alike) >= MIN_PEERS and max(span) <= NODE_UNIFORM_SPREAD * min(span)
            if uniform:
                med = statistics.median(span)
                if med < DEGRADED_FRACTION:
                    findings.append({"test": test, "metric": m, "median_fraction": round(med, 3),
                                     "min_fraction": round(min(span), 3), "max_fraction": round(max(span), 3),
                                     "gpus": len(alike), "below_floor": med < FAIL_FRACTION})
                if med >= FAIL_FRACTION:
                    continue
                # alike but under the absolute failure floor: peers excuse a shortfall between the degraded and
                # the failure lines only -- eight GPUs at 30 % of the reference are eight failed GPUs, not a
                # node-level note (the floor stays, models/fleet.py)
            for d in alike:  # GPUs that disagree without a clear outlier, or alike under the floor: the references
                res = members[d]
                v, e = res["rates"][m], res["expect"][m]
                txt = f"{m} {v:.3g} {res.get('unit', '')} = {vals[d]:.0%} of {e:.3g}"
                if vals[d] < FAIL_FRACTION:
                    problems[d].append(txt)
                elif vals[d] < DEGRADED_FRACTION:
                    slow[d].append(txt)
        for d, res in members.items():
            # pass / degraded from the per-metric judgements above, plus what peers cannot excuse
            worst = min(fr[d].values()) if fr[d] else 1.0
            probs = ([res["numerics"]] if res.get("numerics") else []) + problems[d]
            notes = [str(x) for key in ("lag", "drift") for x in (res.get(key) or []) if x]
            res["pass"] = not probs
            res["degraded"] = bool(slow[d] or notes) and not probs
            res["fraction"] = round(worst, 3)
            res["detail"] = "; ".join(probs or (slow[d] + notes))
            res["peers"] = {"gpus": len(members), "ratio": peer_ratio[d]}
    return findings


def finding_text(f: Dict[str, Any]) -> str:
    """One node-level finding as a verdict reason (``models/health`` warnings)."""
    lo, hi = f.get("min_fraction"), f.get("max_fraction")
    span = f" ({lo:.0%}-{hi:.0%})" if isinstance(lo, (int, float)) and isinstance(hi, (int, float)) else ""
    return (f"node-wide: diag {f.get('test')} {f.get('metric')} at {f.get('median_fraction', 0):.0%} of the "
            f"MI355X reference on all {f.get('gpus')} GPUs alike{span} (the node's cooling, power or firmware, "
            f"not one GPU)")
