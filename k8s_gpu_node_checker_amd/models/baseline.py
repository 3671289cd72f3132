"""Per-GPU self-baselines for the active diagnostics' rates (the node agent keeps one per GPU).

The first ``runs`` clean results of a GPU (passed, not degraded, on the same test shape) fix its baseline:
the median of each rate as a fraction of its scaled reference.  From then on a result whose rate falls below
``drift_ratio`` of that GPU's own baseline carries a ``drift`` note, which the judgements
(``ops/diag.judge_absolute``, ``models/peers.judge_node``) turn into ``degraded``: the GPU got slower than it
used to be, even when it is still above the fleet-wide references and in line with its node's other GPUs
(a node whose GPUs all age alike).  Drift is a warning, never a failure: the absolute and peer floors decide
failures.

Keyed by the GPU's amd-smi UUID (its PCI address when there is none) so a replaced board starts a new
baseline; the test's shape is part of the key (the level-1 4096^3 and level-2 8192^3 GEMMs differ).  With a
``path`` the baselines persist as JSON across agent restarts (written atomically; an unreadable file starts
empty rather than failing the agent).  Reference analogue: none -- the reference re-derives its binary
verdict from each LIST (``/root/reference/check-gpu-node.py:172-178``); this is the per-GPU memory that
lets a verdict stay stable across boxes without re-tuning constants.
"""

from __future__ import annotations

import json
import os
import statistics
import threading
import time
from typing import Any, Dict, List, Optional

SCHEMA = "mi355x-diag-baseline/v1"
BASELINE_RUNS = 5
DRIFT_RATIO = 0.90


def _fractions(res: Dict[str, Any]) -> Dict[str, float]:
    from .peers import _rate_fractions
    return _rate_fractions(res)


def _shape(test: str, res: Dict[str, Any]) -> str:
    for k in ("shape", "gib", "slice_mib"):
        if k in res:
            return f"{test}@{json.dumps(res[k], separators=(',', ':'))}"
    return test


def gpu_key(entry: Dict[str, Any], fallback: str = "") -> str:
    """The identity a baseline belongs to: amd-smi UUID, else PCI address, else ``fallback``."""
    for k in ("uuid", "bdf"):
        v = entry.get(k) if isinstance(entry, dict) else None
        if isinstance(v, str) and v.strip():
            return f"{k}:{v.strip().lower()}"
    return fallback


class Baselines:
    def __init__(self, path: Optional[str] = None, runs: int = BASELINE_RUNS, drift_ratio: float = DRIFT_RATIO):
        if runs < 1:
            raise ValueError("runs must be >= 1")
        self.path = path
        self.runs = runs
        self.drift_ratio = drift_ratio
        self.lock = threading.Lock()
        self.data: Dict[str, Dict[str, Any]] = {}
        if path:
            self._load()

    def _load(self) -> None:
        try:
            with open(self.path, encoding="utf-8") as f:  # type: ignore[arg-type]
                doc = json.load(f)
        except (OSError, ValueError):
            return
        if isinstance(doc, dict) and doc.get("schema") == SCHEMA and isinstance(doc.get("gpus"), dict):
            self.data = {k: v for k, v in doc["gpus"].items() if isinstance(v, dict)}

    def _save(self) -> None:
        if not self.path:
            return
        tmp = f"{self.path}.tmp{os.getpid()}"
        try:
            with open(tmp, "w", encoding="utf-8") as f:
                json.dump({"schema": SCHEMA, "gpus": self.data}, f, indent=1, sort_keys=True)
            os.replace(tmp, self.path)
        except OSError:
            try:
                os.unlink(tmp)
            except OSError:
                pass

    def baseline(self, gpu: str, test: str, res: Dict[str, Any]) -> Optional[Dict[str, float]]:
        entry = self.data.get(gpu, {}).get(_shape(test, res))
        return dict(entry["baseline"]) if isinstance(entry, dict) and isinstance(entry.get("baseline"), dict) else None

    def observe(self, gpu: str, results: Dict[str, Dict[str, Any]], now: Optional[float] = None) -> List[str]:
        """Fold one fresh diagnostic result of GPU ``gpu`` (test -> result) in: set ``drift`` on each rate test
        below ``drift_ratio`` of its baseline (``baseline`` records the ratios), or add the clean ones to the
        baseline still forming.  Returns the drift notes.  Call once per fresh result: the judgement is
        re-applied from the recorded fields, so cached results keep their notes without being observed again."""
        notes: List[str] = []
        now = time.time() if now is None else now
        changed = False
        with self.lock:
            per = self.data.setdefault(gpu, {})
            for test, res in results.items():
                if not isinstance(res, dict):
                    continue
                fr = _fractions(res)
                if not fr:
                    continue
                key = _shape(test, res)
                entry = per.get(key)
                if not isinstance(entry, dict):
                    entry = per[key] = {"samples": []}
                base = entry.get("baseline")
                if isinstance(base, dict):
                    ratios = {m: round(v / base[m], 3) for m, v in fr.items()
                              if isinstance(base.get(m), (int, float)) and base[m] > 0}
                    res["baseline"] = {"ratio": ratios, "runs": entry.get("runs", self.runs)}
                    drift = [f"{m} at {r:.0%} of this GPU's own baseline ({entry.get('runs', self.runs)} clean runs)"
                             for m, r in sorted(ratios.items()) if r < self.drift_ratio]
                    if drift:
                        res["drift"] = drift
                        notes += [f"{test}: {d}" for d in drift]
                    else:
                        res.pop("drift", None)
                    continue
                clean = res.get("pass") is True and not res.get("degraded") and not res.get("numerics")
                if clean:
                    samples = entry.get("samples")  # a hand-edited or truncated file: keep what is well-formed
                    entry["samples"] = [s for s in samples if isinstance(s, dict)] if isinstance(samples, list) else []
                    entry["samples"].append({m: round(v, 4) for m, v in fr.items()})
                    changed = True
                    if len(entry["samples"]) >= self.runs:
                        ms = set.intersection(*(set(s) for s in entry["samples"]))
                        entry["baseline"] = {m: round(statistics.median(s[m] for s in entry["samples"]), 4)
                                             for m in sorted(ms)}
                        entry["runs"] = len(entry["samples"])
                        entry["since"] = round(now, 1)
                        del entry["samples"]
            if changed:
                self._save()
        return notes
