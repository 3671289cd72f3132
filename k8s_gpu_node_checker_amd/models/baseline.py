"""Per-GPU self-baselines for the active diagnostics' rates (the node agent keeps one per GPU).

The first ``runs`` clean results of a GPU (same test shape) fix its baseline: the median of each rate as a
fraction of its scaled reference.  From then on a result whose rate falls below ``drift_ratio`` of that GPU's
own baseline carries a ``drift`` note, which the judgements (``ops/diag.judge_absolute``,
``models/peers.judge_node``) turn into ``degraded``: the GPU got slower than it used to be, even when it is
still above the fleet-wide references and in line with its node's other GPUs (a node whose GPUs all age
alike).  Drift is a warning, never a failure: the absolute and peer floors decide failures.

**Clean** is decided from the result's own numbers, not from the peer- or fleet-adjusted ``pass`` /
``degraded`` flags: no numerics failure, no lagging XCD/CU, and every rate at or above the absolute failure
line (``FAIL_FRACTION`` of the reference).  So a lone GPU that sits at 0.93 -- absolutely "degraded" --
still forms a baseline and later sees its own decay as drift, while a GPU whose peers excused a shortfall
never forms a baseline at a fault level.

**Epochs.**  A baseline belongs to the software it was measured under: the amdgpu driver release, the VBIOS
and the firmware image set amd-smi reports for that GPU.  When the epoch changes (a ROCm or firmware
upgrade that moves a rate by more than the drift margin, either way) the GPU's baselines are re-formed from
the next clean runs, with no drift warning in between; the old epoch is kept as ``previous``.  Epochs are compared
component by component (driver, VBIOS, each firmware image), and only a component both sides know and that differs
is a change: one probe where amd-smi could not read the VBIOS or the driver is not a new epoch (the missing part is
kept from before), and a component seen for the first time is filled in without re-forming anything.

**Revisions.**  A baseline is a fraction of the diagnostics' reference rates, so it also belongs to those and to
the kernel that measured them (``ops/diag.rate_revision``): each test's entry records the revision it formed
under, and a test whose kernel or references changed re-forms alone.  Entries from before revisions (schema v1
and v2 files) were formed under references that can no longer be told, so they are dropped on load and re-form.

Keyed by the GPU's amd-smi UUID (its PCI address when there is none) so a replaced board starts a new
baseline; the test's shape is part of the key (the level-1 4096^3 and level-2 8192^3 GEMMs differ).  With a
``path`` the baselines persist as JSON across agent restarts (written atomically; an unreadable file starts
empty rather than failing the agent).  :meth:`Baselines.drop` forgets chosen GPUs (agent
``--diag-baseline-reset``, ``POST /baseline/reset`` from inside the pod).  Reference analogue: none -- the
reference re-derives its binary verdict from each LIST (``/root/reference/check-gpu-node.py:172-178``); this
is the per-GPU memory that lets a verdict stay stable across boxes without re-tuning constants.
"""

from __future__ import annotations

import json
import os
import statistics
import threading
import time
from typing import Any, Callable, Dict, Iterable, List, Optional

SCHEMA = "mi355x-diag-baseline/v3"
SCHEMA_V2 = "mi355x-diag-baseline/v2"
SCHEMA_V1 = "mi355x-diag-baseline/v1"
BASELINE_RUNS = 5
DRIFT_RATIO = 0.90
# the absolute failure line of ops/diag (and models/peers): a run under it is never part of a baseline
FAIL_FRACTION = 0.85


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


def epoch_of(entry: Optional[Dict[str, Any]], driver_version: Any = None) -> Optional[str]:
    """The software a GPU's rates are measured under, as one string: ``driver <release>; vbios <version>;
    fw <image>=<version>,...`` (amd-smi's firmware list, sorted).  None when nothing is known."""
    from .health import driver_release, fw_version_str
    parts: Dict[str, str] = {}
    if driver_version:
        parts["driver"] = str(driver_release(driver_version))
    e = entry if isinstance(entry, dict) else {}
    vb = e.get("vbios_version")
    if isinstance(vb, str) and vb.strip():
        parts["vbios"] = vb.strip()
    fw = e.get("fw")
    if isinstance(fw, dict):
        for k in fw:
            parts[f"fw:{k}"] = fw_version_str(k, fw[k])
    return epoch_str(parts)


def epoch_str(parts: Dict[str, str]) -> Optional[str]:
    """:func:`epoch_of`'s string of an epoch's components (``driver``, ``vbios``, ``fw:<image>``)."""
    out = [f"{k} {parts[k]}" for k in ("driver", "vbios") if parts.get(k)]
    fw = sorted((k[3:], v) for k, v in parts.items() if k.startswith("fw:"))
    if fw:
        out.append("fw " + ",".join(f"{k}={v}" for k, v in fw))
    return "; ".join(out) or None


def epoch_parts(epoch: Optional[str]) -> Dict[str, str]:
    """The components of an :func:`epoch_of` string (the inverse of :func:`epoch_str`)."""
    parts: Dict[str, str] = {}
    for piece in (epoch or "").split("; "):
        kind, _, rest = piece.partition(" ")
        if kind in ("driver", "vbios") and rest:
            parts[kind] = rest
        elif kind == "fw" and rest:
            for image in rest.split(","):
                k, eq, v = image.partition("=")
                if eq:
                    parts[f"fw:{k}"] = v
    return parts


def epoch_change(old: Optional[str], new: Optional[str]) -> tuple:
    """(changed, merged epoch) of a GPU's stored epoch ``old`` against this probe's ``new``: changed only when a
    component both know differs; merged keeps what ``new`` lacks from ``old`` (a transient amd-smi miss) and
    takes the rest from ``new``."""
    if not new:
        return False, old
    if not old:
        return False, new
    op, np = epoch_parts(old), epoch_parts(new)
    changed = any(op[k] != np[k] for k in op.keys() & np.keys())
    return changed, epoch_str(dict(op, **np)) if not changed else new


def clean_run(res: Dict[str, Any], fractions: Optional[Dict[str, float]] = None) -> bool:
    """A result that may enter its GPU's baseline (module docstring): judged on its own numbers."""
    fr = _fractions(res) if fractions is None else fractions
    return bool(fr) and not res.get("numerics") and not res.get("lag") and min(fr.values()) >= FAIL_FRACTION


class Baselines:
    def __init__(self, path: Optional[str] = None, runs: int = BASELINE_RUNS, drift_ratio: float = DRIFT_RATIO):
        if runs < 1:
            raise ValueError("runs must be >= 1")
        self.path = path
        self.runs = runs
        self.drift_ratio = drift_ratio
        self.lock = threading.Lock()
        #: gpu key -> {"epoch": str | None, "tests": {shape key: entry}, ["previous": {...}]}
        self.data: Dict[str, Dict[str, Any]] = {}
        if path:
            self._load()

    def _load(self) -> None:
        try:
            with open(self.path, encoding="utf-8") as f:  # type: ignore[arg-type]
                doc = json.load(f)
        except (OSError, ValueError, RecursionError):
            return
        if not isinstance(doc, dict) or not isinstance(doc.get("gpus"), dict):
            return
        if doc.get("schema") in (SCHEMA, SCHEMA_V2):
            for k, v in doc["gpus"].items():
                if isinstance(v, dict) and isinstance(v.get("tests"), dict):
                    ep = v.get("epoch")
                    # an entry without the revision it formed under (v2) cannot be trusted: it re-forms
                    tests = {t: e for t, e in v["tests"].items() if isinstance(e, dict) and isinstance(e.get("rev"), str)}
                    self.data[k] = dict(v, epoch=ep if isinstance(ep, str) else None, tests=tests)
        # a v1 file (before epochs and revisions) is dropped as a whole: its baselines re-form from the next runs

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

    def _tests(self, gpu: str) -> Dict[str, Any]:
        per = self.data.get(gpu)
        return per["tests"] if isinstance(per, dict) and isinstance(per.get("tests"), dict) else {}

    def baseline(self, gpu: str, test: str, res: Dict[str, Any]) -> Optional[Dict[str, float]]:
        entry = self._tests(gpu).get(_shape(test, res))
        return dict(entry["baseline"]) if isinstance(entry, dict) and isinstance(entry.get("baseline"), dict) else None

    def epoch(self, gpu: str) -> Optional[str]:
        per = self.data.get(gpu)
        return per.get("epoch") if isinstance(per, dict) else None

    def drop(self, gpus: Optional[Iterable[str]] = None) -> List[str]:
        """Forget the baselines of ``gpus`` (keys, or a GPU's UUID / PCI address / ``hip:N`` spelled without its
        ``uuid:`` / ``bdf:`` prefix), or of every GPU when None.  Returns the keys dropped; each re-forms from its
        next clean runs."""
        with self.lock:
            if gpus is None:
                gone = sorted(self.data)
            else:
                want = {str(g).strip().lower() for g in gpus if str(g).strip()}
                gone = sorted(k for k in self.data if k.lower() in want or k.split(":", 1)[-1].lower() in want)
            for k in gone:
                del self.data[k]
            if gone:
                self._save()
        return gone

    def observe(self, gpu: str, results: Dict[str, Dict[str, Any]], now: Optional[float] = None,
                epoch: Optional[str] = None, revision: Optional[Callable[[str], str]] = None) -> List[str]:
        """Fold one fresh diagnostic result of GPU ``gpu`` (test -> result), measured under ``epoch``, in: set
        ``drift`` on each rate test below ``drift_ratio`` of its baseline (``baseline`` records the ratios), or
        add the clean ones to the baseline still forming.  A new epoch first re-forms the GPU's baselines, a test
        whose ``revision`` (default ``ops/diag.rate_revision``) changed re-forms its own.  Returns the drift notes.
        Call once per fresh result: the judgement is re-applied from the recorded fields, so cached results keep
        their notes without being observed again."""
        if revision is None:
            from ..ops.diag import rate_revision as revision  # ctypes-free at import
        notes: List[str] = []
        now = time.time() if now is None else now
        changed = False
        with self.lock:
            per = self.data.get(gpu)
            if not isinstance(per, dict) or not isinstance(per.get("tests"), dict):
                per = self.data[gpu] = {"epoch": epoch, "tests": {}}
                changed = True
            else:
                moved, merged = epoch_change(per.get("epoch"), epoch)
                if moved:
                    formed = {t: e["baseline"] for t, e in per["tests"].items()
                              if isinstance(e, dict) and isinstance(e.get("baseline"), dict)}
                    per = self.data[gpu] = {"epoch": epoch, "tests": {},
                                            "previous": {"epoch": per.get("epoch"), "until": round(now, 1),
                                                         "baselines": formed}}
                    changed = True
                elif merged != per.get("epoch"):
                    per["epoch"] = merged  # a component seen for the first time: filled in, nothing re-forms
                    changed = True
            tests = per["tests"]
            for test, res in results.items():
                if not isinstance(res, dict):
                    continue
                fr = _fractions(res)
                if not fr:
                    continue
                key = _shape(test, res)
                rev = revision(test)
                entry = tests.get(key)
                if isinstance(entry, dict) and entry.get("rev") != rev:
                    # the kernel or the references this test's fractions are relative to changed: its baseline says
                    # nothing about today's fractions, so it re-forms (no drift in between)
                    entry = None
                if not isinstance(entry, dict):
                    entry = tests[key] = {"samples": [], "rev": rev}
                    changed = True
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
                res.pop("drift", None)
                if clean_run(res, fr):
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
