"""Alert de-duplication state (SURVEY §5 "Checkpoint / resume": the reference is stateless).

Under cron (reference ``README.md:188-189``) every failing run re-alerts and a
recovery is never announced.  With ``--state-file PATH --slack-on-change`` the
checker remembers the previous outcome and only notifies when it changes:

* a different exit code or a different set of (node, ready) pairs -> send;
* with ``--slack-only-on-error``: send on a change *into* an error state, and
  once more on the recovery back to exit 0;
* with ``--slack-only-on-error --slack-on-node-change``: also send when the set of
  not-Ready GPU nodes changes while the exit code stays 0 (1 of 8 MI355X nodes turning
  unhealthy, and its recovery) -- the reference's "zero Ready nodes" rule
  (``check-gpu-node.py:154-155``) alone never reports a single node -- and when a node
  leaves the GPU-node set altogether (:func:`left_gpu_set`);
* a notification that was due but not delivered (the webhook failed on every
  attempt) stays due: the next run sends it, so an alert is not lost to a
  Slack outage.

Without ``--slack-on-change`` the file is still written (last outcome, for
dashboards) and Slack behaves exactly like the reference.
"""

from __future__ import annotations

import hashlib
import json
import os
import tempfile
import time
from typing import Any, Dict, Optional


def fingerprint(result: Any) -> str:
    h = hashlib.sha256()
    h.update(str(result.exit_code).encode())
    for n in result.gpu_nodes:
        h.update(f"\0{n['name']}\0{n['ready']}\0{n['gpus']}".encode())
    return h.hexdigest()[:16]


def load(path: str) -> Optional[Dict[str, Any]]:
    """The previous run's state, or None when there is none or it is unreadable; a field of the wrong type (a
    hand-edited or truncated-and-rewritten file) is dropped rather than failing the run."""
    try:
        with open(path, encoding="utf-8") as f:
            doc = json.load(f)
    except (OSError, ValueError, RecursionError):
        return None
    if not isinstance(doc, dict):
        return None
    for k in ("not_ready", "gpu_nodes"):
        if not isinstance(doc.get(k, []), list) or not all(isinstance(n, str) for n in doc.get(k, [])):
            doc.pop(k, None)
    for k in ("exit_code", "runs"):
        if not isinstance(doc.get(k, 0), int) or isinstance(doc.get(k), bool):
            doc.pop(k, None)
    if "gpu_sketch" in doc and sketch_members(doc["gpu_sketch"]) is None:
        doc.pop("gpu_sketch")
    if not isinstance(doc.get("not_ready_digest", ""), str):
        doc.pop("not_ready_digest")
    return doc


def members(result: Any) -> list:
    """Names of the GPU-node set, sorted."""
    return sorted(n["name"] for n in result.gpu_nodes)


def members_digest(names: list) -> str:
    h = hashlib.sha256()
    for n in names:
        h.update(n.encode("utf-8", "surrogatepass") + b"\0")
    return h.hexdigest()[:16]


def outcome(result: Any) -> Dict[str, Any]:
    """What the next evaluation's :func:`should_notify` compares against (state file, watcher memo)."""
    names = members(result)
    return {"fingerprint": fingerprint(result), "exit_code": result.exit_code,
            "slack_pending": result.slack_sent is False, "not_ready": not_ready(result),
            "gpu_nodes": names, "gpu_count": len(names), "members": members_digest(names)}


#: what a published outcome (the watcher's Lease annotation, ``kube/lease.STATE_MAX_BYTES``) may take as JSON
STATE_MAX_BYTES = 64 << 10


def name_hash(name: str, width: int) -> bytes:
    """The first ``width`` bytes of a node name's SHA-256 (a member of the compacted set's sketch)."""
    return hashlib.sha256(name.encode("utf-8", "surrogatepass")).digest()[:width]


def sketch(names: list, width: int) -> str:
    """The member set as sorted ``width``-byte name hashes, base64: ``width`` x 4/3 bytes a member instead of the
    name, and still able to tell that a previous member is gone when the set also grew (:func:`left_gpu_set`)."""
    import base64
    return f"{width}:" + base64.b64encode(b"".join(sorted({name_hash(n, width) for n in names}))).decode()


def sketch_members(value: Any) -> Optional[tuple]:
    """(width, set of hashes) of a :func:`sketch`, None when it is not one."""
    import base64
    import binascii
    if not isinstance(value, str) or ":" not in value:
        return None
    w, _, b64 = value.partition(":")
    try:
        width, raw = int(w), base64.b64decode(b64, validate=True)
    except (ValueError, binascii.Error):
        return None
    if width not in (4, 8) or len(raw) % width:
        return None
    return width, {raw[i:i + width] for i in range(0, len(raw), width)}


def _size(state: Dict[str, Any]) -> int:
    return len(json.dumps(state, sort_keys=True, separators=(",", ":")))


def compact(state: Dict[str, Any], max_bytes: int = STATE_MAX_BYTES) -> Dict[str, Any]:
    """The outcome shrunk until it fits ``max_bytes`` of JSON (the Lease), losing as little as it can:

    1. as it is;
    2. the member names replaced by an 8-byte hash each (:func:`sketch`; ~6,000 members), then a 4-byte one
       (~12,000) -- a departure is still seen when the set also grew (one node leaves while two join);
    3. no member list (digest and count: a departure hidden by growth is missed);
    4. the not-Ready names replaced by their digest and count (a change of that set is still seen).

    Sized by serialized bytes, not by count: 1,000 real node names (40-70 characters) alone exceed 64 KiB."""
    if _size(state) <= max_bytes:
        return state
    base = {k: v for k, v in state.items() if k != "gpu_nodes"}
    names = state.get("gpu_nodes") if isinstance(state.get("gpu_nodes"), list) else None
    if names is not None:
        for width in (8, 4):
            s = dict(base, gpu_sketch=sketch(names, width))
            if _size(s) <= max_bytes:
                return s
    if _size(base) <= max_bytes:
        return base
    nr = base.get("not_ready")
    if isinstance(nr, list):
        base = {k: v for k, v in base.items() if k != "not_ready"}
        base.update(not_ready_digest=members_digest(sorted(nr)), not_ready_count=len(nr))
    return base


def save(path: str, result: Any, prev: Optional[Dict[str, Any]] = None) -> None:
    doc = {
        "version": 1,
        "ts": time.time(),
        "exit_code": result.exit_code,
        "fingerprint": fingerprint(result),
        "total_nodes": len(result.gpu_nodes),
        "ready_nodes": len(result.ready_gpu_nodes),
        "not_ready": not_ready(result),
        "slack_sent": result.slack_sent,
        # sent and failed (None: nothing was due): the next run's gate sends again
        "slack_pending": result.slack_sent is False,
        "runs": (prev or {}).get("runs", 0) + 1,
    }
    doc.update({k: v for k, v in outcome(result).items() if k in ("gpu_nodes", "gpu_count", "members")})
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".state-", dir=d)
    with os.fdopen(fd, "w", encoding="utf-8") as f:
        json.dump(doc, f, ensure_ascii=False, indent=2)
    os.replace(tmp, path)


def not_ready(result: Any) -> list:
    return sorted(n["name"] for n in result.gpu_nodes if not n["ready"])


def should_notify(prev: Optional[Dict[str, Any]], result: Any, only_on_error: bool,
                  on_node_change: bool = False) -> bool:
    fp = fingerprint(result)
    if prev is not None and prev.get("slack_pending"):
        return True  # the last notification never arrived
    if prev is not None and prev.get("fingerprint") == fp:
        return False
    if not only_on_error:
        return True
    if result.exit_code != 0:
        return True
    if prev is not None and prev.get("exit_code", 0) != 0:
        return True  # recovery
    if on_node_change:
        now = not_ready(result)
        if prev is not None and isinstance(prev.get("not_ready_digest"), str) and "not_ready" not in prev:
            if members_digest(now) != prev["not_ready_digest"]:  # compacted: the names are gone, the digest is not
                return True
        elif now != (sorted(prev.get("not_ready") or []) if prev is not None else []):
            return True  # a node went down (or came back) while others stay Ready
        return left_gpu_set(prev, result)
    return False


def left_gpu_set(prev: Optional[Dict[str, Any]], result: Any) -> bool:
    """A node of the previous GPU-node set is gone from this one (deleted, relabelled, or -- counting
    capacity -- its device plugin deregistered the GPUs): nothing of it is Not Ready any more, it is
    simply absent, and only this comparison notices.  A state from before the member list was kept
    (no ``gpu_nodes``/``members``) says nothing."""
    if prev is None:
        return False
    names = prev.get("gpu_nodes")
    if isinstance(names, list):
        now = {n["name"] for n in result.gpu_nodes}
        return any(n not in now for n in names)
    sk = sketch_members(prev.get("gpu_sketch"))
    if sk is not None:
        # compacted to name hashes: a previous member whose hash no current name has is gone (a departed node whose
        # hash collides with a current node's is missed: 1 in 2^64 / 2^32 per name)
        width, before = sk
        return bool(before - {name_hash(n["name"], width) for n in result.gpu_nodes})
    digest, count = prev.get("members"), prev.get("gpu_count")
    if isinstance(digest, str) and isinstance(count, int) and not isinstance(count, bool):
        # names not kept (a large fleet's compacted Lease state): a different set that did not grow lost a node
        cur = members(result)
        return members_digest(cur) != digest and len(cur) <= count
    return False


def gate_webhook(prev: Optional[Dict[str, Any]], opts: Any, cluster: Any, on_node_change: bool = False) -> Optional[str]:
    """Install a de-dup gate on ``opts``; returns the (unchanged) webhook flag value."""
    only = opts.slack_only_on_error

    def gate(result: Any) -> bool:
        return should_notify(prev, result, only, on_node_change)

    opts.slack_gate = gate
    if only:
        # the gate decides (recoveries must be able to send although Ready > 0)
        opts.slack_only_on_error = False
    return opts.slack_webhook
