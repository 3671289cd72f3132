"""CPU hot path: decode a ``NodeList`` page and render the JSON report.

Two implementations with identical results:

* native (``_native/_fastpath*.so``, ``csrc/fastpath/fastpath.cpp``): a
  single-pass JSON scanner that materialises only the fields the checker
  consumes (name, labels, capacity/allocatable GPU keys, Ready condition,
  taints, the health annotation, ``metadata.continue``) and skips images,
  managedFields, nodeInfo, addresses, ... without building Python objects for
  them; plus a byte-exact ``json.dumps(ensure_ascii=False, indent=2)``
  emitter for the report schema.
* pure Python (``json.loads`` + :func:`models.node.scan_items`), used when
  the extension is not built or when the native scanner reports malformed
  input (then the stdlib decoder produces the canonical error).

SURVEY §6 takeaway 2: at 1000 nodes (5.9 MB NodeList) parse + projection is
~90 ms of the reference's check; this is the lever.
"""

from __future__ import annotations

TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Optional, Sequence, Tuple

from ..models.node import HEALTH_ANNOTATION, HEALTH_CONDITION, NodeExtras, ScanResult, scan_items
from ..models.resources import GPU_RESOURCE_KEYS
from .native import load_extension

_ext = None
_ext_loaded = False


def ext():
    global _ext, _ext_loaded
    if not _ext_loaded:
        _ext = load_extension("_fastpath")
        _ext_loaded = True
    return _ext


def loads(data: Any) -> Any:
    """``json.loads(data)``: the native parser when it can prove the result identical, else the json
    package (which then raises exactly what it always raises)."""
    mod = ext()
    if mod is not None:
        try:
            return mod.loads(data)
        except mod.FallbackError:
            pass
    import json
    return json.loads(data)


def backend() -> str:
    return "native" if ext() is not None else "python"


def prescan(body: bytes, keys: Sequence[str] = GPU_RESOURCE_KEYS) -> Optional[Tuple[tuple, Any]]:
    """Pass 1 of the native scan (GIL released), for a thread that has just received ``body``.

    Hand the result to :func:`scan_page` (``pre=``) with the same ``keys``; ``None`` when the
    extension is missing.
    """
    mod = ext()
    if mod is None:
        return None
    keys = tuple(keys)
    return keys, mod.prescan_nodelist(body, keys, HEALTH_ANNOTATION, HEALTH_CONDITION)


def scan_page(body: bytes, result: ScanResult, keys: Sequence[str] = GPU_RESOURCE_KEYS,
              gpu_source: str = "capacity", want_extras: bool = False,
              annotation_mode: int = 2, pre: Optional[Tuple[tuple, Any]] = None) -> Tuple[Optional[str], int]:
    """Scan one ``NodeList`` page into ``result``.

    Returns ``(continue_token, item_count)``.  Raises ``ValueError`` on a body
    that is not a JSON object (mirrors ``json.loads`` errors).  ``pre`` is
    :func:`prescan` of the same ``body``: only pass 2 is left to do.
    """
    mod = ext()
    if mod is not None:
        if pre is not None and pre[0] == tuple(keys):
            try:
                return mod.scan_prescanned(pre[1], result, pre[0], gpu_source == "allocatable", want_extras,
                                           NodeExtras, annotation_mode)
            except mod.FallbackError:
                return _scan_python(body, result, keys, gpu_source, want_extras, annotation_mode)
        try:
            return mod.scan_nodelist(body, result, tuple(keys), gpu_source == "allocatable",
                                     want_extras, HEALTH_ANNOTATION, NodeExtras, HEALTH_CONDITION,
                                     annotation_mode)
        except mod.FallbackError:
            pass  # unusual shape: let the reference-semantics Python path decide
    return _scan_python(body, result, keys, gpu_source, want_extras, annotation_mode)


def _scan_python(body: bytes, result: ScanResult, keys: Sequence[str], gpu_source: str, want_extras: bool,
                 annotation_mode: int) -> Tuple[Optional[str], int]:
    import json
    doc = json.loads(body)
    if not isinstance(doc, dict):
        raise ValueError("NodeList response is not a JSON object")
    items = doc.get("items") or []
    before = result.items_seen
    scan_items(items, result, keys, gpu_source, want_extras, annotation_mode)
    meta = doc.get("metadata") or {}
    token = meta.get("continue") if isinstance(meta, dict) else None
    return (token or None), result.items_seen - before


def dumps_indent2(payload: Any) -> str:
    """``json.dumps(payload, ensure_ascii=False, indent=2)`` -- byte-identical."""
    mod = ext()
    if mod is not None:
        try:
            return mod.dumps_indent2(payload)
        except mod.FallbackError:
            pass
    import json
    return json.dumps(payload, ensure_ascii=False, indent=2)
