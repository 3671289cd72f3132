"""GPU extended-resource registry and quantity parsing.

The registry order is part of the output contract: ``gpu_breakdown`` keys are
emitted in this order in the JSON report, the text table and the Slack text
(reference ``check-gpu-node.py:39-44``, iterated at ``:186``).

MI355X-first: ``amd.com/gpu`` (the ROCm Kubernetes device plugin) is the
*primary* key -- it is the one the MI355X health gate looks at -- but the list
order is kept as in the reference so that breakdowns stay byte-identical.
"""

from __future__ import annotations

from _collections_abc import Mapping  # collections.abc.Mapping; loaded by os, unlike collections
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Dict, Iterable, Optional, Tuple

NVIDIA_GPU = "nvidia.com/gpu"
AMD_GPU = "amd.com/gpu"
INTEL_I915 = "gpu.intel.com/i915"
INTEL_GPU = "intel.com/gpu"

#: Output order of ``gpu_breakdown`` (byte parity with the reference).
GPU_RESOURCE_KEYS: Tuple[str, ...] = (NVIDIA_GPU, AMD_GPU, INTEL_I915, INTEL_GPU)

#: The key the MI355X health gate is centred on.
PRIMARY_GPU_KEY = AMD_GPU


def quantity_text(value: Any) -> Optional[str]:
    """Render a raw JSON capacity value the way the Kubernetes client does.

    The upstream client models ``status.capacity`` as ``dict(str, str)``: a
    JSON ``null`` stays ``None`` and every other scalar goes through ``str()``
    (so the number ``0`` becomes ``"0"`` and ``true`` becomes ``"True"``).
    """
    if value is None:
        return None
    if isinstance(value, str):
        return value
    return str(value)


def parse_gpu_quantity(value: Any) -> Optional[int]:
    """Bug-compatible quantity parse (reference ``:187-195``).

    * missing / ``None`` / empty string -> ``None`` (skipped, ``:188``)
    * ``"0"`` -> ``0`` (kept: zeros appear in the breakdown)
    * anything ``int()`` rejects (``"1k"``, ``"500m"``, ``"8.0"``) -> ``None``
      (silently dropped, ``:193-195``)
    * ``int()`` semantics are Python's: surrounding whitespace, a sign,
      leading zeros and ``_`` digit separators are accepted.
    """
    text = quantity_text(value)
    if not text:
        return None
    try:
        return int(text)
    except (ValueError, TypeError):
        return None


def gpu_breakdown(capacity: Optional[Mapping[str, Any]],
                  keys: Iterable[str] = GPU_RESOURCE_KEYS) -> Dict[str, int]:
    """Per-key GPU counts in registry order (reference ``gpu_capacity``, ``:181-196``)."""
    caps: Dict[str, int] = {}
    if not capacity or not isinstance(capacity, Mapping):
        return caps
    for key in keys:
        n = parse_gpu_quantity(capacity.get(key))
        if n is not None:
            caps[key] = n
    return caps
