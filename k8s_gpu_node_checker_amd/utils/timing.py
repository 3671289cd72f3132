"""Per-phase wall-clock tracer (SURVEY §5 "Tracing / profiling": the reference has none).

Phases used by the checker: ``config``, ``list`` (network + server), and within it
``connect`` (TCP + TLS), ``first_byte`` (request sent to response head), ``body``
(the rest of the response) and ``parse`` (NodeList scan); ``health``, ``slack``,
``render``, ``total``.  Shown with ``--trace`` on stderr and, with ``--json-extended``,
as ``timings_ms`` in the payload; the default JSON is never touched.
"""

from __future__ import annotations

import time

TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Dict


class Tracer:
    #: records anything (the transport skips its per-request spans for a :class:`NullTracer`)
    live = True

    def __init__(self) -> None:
        self.spans: Dict[str, float] = {}
        self.t0 = time.perf_counter()

    def add(self, name: str, seconds: float) -> None:
        self.spans[name] = self.spans.get(name, 0.0) + seconds

    def span(self, name: str) -> "_Span":
        """``with tracer.span("list"): ...`` adds the block's wall time to ``name``."""
        return _Span(self, name)

    def finish(self) -> None:
        self.spans["total"] = time.perf_counter() - self.t0

    def as_ms(self) -> Dict[str, float]:
        return {k: round(v * 1e3, 3) for k, v in self.spans.items()}

    def format(self) -> str:
        return " ".join(f"{k}={v:.3f}ms" for k, v in self.as_ms().items())


class _Span:
    """Context manager of :meth:`Tracer.span` (a class, not ``contextlib``: one import less)."""

    __slots__ = ("tracer", "name", "t")

    def __init__(self, tracer: Tracer, name: str) -> None:
        self.tracer, self.name = tracer, name

    def __enter__(self) -> None:
        self.t = time.perf_counter()

    def __exit__(self, *exc: object) -> None:
        self.tracer.add(self.name, time.perf_counter() - self.t)


class NullTracer(Tracer):
    live = False

    def add(self, name: str, seconds: float) -> None:
        pass
