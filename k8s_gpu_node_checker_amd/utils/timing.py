"""Per-phase wall-clock tracer (SURVEY §5 "Tracing / profiling": the reference has none).

Phases used by the checker: ``config``, ``list`` (network + server), ``parse``
(NodeList scan, a sub-span of ``list``), ``health``, ``slack``, ``render``,
``total``.  Shown with ``--trace`` on stderr and, with ``--json-extended``,
as ``timings_ms`` in the payload; the default JSON is never touched.
"""

from __future__ import annotations

import time
from contextlib import contextmanager
from typing import Dict, Iterator


class Tracer:
    def __init__(self) -> None:
        self.spans: Dict[str, float] = {}
        self.t0 = time.perf_counter()

    def add(self, name: str, seconds: float) -> None:
        self.spans[name] = self.spans.get(name, 0.0) + seconds

    @contextmanager
    def span(self, name: str) -> Iterator[None]:
        t = time.perf_counter()
        try:
            yield
        finally:
            self.add(name, time.perf_counter() - t)

    def finish(self) -> None:
        self.spans["total"] = time.perf_counter() - self.t0

    def as_ms(self) -> Dict[str, float]:
        return {k: round(v * 1e3, 3) for k, v in self.spans.items()}

    def format(self) -> str:
        return " ".join(f"{k}={v:.3f}ms" for k, v in self.as_ms().items())


class NullTracer(Tracer):
    def add(self, name: str, seconds: float) -> None:
        pass
