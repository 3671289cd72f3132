"""Bounded, jittered exponential backoff with ``Retry-After`` support (SURVEY §5 "Elastic recovery").

The reference retries Slack 5xx instantly and never retries the kube LIST
(``check-gpu-node.py:83-84``, ``:217``).  Both transports here share this
policy: ``delay_n = min(cap, base * 2**n) * U(1 - jitter, 1)`` unless the
server sent ``Retry-After`` (seconds or an HTTP date), which wins (capped).
"""

from __future__ import annotations

import time
TYPE_CHECKING = False
if TYPE_CHECKING:  # `random` costs a few ms of import time; only a real backoff needs it (typing too)
    import random
    from typing import Optional


class Backoff:
    def __init__(self, base: float = 0.25, cap: float = 30.0, jitter: float = 0.5,
                 rng: "Optional[random.Random]" = None):
        self.base = max(0.0, base)
        self.cap = max(0.0, cap)
        self.jitter = min(max(jitter, 0.0), 1.0)
        self._rng = rng  # seeded lazily: os.urandom seeding costs ~30 us and most checks never back off

    @property
    def rng(self) -> "random.Random":
        if self._rng is None:
            import random
            self._rng = random.Random()
        return self._rng

    def delay(self, attempt: int, retry_after: Optional[str] = None) -> float:
        ra = parse_retry_after(retry_after)
        if ra is not None:
            return min(ra, self.cap)
        raw = min(self.cap, self.base * (2 ** max(0, attempt)))
        if self.jitter:
            raw *= 1.0 - self.jitter * self.rng.random()
        return raw


def parse_retry_after(value: Optional[str], now: Optional[float] = None) -> Optional[float]:
    if not value:
        return None
    value = value.strip()
    try:
        return max(0.0, float(value))
    except ValueError:
        pass
    try:
        from email.utils import parsedate_to_datetime
        dt = parsedate_to_datetime(value)
    except (TypeError, ValueError, IndexError):
        return None
    if dt is None:
        return None
    return max(0.0, dt.timestamp() - (time.time() if now is None else now))
