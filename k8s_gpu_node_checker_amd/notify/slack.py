"""Slack incoming-webhook notifier.

Contract kept from the reference (``check-gpu-node.py:47-157``):

* URL = ``--slack-webhook`` or ``$SLACK_WEBHOOK_URL`` (``or``: an empty flag
  falls back to the env var, ``:144``)
* gating: no URL -> no send; ``--slack-only-on-error`` -> send iff there is
  no Ready GPU node; otherwise always (``:147-157``).  Errors before the scan
  (kubeconfig, API) never reach Slack (``:319-327``).
* body ``{"text", "username", "icon_emoji": ":robot_face:"}`` as
  ``json.dumps`` default (ASCII-escaped, ``", "`` separators) with
  ``Content-Type: application/json``; 10 s timeout per attempt; HTTP 200 is
  the only success; ``--slack-retry-count N`` means N+1 attempts.
* the same stderr lines per attempt (Appendix A.6).

Retry policies (``--slack-retry-policy``):

``reference``  exactly the reference: non-200 retried immediately, reset /
               aborted connections retried after ``retry_delay``, everything
               else (refused, DNS, read timeout) gives up.
``backoff``    (default) the same attempt budget and messages, but 429 / 5xx
               wait a jittered exponential backoff (1 s base, capped at
               ``retry_delay``, ``Retry-After`` honoured) instead of
               hammering the endpoint, and permanent 4xx answers
               (400/403/404/410 -- bad payload, revoked or archived webhook)
               stop immediately.  Divergence documented in ``PARITY.md``.
"""

from __future__ import annotations

import os
import sys
import time
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Callable, Optional, TextIO

from ..utils.backoff import Backoff
from ..utils.http import HTTPError

ICON = ":robot_face:"
DEFAULT_USERNAME = "k8s-gpu-checker"
_BACKOFF_STATUS = frozenset((408, 425, 429, 500, 502, 503, 504))


def get_slack_webhook_url(flag_value: Optional[str]) -> Optional[str]:
    return flag_value or os.environ.get("SLACK_WEBHOOK_URL")


def should_send(url: Optional[str], only_on_error: bool, ready_count: int) -> bool:
    if not url:
        return False
    if only_on_error:
        return ready_count == 0
    return True


def slack_payload(message: str, username: str) -> bytes:
    import json
    return json.dumps({"text": message, "username": username, "icon_emoji": ICON}).encode("ascii")


def send_slack_message(webhook_url: Optional[str], message: str, username: str = DEFAULT_USERNAME,
                       max_retries: int = 3, retry_delay: float = 30, *, policy: str = "backoff",
                       timeout: float = 10.0, err: Optional[TextIO] = None,
                       sleep: Callable[[float], Any] = time.sleep, backoff: Optional[Backoff] = None,
                       ssl_context=None) -> bool:
    """POST ``message`` to the webhook; ``True`` iff some attempt got HTTP 200."""
    if not webhook_url:
        return False
    err = err if err is not None else sys.stderr
    body = slack_payload(message, username)
    bo = backoff or Backoff(base=1.0, cap=max(0.0, float(retry_delay)), jitter=0.5)
    attempts = max_retries + 1
    from . import webhook
    for attempt in range(attempts):
        # requests.post semantics (notify/webhook.py): URL preparation, .netrc / URL credentials, redirects,
        # the environment's proxy and CA bundle -- every failure of any of it inside this attempt's try, as
        # the reference's requests.post call is (check-gpu-node.py:72-109)
        try:
            resp = webhook.post(webhook_url, body, timeout=timeout, ssl_context=ssl_context)
        except HTTPError as e:
            # requests' ConnectionError / Timeout: retried only when the text names a reset or an aborted
            # connection (the reference's test, :88).  A body cut short after the head ("incomplete": requests'
            # ChunkedEncodingError, a RequestException) is not one of those, whatever its text names (:101-104)
            if e.kind not in ("invalid_url", "incomplete") and (
                    "Connection reset by peer" in str(e) or "Connection aborted" in str(e)):
                if attempt < max_retries:
                    print(f"슬랙 메시지 전송 실패 ({attempt + 1}/{attempts}회 시도): {e}", file=err)
                    print(f"⏳ {retry_delay}초 후 재시도합니다...", file=err)
                    sleep(retry_delay)
                    continue
                print(f"슬랙 메시지 전송 최종 실패: {e}", file=err)
                return False
            print(f"슬랙 메시지 전송 실패: {e}", file=err)
            return False
        except Exception as e:  # malformed URL, unexpected protocol errors (reference :106-109)
            print(f"슬랙 메시지 전송 실패: {e}", file=err)
            return False
        if resp.status == 200:
            if attempt > 0:
                print(f"✅ 슬랙 메시지를 {attempt + 1}번째 시도에서 성공적으로 전송했습니다.", file=err)
            return True
        print(f"슬랙 메시지 전송 실패 (HTTP {resp.status}): {webhook.response_text(resp)}", file=err)
        if policy == "backoff" and attempt < max_retries:
            if resp.status in _BACKOFF_STATUS:
                sleep(bo.delay(attempt, resp.header("Retry-After")))
            elif 400 <= resp.status < 500:
                return False
    return False
