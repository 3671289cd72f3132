"""Error types whose ``str()`` matches what the reference prints in ``{"error": ...}``.

The reference surfaces whatever the ``kubernetes`` client raised through
``str(e)`` (``check-gpu-node.py:322-325``).  The two families a user sees are
reproduced here with the same text shape:

* ``ConfigException`` -- ``"Invalid kube-config file. No configuration found."``
  and friends (kubernetes ``config_exception.py``).
* ``ApiException`` -- ``"({status})\\nReason: {reason}\\n"`` followed by the
  response headers and body (kubernetes ``exceptions.py``).
"""

from __future__ import annotations

TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Mapping, Optional


class ConfigException(Exception):
    pass


class ApiException(Exception):
    def __init__(self, status: int = 0, reason: str = "", headers: Optional[Mapping[str, str]] = None,
                 body: Optional[str] = None):
        self.status = status
        self.reason = reason
        self.headers = dict(headers) if headers else None
        self.body = body
        super().__init__(str(self))

    def __str__(self) -> str:
        msg = "({0})\nReason: {1}\n".format(self.status, self.reason)
        if self.headers:
            msg += "HTTP response headers: HTTPHeaderDict({0})\n".format(self.headers)
        if self.body:
            msg += "HTTP response body: {0}\n".format(self.body)
        return msg


class TransportError(Exception):
    """Connection-level failure (refused, reset, DNS, TLS, timeout).

    Its message follows urllib3's ``MaxRetryError`` shape, which is what the
    reference's client would have raised:
    ``HTTPSConnectionPool(host='h', port=443): Max retries exceeded with url: /api/v1/nodes (Caused by ...)``.
    """

    def __init__(self, scheme: str, host: str, port: int, url: str, cause: BaseException):
        self.cause = cause
        pool = "HTTPSConnectionPool" if scheme == "https" else "HTTPConnectionPool"
        text = str(cause)
        if text.startswith(("HTTPConnectionPool(host=", "HTTPSConnectionPool(host=")) and \
                ": Max retries exceeded with url: " in text:
            # the transport already rendered the urllib3 message (utils/http.py: refused, DNS, connect timeout, TLS,
            # a proxy's failure -- whose pool may be the proxy's)
            super().__init__(text)
            return
        super().__init__(f"{pool}(host='{host}', port={port}): Max retries exceeded with url: {url} "
                         f"(Caused by {type(cause).__name__}({text!r}))")
