"""``auth-provider: gcp`` with a ``cmd-path``: the legacy GKE credential helper (``gcloud config config-helper``).

The reference reaches GKE through ``kubernetes.config.load_kube_config`` (``/root/reference/check-gpu-node.py:160-169``),
whose gcp provider refreshes an expired ``access-token`` with ``google.auth.default()`` -- a library and a metadata /
OAuth round trip this package does not carry (parity unpinned: neither ``kubernetes`` nor ``google-auth`` is
importable here, PARITY.md #19).  What it does carry is client-go's own refresh for the same kubeconfig stanza, the one
``kubectl`` used before the exec plugin: when the cached token has expired and the stanza names a ``cmd-path``, run
``cmd-path cmd-args``, read the token and its expiry from the command's JSON output at ``token-key`` /
``expiry-key`` (``{.access_token}`` / ``{.token_expiry}`` by default; gcloud's stanza says
``{.credential.access_token}``), and use it until it expires.  Without a ``cmd-path`` the stored token is sent as it
is, expired or not (the apiserver's 401 then says so).  The refreshed token is kept in memory, not written back.
"""

from __future__ import annotations

import json
import shlex
import subprocess
import time
from datetime import datetime, timezone
from typing import Any, Dict, Optional

from .errors import ConfigException

# a token this close to its expiry is refreshed first (client-go's gcp plugin uses the same kind of margin)
EXPIRY_MARGIN_S = 10.0


def parse_time(value: Any) -> Optional[float]:
    """RFC 3339 (with or without fractional seconds, ``Z`` or an offset) to Unix seconds; None when absent or
    unparseable."""
    if not isinstance(value, str) or not value.strip():
        return None
    s = value.strip().replace("Z", "+00:00").replace("z", "+00:00")
    date, sep, rest = s.partition("T")
    if "." in rest:  # Python 3.10's fromisoformat takes at most 6 fractional digits
        whole, _, tail = rest.partition(".")
        digits = "".join(c for c in tail if c.isdigit())
        rest = f"{whole}.{digits[:6].ljust(6, '0')}{tail[len(digits):]}"
    try:
        dt = datetime.fromisoformat(date + sep + rest)
    except ValueError:
        return None
    if dt.tzinfo is None:
        dt = dt.replace(tzinfo=timezone.utc)
    return dt.timestamp()


def json_path(doc: Any, path: str) -> Any:
    """The value at a client-go JSONPath of the simple form ``{.a.b.c}`` (what the gcp stanza's keys use)."""
    p = path.strip()
    if p.startswith("{") and p.endswith("}"):
        p = p[1:-1]
    cur = doc
    for part in (x for x in p.split(".") if x):
        if not isinstance(cur, dict) or part not in cur:
            return None
        cur = cur[part]
    return cur


class GcpCmdProvider:
    def __init__(self, cfg: Dict[str, Any], run: Any = None):
        self.access_token = cfg.get("access-token") if isinstance(cfg.get("access-token"), str) else None
        self.expiry = parse_time(cfg.get("expiry"))
        self.cmd = cfg.get("cmd-path") if isinstance(cfg.get("cmd-path"), str) and cfg.get("cmd-path") else None
        self.args = shlex.split(cfg.get("cmd-args") or "") if isinstance(cfg.get("cmd-args", ""), str) else []
        self.token_key = cfg.get("token-key") or "{.access_token}"
        self.expiry_key = cfg.get("expiry-key") or "{.token_expiry}"
        self._run = run or subprocess.run

    def _fresh(self) -> bool:
        return bool(self.access_token) and (self.expiry is None or self.expiry > time.time() + EXPIRY_MARGIN_S)

    def token(self) -> Optional[str]:
        if self._fresh() or not self.cmd:
            return self.access_token
        try:
            p = self._run([self.cmd, *self.args], capture_output=True, text=True, timeout=60)
        except (OSError, subprocess.SubprocessError) as e:
            raise ConfigException(f"gcp auth-provider: cmd-path {self.cmd!r} failed: {e}")
        if p.returncode != 0:
            raise ConfigException(f"gcp auth-provider: cmd-path {self.cmd!r} exited {p.returncode}: "
                                  f"{(p.stderr or '').strip()[:200]}")
        try:
            doc = json.loads(p.stdout)
        except ValueError:
            raise ConfigException(f"gcp auth-provider: cmd-path {self.cmd!r} did not print JSON")
        tok = json_path(doc, self.token_key)
        if not isinstance(tok, str) or not tok:
            raise ConfigException(f"gcp auth-provider: no token at {self.token_key} in the output of {self.cmd!r}")
        self.access_token = tok
        self.expiry = parse_time(json_path(doc, self.expiry_key))
        return tok

    def invalidate(self) -> bool:
        """After a 401: the next :meth:`token` runs the command again (False when there is none to run)."""
        if not self.cmd:
            return False
        self.expiry = 0.0
        return True
