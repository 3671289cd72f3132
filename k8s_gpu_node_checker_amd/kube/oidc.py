"""``auth-provider: oidc`` credentials with refresh, as the reference gets them from
``kubernetes.config.load_kube_config`` (``check-gpu-node.py:160-169`` -> ``KubeConfigLoader._load_oid_token``
/ ``_refresh_oidc`` of the upstream client).

Upstream semantics kept:

* the bearer token is the provider's ``id-token``; a token that is not a well-formed JWT (URL-unsafe
  ``= + /`` characters, not three parts, impossible padding) is not used at all (no Authorization header);
* a token whose ``exp`` is within 5 minutes is refreshed first: ``GET {idp-issuer-url}/.well-known/
  openid-configuration`` -> ``token_endpoint``, then a ``refresh_token`` grant with ``client-id`` /
  ``client-secret`` (HTTP Basic and in the form body, as requests-oauthlib sends them);
* the new ``id-token`` / ``refresh-token`` are written back into the kubeconfig (upstream's default
  ``persist_config=True``); a discovery document that does not answer 200 leaves the old token in place
  (the apiserver's 401 then ends the check); a token endpoint that refuses the grant is an error.

Beyond upstream:

* a 401 from the apiserver forces one refresh and one retry (``ClusterConnection.invalidate_credentials``),
  the way client-go treats a revoked-but-unexpired token;
* concurrent checkers (several ``--watch`` pods / cron runs sharing a kubeconfig) refresh once: the write
  is done under client-go's ``<kubeconfig>.lock`` (``O_CREAT|O_EXCL``, so ``kubectl config`` interoperates),
  and a process that gets the lock re-reads the file first and adopts a token another process already
  refreshed -- with rotating refresh tokens a second refresh of the same token would be refused;
* the IdP's TLS certificate is verified against ``idp-certificate-authority(-data)`` or, without one, the
  system roots (upstream turns verification off in that case).
"""

from __future__ import annotations

import os
import time

from .errors import ConfigException

TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only
    from typing import Any, Dict, Optional

EXPIRY_SKEW_S = 300.0      # upstream EXPIRY_SKEW_PREVENTION_DELAY
LOCK_WAIT_S = 10.0
LOCK_STALE_S = 60.0        # a lock file older than this was left by a crashed writer


def jwt_expiry(token: str) -> "Optional[float]":
    """``exp`` of a JWT, or None when the token carries none.  Raises ValueError for a token upstream
    refuses to use (see the module docstring)."""
    import base64
    import json
    if any(ch in token for ch in "=+/"):
        raise ValueError("id-token has URL-unsafe characters")
    parts = token.split(".")
    if len(parts) != 3:
        raise ValueError("id-token is not a JWT")
    padding = (4 - len(parts[1]) % 4) * "="
    if len(padding) == 3:
        raise ValueError("id-token has impossible base64 padding")
    claims = json.loads(base64.urlsafe_b64decode(parts[1] + padding).decode("utf-8"))
    exp = claims.get("exp") if isinstance(claims, dict) else None
    return float(exp) if isinstance(exp, (int, float)) and not isinstance(exp, bool) else None


class OidcProvider:
    """The ``config`` mapping of one user's ``auth-provider: {name: oidc}`` and where it came from."""

    def __init__(self, cfg: "Dict[str, Any]", user: str, source: "Optional[str]", base: "Optional[str]" = None):
        self.cfg = cfg
        self.user = user
        self.source = source
        self.base = base
        self._force = False
        self._lock = None

    # -- public ------------------------------------------------------------------------------------
    def token(self) -> "Optional[str]":
        """The id-token to present, refreshed first when it is (about to be) expired or a 401 asked for it."""
        if self._lock is None:
            import threading
            self._lock = threading.Lock()
        with self._lock:
            tok = self.cfg.get("id-token")
            if not isinstance(tok, str):
                return None
            try:
                exp = jwt_expiry(tok)
            except ValueError:
                return None  # upstream: not a usable JWT -> no bearer token
            if self._force or (exp is not None and exp - EXPIRY_SKEW_S <= time.time()):
                self._force = False
                self._refresh(tok)
            tok = self.cfg.get("id-token")
            return tok if isinstance(tok, str) else None

    def invalidate(self) -> bool:
        """After a 401: refresh before the next request (True when a refresh is possible)."""
        if self.cfg.get("refresh-token") and self.cfg.get("idp-issuer-url"):
            self._force = True
            return True
        return False

    # -- refresh -----------------------------------------------------------------------------------
    def _refresh(self, stale: str) -> None:
        with _FileLock(self.source):
            if self._adopt_from_file(stale):
                return
            new = self._grant()
            if new is None:
                return  # discovery unavailable: keep the old token (upstream)
            self.cfg["id-token"] = new["id_token"]
            if new.get("refresh_token"):
                self.cfg["refresh-token"] = new["refresh_token"]
            self._persist()

    def _adopt_from_file(self, stale: str) -> bool:
        """Another process refreshed while we waited for the lock: take its (valid) token."""
        if not self.source or not os.path.exists(self.source):
            return False
        try:
            pcfg = _provider_config(_read(self.source), self.user)
        except Exception:
            return False
        tok = pcfg.get("id-token") if pcfg else None
        if not isinstance(tok, str) or tok == stale:
            return False
        try:
            exp = jwt_expiry(tok)
        except ValueError:
            return False
        if exp is not None and exp - EXPIRY_SKEW_S <= time.time():
            return False
        self.cfg["id-token"] = tok
        if pcfg.get("refresh-token"):
            self.cfg["refresh-token"] = pcfg["refresh-token"]
        return True

    def _ssl_context(self):
        import ssl
        ctx = ssl.create_default_context()
        data = self.cfg.get("idp-certificate-authority-data")
        path = self.cfg.get("idp-certificate-authority")
        if data:
            import base64
            ctx = ssl.create_default_context(cadata=base64.b64decode(str(data)).decode("ascii", "replace"))
        elif path:
            if self.base and not os.path.isabs(path):
                path = os.path.join(self.base, path)
            ctx = ssl.create_default_context(cafile=os.path.expanduser(path))
        return ctx

    def _grant(self) -> "Optional[Dict[str, Any]]":
        import base64
        import json
        from urllib.parse import urlencode

        from ..utils.http import HTTPError, request
        for key in ("idp-issuer-url", "client-id", "refresh-token"):
            if not self.cfg.get(key):
                raise ConfigException("Invalid kube-config file. oidc auth-provider needs %s to refresh an "
                                      "expired id-token" % key)
        issuer = str(self.cfg["idp-issuer-url"]).rstrip("/")
        ctx = self._ssl_context() if issuer.startswith("https:") else None
        try:
            disc = request(issuer + "/.well-known/openid-configuration", headers={"Accept": "application/json"},
                           timeout=10.0, ssl_context=ctx)
        except HTTPError as e:
            raise ConfigException("OIDC discovery at %s failed: %s" % (issuer, e)) from e
        if disc.status != 200:
            return None
        try:
            endpoint = json.loads(disc.body)["token_endpoint"]
        except (ValueError, KeyError, TypeError) as e:
            raise ConfigException("OIDC discovery at %s: no token_endpoint (%s)" % (issuer, e)) from e
        cid, secret = str(self.cfg["client-id"]), str(self.cfg.get("client-secret") or "")
        form = {"grant_type": "refresh_token", "refresh_token": str(self.cfg["refresh-token"]), "client_id": cid}
        if secret:
            form["client_secret"] = secret
        basic = base64.b64encode(f"{cid}:{secret}".encode()).decode()
        ctx = self._ssl_context() if str(endpoint).startswith("https:") else None
        try:
            resp = request(str(endpoint), "POST", headers={
                "Content-Type": "application/x-www-form-urlencoded", "Accept": "application/json",
                "Authorization": "Basic " + basic}, body=urlencode(form).encode(), timeout=10.0, ssl_context=ctx)
        except HTTPError as e:
            raise ConfigException("OIDC token refresh at %s failed: %s" % (endpoint, e)) from e
        try:
            doc = json.loads(resp.body)
        except ValueError:
            doc = {}
        if resp.status != 200 or not isinstance(doc, dict) or not doc.get("id_token"):
            err = doc.get("error") if isinstance(doc, dict) else None
            desc = doc.get("error_description") if isinstance(doc, dict) else None
            raise ConfigException("OIDC token refresh at %s failed: HTTP %d %s%s" % (
                endpoint, resp.status, err or resp.reason, f" ({desc})" if desc else ""))
        return doc

    def _persist(self) -> None:
        """Write the new tokens into the kubeconfig file that defines this user (atomically)."""
        if not self.source or not os.path.exists(self.source):
            return
        raw_doc = _read(self.source)
        pcfg = _provider_config(raw_doc, self.user)
        if pcfg is None:
            return
        pcfg["id-token"] = self.cfg["id-token"]
        if self.cfg.get("refresh-token"):
            pcfg["refresh-token"] = self.cfg["refresh-token"]
        with open(self.source, "rb") as f:
            is_json = f.read().lstrip()[:1] == b"{"
        if is_json:
            import json
            text = json.dumps(raw_doc, indent=2) + "\n"
        else:
            import yaml
            text = yaml.safe_dump(raw_doc, default_flow_style=False, sort_keys=False)
        d = os.path.dirname(os.path.abspath(self.source))
        tmp = os.path.join(d, ".%s.tmp-%d" % (os.path.basename(self.source), os.getpid()))
        mode = os.stat(self.source).st_mode & 0o777
        fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, mode)
        try:
            with os.fdopen(fd, "w", encoding="utf-8") as f:
                f.write(text)
            os.replace(tmp, self.source)
        except BaseException:
            try:
                os.unlink(tmp)
            except OSError:
                pass
            raise


def _read(path: str) -> "Any":
    from .config import _load_yaml
    return _load_yaml(path)


def _provider_config(doc: "Any", user: str) -> "Optional[Dict[str, Any]]":
    users = doc.get("users") if isinstance(doc, dict) else None
    for item in users or []:
        if isinstance(item, dict) and item.get("name") == user:
            prov = (item.get("user") or {}).get("auth-provider")
            if isinstance(prov, dict) and isinstance(prov.get("config"), dict):
                return prov["config"]
    return None


class _FileLock:
    """client-go's kubeconfig write lock: ``<file>.lock`` created with O_EXCL, removed after."""

    def __init__(self, path: "Optional[str]"):
        self.path = (path + ".lock") if path else None
        self.held = False

    def __enter__(self) -> "_FileLock":
        if not self.path:
            return self
        deadline = time.monotonic() + LOCK_WAIT_S
        delay = 0.005
        while True:
            try:
                os.close(os.open(self.path, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o600))
                self.held = True
                return self
            except FileExistsError:
                try:
                    if time.time() - os.stat(self.path).st_mtime > LOCK_STALE_S:
                        os.unlink(self.path)  # left by a crashed writer
                        continue
                except OSError:
                    continue
                if time.monotonic() > deadline:
                    raise ConfigException("kubeconfig is locked (%s exists): another process is writing it"
                                          % self.path)
                time.sleep(delay)
                delay = min(delay * 2, 0.1)
            except OSError:
                return self  # read-only directory: refresh in memory only

    def __exit__(self, *exc: object) -> None:
        if self.held:
            try:
                os.unlink(self.path)  # type: ignore[arg-type]
            except OSError:
                pass
            self.held = False
