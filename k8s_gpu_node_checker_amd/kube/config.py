"""kubeconfig loading and auth resolution (SURVEY R6, §7.2 layer 1).

Replaces ``kubernetes.config.load_kube_config`` (reference
``check-gpu-node.py:160-169``) without the ``kubernetes`` package:

Resolution order (reference semantics, byte-for-byte error texts):

1. ``--kubeconfig PATH`` (a ``:``-separated list is merged, as upstream does)
2. ``$KUBECONFIG`` **if ``os.path.exists`` of the whole value** (``:165-167``)
3. library default: ``$KUBECONFIG`` as a ``:``-list, else ``~/.kube/config``
4. (additive, off unless nothing above yields a config) in-cluster service
   account -- the reference never calls ``load_incluster_config``; using it
   only when no kubeconfig exists keeps every reference outcome identical
   except the one that was an error.

Merging follows the upstream ``KubeConfigMerger``: the first file that parses
provides the top level (``current-context``, ...); ``clusters``, ``contexts``
and ``users`` are merged by ``name``, first occurrence wins.

Auth matrix: bearer ``token`` / ``tokenFile``, ``username``/``password``,
client certificate + key (file or ``*-data``), ``certificate-authority``
(file or data), ``insecure-skip-tls-verify``, ``tls-server-name``,
``proxy-url`` (HTTP CONNECT), ``exec`` credential plugins
(``client.authentication.k8s.io/v1`` and ``v1beta1``) and the legacy
``auth-provider`` (``oidc`` with id-token refresh and write-back, ``kube/oidc.py``; other providers'
``id-token`` / ``access-token`` as static tokens).
"""

from __future__ import annotations

import os
import time
TYPE_CHECKING = False
if TYPE_CHECKING:  # annotations only (PEP 563): importing typing is ~10 ms of a cold start
    from typing import Any, Dict, List, Optional, Tuple

from .errors import ConfigException

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"
_NO_CONFIG = "Invalid kube-config file. No configuration found."


def _default_location() -> str:
    return os.environ.get("KUBECONFIG", os.path.expanduser("~/.kube/config"))


def _load_yaml(path: str) -> Any:
    with open(path, "rb") as f:
        raw = f.read()
    stripped = raw.lstrip()
    if stripped[:1] == b"{":  # JSON kubeconfigs skip the YAML import entirely
        import json
        try:
            return json.loads(raw)
        except ValueError:
            pass
    try:  # the kubeconfig YAML subset, without the ~10 ms PyYAML import
        from ..utils.miniyaml import Unsupported, loads
        try:
            return loads(raw.decode("utf-8"))
        except (Unsupported, UnicodeDecodeError):
            pass
    except ImportError:  # pragma: no cover
        pass
    import yaml  # full YAML (anchors, block scalars, ...)
    loader = getattr(yaml, "CSafeLoader", yaml.SafeLoader)
    return yaml.load(raw, Loader=loader)


def _named(items: Any) -> List[Dict[str, Any]]:
    return [i for i in (items or []) if isinstance(i, dict)]


def merge_kubeconfigs(paths: str) -> Tuple[Optional[Dict[str, Any]], Optional[str]]:
    """Merge a ``:``-separated list of kubeconfig files (first wins).

    Returns ``(config, path_of_first_file)``; ``config`` is ``None`` when no
    file exists or all are empty.
    """
    merged: Optional[Dict[str, Any]] = None
    first: Optional[str] = None
    for path in paths.split(os.pathsep):
        if not path:
            continue
        path = os.path.expanduser(path)
        if not os.path.exists(path):
            continue
        cfg = _load_yaml(path)
        if not cfg:
            continue
        if not isinstance(cfg, dict):
            raise ConfigException("Invalid kube-config file. Expected a mapping in %s" % path)
        base = os.path.dirname(os.path.abspath(path))
        # resolve relative file references against the file that defines them
        for section, inner in (("clusters", "cluster"), ("users", "user")):
            for item in _named(cfg.get(section)):
                body = item.get(inner)
                if isinstance(body, dict):
                    body.setdefault("__base__", base)
                    body.setdefault("__file__", os.path.abspath(path))  # where refreshed tokens go back
        if merged is None:
            merged = cfg
            first = path
            for section in ("clusters", "contexts", "users"):
                merged[section] = _named(cfg.get(section))
            continue
        for section in ("clusters", "contexts", "users"):
            have = {i.get("name") for i in merged[section]}
            for item in _named(cfg.get(section)):
                if item.get("name") not in have:
                    merged[section].append(item)
                    have.add(item.get("name"))
    return merged, first


def _get_named(cfg: Dict[str, Any], section: str, name: str) -> Dict[str, Any]:
    for item in cfg.get(section) or []:
        if isinstance(item, dict) and item.get("name") == name:
            return item
    raise ConfigException("Invalid kube-config file. Expected object with name %s in kube-config/%s list"
                          % (name, section))


def _need(node: Dict[str, Any], key: str, where: str) -> Any:
    if not isinstance(node, dict) or node.get(key) is None:
        raise ConfigException("Invalid kube-config file. Expected key %s in %s" % (key, where))
    return node[key]


class ClusterConnection:
    """Everything needed to talk to one kube-apiserver."""

    def __init__(self, server: str):
        self.server = server.rstrip("/")
        self.ca_file: Optional[str] = None
        self.ca_data: Optional[bytes] = None
        self.insecure = False
        self.tls_server_name: Optional[str] = None
        self.cert_file: Optional[str] = None
        self.key_file: Optional[str] = None
        self.cert_data: Optional[bytes] = None
        self.key_data: Optional[bytes] = None
        self.token: Optional[str] = None
        self.token_file: Optional[str] = None
        self.username: Optional[str] = None
        self.password: Optional[str] = None
        self.exec_spec: Optional[Dict[str, Any]] = None
        self.exec_base: Optional[str] = None
        self.proxy_url: Optional[str] = None
        self.source = "kubeconfig"
        self._exec_cache: Optional[Tuple[Dict[str, Any], float]] = None
        self.oidc = None  # kube/oidc.OidcProvider for `auth-provider: oidc`
        self.gcp = None  # kube/gcp_cmd.GcpCmdProvider for `auth-provider: gcp`
        self._ssl_ctx = None

    # -- auth -----------------------------------------------------------------
    def _run_exec(self) -> Dict[str, Any]:
        if self._exec_cache and (self._exec_cache[1] == 0 or self._exec_cache[1] > time.time() + 10):
            return self._exec_cache[0]
        from .exec_plugin import run_exec_plugin
        status, expiry = run_exec_plugin(self.exec_spec or {}, self.exec_base, self)
        self._exec_cache = (status, expiry)
        return status

    def invalidate_credentials(self) -> bool:
        """Drop cached exec-plugin credentials (after a 401); True if the next request can present
        different credentials (exec plugin re-run or a re-read tokenFile), as client-go does."""
        self._exec_cache = None
        refreshable = (self.oidc is not None and self.oidc.invalidate()) or (
            self.gcp is not None and self.gcp.invalidate())
        return self.exec_spec is not None or bool(self.token_file) or refreshable

    def auth_headers(self) -> Dict[str, str]:
        token = self.token
        if self.token_file:
            try:
                with open(self.token_file, encoding="utf-8") as f:
                    token = f.read().strip()
            except OSError as e:
                raise ConfigException("Invalid kube-config file. tokenFile %s: %s" % (self.token_file, e))
        if self.oidc is not None:  # upstream tries the auth-provider first
            token = self.oidc.token() or token
        elif self.gcp is not None:
            token = self.gcp.token() or token
        if self.exec_spec is not None:
            status = self._run_exec()
            if status.get("token"):
                token = status["token"]
            if status.get("clientCertificateData") and status.get("clientKeyData"):
                self.cert_data = status["clientCertificateData"].encode()
                self.key_data = status["clientKeyData"].encode()
                self._ssl_ctx = None
        if token:
            return {"Authorization": "Bearer " + token}
        if self.username is not None and self.password is not None:
            import base64
            cred = base64.b64encode(f"{self.username}:{self.password}".encode()).decode()
            return {"Authorization": "Basic " + cred}
        return {}

    # -- TLS ------------------------------------------------------------------
    def ssl_context(self):
        if self._ssl_ctx is not None:
            return self._ssl_ctx
        import ssl
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_CLIENT)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        if self.insecure:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        elif self.ca_data is not None or self.ca_file is not None:
            if self.ca_file:
                ctx.load_verify_locations(cafile=self.ca_file)
            if self.ca_data is not None:
                ctx.load_verify_locations(cadata=self.ca_data.decode("ascii", "replace"))
        else:
            ctx.load_default_certs()
        if self.cert_file or self.cert_data:
            self._load_client_cert(ctx)
        self._ssl_ctx = ctx
        return ctx

    def _load_client_cert(self, ctx) -> None:
        if self.cert_file and self.key_file and self.cert_data is None:
            ctx.load_cert_chain(self.cert_file, self.key_file)
            return
        # ssl.load_cert_chain only takes paths: stage *-data in a private 0700 dir
        import tempfile
        d = tempfile.mkdtemp(prefix="k8sgpu-")
        try:
            cert = os.path.join(d, "client.crt")
            key = os.path.join(d, "client.key")
            for path, data, src in ((cert, self.cert_data, self.cert_file), (key, self.key_data, self.key_file)):
                if data is None and src:
                    with open(src, "rb") as f:
                        data = f.read()
                fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
                with os.fdopen(fd, "wb") as f:
                    f.write(data or b"")
            ctx.load_cert_chain(cert, key)
        finally:
            for name in ("client.crt", "client.key"):
                try:
                    os.unlink(os.path.join(d, name))
                except OSError:
                    pass
            os.rmdir(d)

    def describe(self) -> Dict[str, Any]:
        return {"server": self.server, "source": self.source, "insecure": self.insecure,
                "auth": ("exec" if self.exec_spec else "oidc" if self.oidc is not None
                         else "gcp" if self.gcp is not None
                         else "token" if (self.token or self.token_file)
                         else "cert" if (self.cert_file or self.cert_data) else
                         "basic" if self.username else "none")}


def _b64(data: Any) -> bytes:
    import base64
    if isinstance(data, bytes):
        return base64.b64decode(data)
    return base64.b64decode(str(data).encode())


def _path(base: Optional[str], p: Optional[str]) -> Optional[str]:
    if not p:
        return None
    p = os.path.expanduser(p)
    if base and not os.path.isabs(p):
        p = os.path.join(base, p)
    return p


def connection_from_config(cfg: Dict[str, Any], context: Optional[str] = None) -> ClusterConnection:
    ctx_name = context or _need(cfg, "current-context", "kube-config")
    ctx = _get_named(cfg, "contexts", ctx_name)
    ctx_body = _need(ctx, "context", "kube-config/contexts/%s" % ctx_name)
    cluster_name = _need(ctx_body, "cluster", "kube-config/contexts/%s/context" % ctx_name)
    cluster = _need(_get_named(cfg, "clusters", cluster_name), "cluster", "kube-config/clusters/%s" % cluster_name)
    server = _need(cluster, "server", "kube-config/clusters/%s/cluster" % cluster_name)
    conn = ClusterConnection(str(server))
    cbase = cluster.get("__base__")
    if cluster.get("certificate-authority-data"):
        conn.ca_data = _b64(cluster["certificate-authority-data"])
    conn.ca_file = _path(cbase, cluster.get("certificate-authority"))
    insecure = cluster.get("insecure-skip-tls-verify")
    if insecure is not None and not isinstance(insecure, bool):
        # kubectl refuses a non-boolean here (Go's bool unmarshal); bool("no") would silently turn TLS off
        raise ConfigException("Invalid kube-config file. kube-config/clusters/%s/cluster/insecure-skip-tls-verify "
                              "must be a boolean, got %r" % (cluster_name, insecure))
    conn.insecure = bool(insecure)
    conn.tls_server_name = cluster.get("tls-server-name")
    conn.proxy_url = cluster.get("proxy-url")
    user_name = ctx_body.get("user")
    user: Dict[str, Any] = {}
    if user_name:
        try:
            user = _get_named(cfg, "users", user_name).get("user") or {}
        except ConfigException:
            user = {}
    ubase = user.get("__base__")
    if user.get("client-certificate-data"):
        conn.cert_data = _b64(user["client-certificate-data"])
    if user.get("client-key-data"):
        conn.key_data = _b64(user["client-key-data"])
    conn.cert_file = _path(ubase, user.get("client-certificate"))
    conn.key_file = _path(ubase, user.get("client-key"))
    conn.token = user.get("token")
    conn.token_file = _path(ubase, user.get("tokenFile"))
    conn.username = user.get("username")
    conn.password = user.get("password")
    provider = user.get("auth-provider")
    if isinstance(provider, dict) and provider.get("name") == "oidc" and isinstance(provider.get("config"), dict):
        from .oidc import OidcProvider
        conn.oidc = OidcProvider(provider["config"], str(user_name), user.get("__file__"), ubase)
    elif isinstance(provider, dict) and provider.get("name") == "gcp" and not conn.token:
        # the stored access-token, refreshed through cmd-path when it has expired (kube/gcp_cmd.py, PARITY.md #19)
        from .gcp_cmd import GcpCmdProvider
        conn.gcp = GcpCmdProvider(provider.get("config") if isinstance(provider.get("config"), dict) else {})
    elif isinstance(provider, dict) and not conn.token:
        # azure and any other provider: its stored token, used as it is (PARITY.md #19)
        pcfg = provider.get("config") or {}
        conn.token = pcfg.get("id-token") or pcfg.get("access-token")
    if isinstance(user.get("exec"), dict):
        conn.exec_spec = dict(user["exec"])
        conn.exec_spec["__cluster__"] = {
            "server": conn.server,
            "certificate-authority-data": cluster.get("certificate-authority-data"),
            "insecure-skip-tls-verify": conn.insecure,
            "tls-server-name": conn.tls_server_name,
            "proxy-url": conn.proxy_url,
            "config": (cluster.get("extensions") or [{}])[0].get("extension")
            if isinstance(cluster.get("extensions"), list) and cluster.get("extensions") else None,
        }
        conn.exec_base = ubase
    return conn


def incluster_connection(sa_dir: Optional[str] = None) -> Optional[ClusterConnection]:
    sa_dir = sa_dir or SA_DIR
    host = os.environ.get("KUBERNETES_SERVICE_HOST")
    port = os.environ.get("KUBERNETES_SERVICE_PORT")
    token_path = os.path.join(sa_dir, "token")
    if not host or not port or not os.path.isfile(token_path):
        return None
    if ":" in host and not host.startswith("["):
        host = "[" + host + "]"
    conn = ClusterConnection(f"https://{host}:{port}")
    conn.token_file = token_path
    ca = os.path.join(sa_dir, "ca.crt")
    if os.path.isfile(ca):
        conn.ca_file = ca
    conn.source = "in-cluster"
    return conn


def load_kube_config(kubeconfig: Optional[str] = None, context: Optional[str] = None,
                     allow_incluster: bool = True) -> ClusterConnection:
    """Reference ``load_kube_config`` (``:160-169``) + the upstream loader it calls."""
    if kubeconfig:
        paths = kubeconfig
    else:
        env = os.environ.get("KUBECONFIG")
        paths = env if env and os.path.exists(env) else _default_location()
    cfg, first = merge_kubeconfigs(paths)
    if not cfg:
        if allow_incluster and not kubeconfig:
            conn = incluster_connection()
            if conn is not None:
                return conn
        raise ConfigException(_NO_CONFIG)
    conn = connection_from_config(cfg, context)
    conn.source = first or "kubeconfig"
    return conn
