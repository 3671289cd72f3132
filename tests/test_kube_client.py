"""kube-apiserver client: pagination, retries/backoff, errors, gzip, chunked, TLS (SURVEY §7.2 layer 2)."""
import subprocess

import pytest

from k8s_gpu_node_checker_amd.kube.client import KubeClient
from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
from k8s_gpu_node_checker_amd.kube.errors import ApiException, TransportError
from k8s_gpu_node_checker_amd.models.node import scan_items
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.mock_apiserver import MockApiServer


def names(res):
    return [n["name"] for n in res.gpu_nodes]


def client(srv, **kw):
    kw.setdefault("sleep", lambda s: None)
    return KubeClient(ClusterConnection(srv.url), **kw)


def test_pagination_preserves_order_and_uses_one_connection(mock_cluster):
    nodes = fixtures.cluster(23, "mixed", not_ready=[4])
    srv = mock_cluster(nodes)
    with client(srv) as c:
        res = c.scan_nodes(limit=5)
    assert names(res) == names(scan_items(nodes))
    assert res.items_seen == 23
    assert [e["path"] for e in srv.log][:2] == ["/api/v1/nodes?limit=5", "/api/v1/nodes?limit=5&continue=c5.1000"]
    assert len(srv.log) == 5


def test_unpaginated(mock_cluster):
    srv = mock_cluster(fixtures.cluster(7, "amd"))
    with client(srv) as c:
        res = c.scan_nodes(limit=0)
    assert len(res.gpu_nodes) == 7 and srv.log[0]["path"] == "/api/v1/nodes"


def test_expired_continue_falls_back_to_full_list(mock_cluster):
    nodes = fixtures.cluster(12, "amd")
    srv = mock_cluster(nodes, expire_continue=True)
    with client(srv) as c:
        res = c.scan_nodes(limit=5)
    assert names(res) == names(scan_items(nodes))  # no duplicates from the partial first page
    assert srv.log[-1]["path"] == "/api/v1/nodes"


def test_transient_503_is_retried_honouring_retry_after(mock_cluster):
    srv = mock_cluster(fixtures.cluster(2, "amd"), fail_first=2, retry_after="0.5")
    slept = []
    with KubeClient(ClusterConnection(srv.url), retries=2, sleep=slept.append) as c:
        res = c.scan_nodes()
    assert len(res.gpu_nodes) == 2 and slept == [0.5, 0.5]


def test_retries_exhausted_raises_api_exception(mock_cluster):
    srv = mock_cluster(fixtures.cluster(2, "amd"), fail_first=10)
    with client(srv, retries=1) as c:
        with pytest.raises(ApiException) as e:
            c.scan_nodes()
    assert e.value.status == 503
    assert str(e.value).startswith("(503)\nReason: Service Unavailable\n")


def test_403_not_retried(mock_cluster):
    srv = mock_cluster(fixtures.cluster(2, "amd"), status=403)
    with client(srv, retries=3) as c:
        with pytest.raises(ApiException) as e:
            c.scan_nodes()
    assert len(srv.log) == 1
    s = str(e.value)
    assert s.startswith("(403)\nReason: Forbidden\nHTTP response headers: HTTPHeaderDict({")
    assert "HTTP response body: " in s and "forbidden" in s


def test_connection_refused_message():
    c = KubeClient(ClusterConnection("http://127.0.0.1:9"), retries=1, sleep=lambda s: None)
    with pytest.raises(TransportError) as e:
        c.scan_nodes()
    msg = str(e.value)
    assert msg.startswith("HTTPConnectionPool(host='127.0.0.1', port=9): Max retries exceeded with url: /api/v1/nodes")


def test_read_timeout(mock_cluster):
    srv = mock_cluster(fixtures.cluster(1, "amd"), delay=1.0)
    c = KubeClient(ClusterConnection(srv.url), timeout=0.2, retries=0)
    with pytest.raises(TransportError) as e:
        c.scan_nodes()
    assert "Read timed out. (read timeout=0.2)" in str(e.value)


def test_reset_by_server(mock_cluster):
    srv = mock_cluster(fixtures.cluster(1, "amd"), reset=True)
    c = KubeClient(ClusterConnection(srv.url), retries=0)
    with pytest.raises(TransportError) as e:
        c.scan_nodes()
    assert "Connection aborted" in str(e.value) or "Connection reset" in str(e.value)


def test_gzip_and_chunked(mock_cluster):
    nodes = fixtures.cluster(9, "amd")
    for cfg in ({"gzip": True}, {"chunked": True}):
        srv = mock_cluster(nodes, **cfg)
        with KubeClient(ClusterConnection(srv.url), gzip=True) as c:
            res = c.scan_nodes(limit=4)
        assert len(res.gpu_nodes) == 9


def test_gzip_off_for_loopback_on_for_remote():
    assert KubeClient(ClusterConnection("http://127.0.0.1:1")).gzip is False
    assert KubeClient(ClusterConnection("https://api.example.com")).gzip is True


def test_label_selector_and_resource_version(mock_cluster):
    srv = mock_cluster(fixtures.cluster(2, "amd"))
    with client(srv) as c:
        c.scan_nodes(limit=0, label_selector="pool=training,amd.com/gpu.family=MI355X", resource_version="0")
    assert srv.log[0]["path"] == "/api/v1/nodes?labelSelector=pool%3Dtraining%2Camd.com%2Fgpu.family%3DMI355X&resourceVersion=0"


def test_patch_annotations_and_get(mock_cluster):
    srv = mock_cluster(fixtures.cluster(2, "amd"))
    with client(srv) as c:
        c.patch_node_annotations("mi355x-node-0001", {"amd.com/x": "1"})
        node = c.get_node("mi355x-node-0001")
    assert node["metadata"]["annotations"]["amd.com/x"] == "1"
    assert srv.log[0]["method"] == "PATCH"


def test_tls_with_ca_file_and_sni(certs):
    crt, key = certs
    with MockApiServer(fixtures.cluster(3, "amd"), certfile=crt, keyfile=key) as srv:
        conn = ClusterConnection(srv.url)
        conn.ca_file = crt
        with KubeClient(conn) as c:
            assert len(c.scan_nodes().gpu_nodes) == 3
        conn2 = ClusterConnection(srv.url.replace("127.0.0.1", "localhost"))
        with open(crt, "rb") as f:
            conn2.ca_data = f.read()
        conn2.tls_server_name = "localhost"
        with KubeClient(conn2) as c:
            assert len(c.scan_nodes().gpu_nodes) == 3


def test_tls_verification_failure_is_not_retried(certs):
    crt, key = certs
    with MockApiServer(fixtures.cluster(1, "amd"), certfile=crt, keyfile=key) as srv:
        c = KubeClient(ClusterConnection(srv.url), retries=3, sleep=lambda s: None)  # system CAs: untrusted
        with pytest.raises(TransportError) as e:
            c.scan_nodes()
        assert "SSLError" in str(e.value) or "CERTIFICATE_VERIFY_FAILED" in str(e.value)
        assert len(srv.log) == 0


def test_tls_insecure_skip_verify(certs):
    crt, key = certs
    with MockApiServer(fixtures.cluster(2, "amd"), certfile=crt, keyfile=key) as srv:
        conn = ClusterConnection(srv.url)
        conn.insecure = True
        with KubeClient(conn) as c:
            assert len(c.scan_nodes().gpu_nodes) == 2


@pytest.fixture(scope="module")
def mtls(tmp_path_factory):
    """A CA, a server cert and a client cert (openssl CLI)."""
    d = tmp_path_factory.mktemp("mtls")

    def run(*a):
        r = subprocess.run(["openssl", *a], capture_output=True, cwd=str(d))
        if r.returncode != 0:
            pytest.skip("openssl failed: " + r.stderr.decode()[-200:])
    run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "ca.key", "-out", "ca.crt", "-days", "1",
        "-subj", "/CN=test-ca")
    for name, ext in (("srv", "subjectAltName=IP:127.0.0.1"), ("cli", "extendedKeyUsage=clientAuth")):
        run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{name}.key", "-out", f"{name}.csr", "-subj",
            f"/CN={name}")
        (d / f"{name}.ext").write_text(ext + "\n")
        run("x509", "-req", "-in", f"{name}.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial", "-out",
            f"{name}.crt", "-days", "1", "-extfile", f"{name}.ext")
    return d


def test_mutual_tls_client_certificate_data(mtls, tmp_path):
    """kubeconfig client-certificate-data/client-key-data + certificate-authority-data against an mTLS server."""
    import base64
    import ssl
    import yaml
    from k8s_gpu_node_checker_amd.kube.config import load_kube_config
    srv = MockApiServer(fixtures.cluster(2, "amd"), certfile=str(mtls / "srv.crt"), keyfile=str(mtls / "srv.key"))
    ctx = srv.socket.context
    ctx.verify_mode = ssl.CERT_REQUIRED
    ctx.load_verify_locations(str(mtls / "ca.crt"))
    with srv:
        b64 = lambda f: base64.b64encode((mtls / f).read_bytes()).decode()
        cfg = {"apiVersion": "v1", "kind": "Config", "current-context": "m",
               "clusters": [{"name": "m", "cluster": {"server": srv.url, "certificate-authority-data": b64("ca.crt")}}],
               "contexts": [{"name": "m", "context": {"cluster": "m", "user": "u"}}],
               "users": [{"name": "u", "user": {"client-certificate-data": b64("cli.crt"),
                                                "client-key-data": b64("cli.key")}}]}
        kc = tmp_path / "kc.yaml"
        kc.write_text(yaml.safe_dump(cfg))
        with KubeClient(load_kube_config(str(kc))) as c:
            assert len(c.scan_nodes().gpu_nodes) == 2
        cfg["users"][0]["user"] = {}  # no client cert: the handshake must fail
        kc.write_text(yaml.safe_dump(cfg))
        with pytest.raises(TransportError):
            KubeClient(load_kube_config(str(kc)), retries=0).scan_nodes()


def test_https_through_connect_proxy(certs, tmp_path):
    """cluster.proxy-url: HTTPS to the apiserver tunnelled through an HTTP CONNECT proxy."""
    from k8s_gpu_node_checker_amd.testing.proxy import ForwardProxy
    crt, key = certs
    with ForwardProxy() as px, MockApiServer(fixtures.cluster(3, "amd"), certfile=crt, keyfile=key) as srv:
        conn = ClusterConnection(srv.url)
        conn.ca_file = crt
        conn.proxy_url = px.url
        with KubeClient(conn) as c:
            assert len(c.scan_nodes().gpu_nodes) == 3
        assert px.seen and px.seen[0][0].startswith("CONNECT 127.0.0.1:") and px.seen[0][1] is None


def test_pipelined_pagination_uses_two_connections(mock_cluster):
    nodes = fixtures.cluster(30, "mixed", not_ready=[7])
    srv = mock_cluster(nodes)
    with client(srv) as c:
        res = c.scan_nodes(limit=4)
        assert c._conn2 is not None  # the next page was requested while the previous one was read
    assert names(res) == names(scan_items(nodes)) and res.items_seen == 30
    with KubeClient(ClusterConnection(srv.url), pipeline=False) as c:
        assert names(c.scan_nodes(limit=4)) == names(res) and c._conn2 is None


def test_401_refetches_rotated_credentials_once(tmp_path, mock_cluster):
    """A token rejected with 401 (rotated service-account token, expired exec credential) is fetched
    again once -- the exec plugin re-runs even though its credential had no expiry -- then the
    request is repeated; a second 401 is final."""
    import sys as _sys
    from k8s_gpu_node_checker_amd.kube.config import load_kube_config
    srv = mock_cluster(fixtures.cluster(1, "amd"), token="fresh")
    counter = tmp_path / "n"
    plugin = tmp_path / "plugin.py"
    plugin.write_text(
        "import json, pathlib\n"
        f"p = pathlib.Path({str(counter)!r})\n"
        "n = int(p.read_text()) if p.exists() else 0\n"
        "p.write_text(str(n + 1))\n"
        "tok = 'stale' if n == 0 else 'fresh'\n"
        "print(json.dumps({'apiVersion': 'client.authentication.k8s.io/v1', 'kind': 'ExecCredential',"
        " 'status': {'token': tok}}))\n")
    import yaml as _yaml
    cfg = {"apiVersion": "v1", "kind": "Config", "current-context": "c",
           "clusters": [{"name": "c", "cluster": {"server": srv.url}}],
           "contexts": [{"name": "c", "context": {"cluster": "c", "user": "u"}}],
           "users": [{"name": "u", "user": {"exec": {"apiVersion": "client.authentication.k8s.io/v1",
                                                     "command": _sys.executable, "args": [str(plugin)]}}}]}
    kc = tmp_path / "kc"
    kc.write_text(_yaml.safe_dump(cfg))
    cluster = load_kube_config(str(kc))
    with KubeClient(cluster) as c:
        assert c.scan_nodes().gpu_nodes
    assert counter.read_text() == "2"
    auths = [e["auth"] for e in srv.log]
    assert auths == ["Bearer stale", "Bearer fresh"]
    # a credential that stays wrong: one re-fetch, then the 401 surfaces
    srv.cfg.token = "other"
    with KubeClient(cluster) as c:
        with pytest.raises(ApiException) as ei:
            c.scan_nodes()
    assert ei.value.status == 401


def test_a_repeated_continue_token_ends_in_one_full_list():
    """An apiserver (or a proxy in front of it) that hands out the same continue token again would make the
    pager loop forever, collecting the same nodes each time: the second sighting of a token switches to one
    consistent full LIST, as an expired token does."""
    import json
    import threading
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
    nodes = fixtures.cluster(6, "amd")
    paths = []

    class H(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, *a):
            pass

        def do_GET(self):  # noqa: N802
            paths.append(self.path)
            full = "limit=" not in self.path
            doc = {"kind": "NodeList", "apiVersion": "v1",
                   "metadata": {"resourceVersion": "7"} if full else {"resourceVersion": "7", "continue": "same"},
                   "items": nodes if full else nodes[:2]}
            body = json.dumps(doc).encode()
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)
    srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        with KubeClient(ClusterConnection(f"http://127.0.0.1:{srv.server_address[1]}"), sleep=lambda s: None) as c:
            res = c.scan_nodes(limit=2)
        assert names(res) == names(scan_items(nodes))  # each node once
        assert paths[-1] == "/api/v1/nodes" and len(paths) <= 4, paths
    finally:
        srv.shutdown()
        srv.server_close()
