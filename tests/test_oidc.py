"""``auth-provider: oidc`` refresh (kube/oidc.py) against a mock IdP and the mock kube-apiserver:
refresh on expiry, refresh on a 401, write-back into the kubeconfig, a refused refresh (exit 1, the
reference's error shape), and concurrent checkers sharing one kubeconfig with single-use (rotating)
refresh tokens.  Parity unpinned: the `kubernetes` package whose loader the reference uses is not
importable here; the semantics follow its KubeConfigLoader._load_oid_token / _refresh_oidc."""
import base64
import json
import subprocess
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs

import pytest
import yaml

from k8s_gpu_node_checker_amd.kube import config as K
from k8s_gpu_node_checker_amd.kube import oidc
from k8s_gpu_node_checker_amd.kube.errors import ConfigException
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.mock_apiserver import MockApiServer, MockConfig

from conftest import REPO


def jwt(exp, sub="user", n=0):
    def b64(d):
        return base64.urlsafe_b64encode(json.dumps(d, separators=(",", ":")).encode()).decode().rstrip("=")
    return f"{b64({'alg': 'RS256'})}.{b64({'sub': sub, 'exp': exp, 'n': n})}.c2ln"


class MockIdP:
    """Discovery + token endpoint; every refresh token is single-use (rotated on each grant)."""

    def __init__(self, fail=None, discovery_status=200):
        self.valid_refresh = {"rt-0"}
        self.grants = []
        self.fail = fail
        self.discovery_status = discovery_status
        self.lock = threading.Lock()
        self.n = 0
        self.exp = int(time.time()) + 3600  # every minted id-token: jwt(self.exp, n=<grant number>)
        idp = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _json(self, code, doc):
                body = json.dumps(doc).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):
                if self.path == "/.well-known/openid-configuration":
                    return self._json(idp.discovery_status, {"issuer": idp.url, "token_endpoint": idp.url + "/token"})
                self._json(404, {})

            def do_POST(self):
                form = {k: v[0] for k, v in parse_qs(self.rfile.read(int(self.headers["Content-Length"])).decode()).items()}
                auth = self.headers.get("Authorization", "")
                with idp.lock:
                    idp.grants.append({"form": form, "auth": auth})
                    if idp.fail:
                        return self._json(400, {"error": idp.fail, "error_description": "refresh token revoked"})
                    if auth != "Basic " + base64.b64encode(b"kube:s3cret").decode() or form.get("client_id") != "kube":
                        return self._json(401, {"error": "invalid_client"})
                    rt = form.get("refresh_token")
                    if form.get("grant_type") != "refresh_token" or rt not in idp.valid_refresh:
                        return self._json(400, {"error": "invalid_grant"})
                    idp.valid_refresh.discard(rt)
                    idp.n += 1
                    new_rt = f"rt-{idp.n}"
                    idp.valid_refresh.add(new_rt)
                    idp.current = jwt(idp.exp, n=idp.n)
                    return self._json(200, {"id_token": idp.current, "refresh_token": new_rt, "token_type": "Bearer"})

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        self.current = None

    def __enter__(self):
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()
        return self

    def __exit__(self, *a):
        self.srv.shutdown()
        self.srv.server_close()


def kubeconfig(path, api_url, idp_url, id_token, refresh="rt-0"):
    doc = {"apiVersion": "v1", "kind": "Config", "current-context": "c",
           "clusters": [{"name": "k", "cluster": {"server": api_url}}],
           "contexts": [{"name": "c", "context": {"cluster": "k", "user": "oidc-user"}}],
           "users": [{"name": "oidc-user", "user": {"auth-provider": {"name": "oidc", "config": {
               "client-id": "kube", "client-secret": "s3cret", "id-token": id_token, "refresh-token": refresh,
               "idp-issuer-url": idp_url}}}}]}
    path.write_text("# managed by kubelogin\n" + yaml.safe_dump(doc))
    return str(path)


def persisted(path):
    with open(path) as f:
        d = yaml.safe_load(f)
    return d["users"][0]["user"]["auth-provider"]["config"]


def run_check(kc, *extra):
    return subprocess.run([sys.executable, f"{REPO}/check-gpu-node.py", "--kubeconfig", kc, "--json", *extra],
                          capture_output=True, text=True, timeout=60)


def test_jwt_expiry_rules():
    assert oidc.jwt_expiry(jwt(123)) == 123.0
    assert oidc.jwt_expiry("eyJhIjoxfQ.eyJzdWIiOiJ1In0.x") is None  # no exp claim
    for bad in ("a.b", "x+y.z.w", "a.b=.c", "a.abcde.c"):  # not 3 parts, unsafe chars, 3-char padding
        with pytest.raises(ValueError):
            oidc.jwt_expiry(bad)


def test_expired_token_is_refreshed_and_written_back(tmp_path):
    with MockIdP() as idp, MockApiServer([fixtures.realistic_node("a")], cfg=MockConfig(token="never")) as api:
        kc = kubeconfig(tmp_path / "config", api.url, idp.url, jwt(int(time.time()) - 10))
        conn = K.load_kube_config(kc)
        hdr = conn.auth_headers()
        assert len(idp.grants) == 1 and hdr == {"Authorization": "Bearer " + idp.current}
        g = idp.grants[0]["form"]
        assert g == {"grant_type": "refresh_token", "refresh_token": "rt-0", "client_id": "kube",
                     "client_secret": "s3cret"}
        p = persisted(kc)
        assert p["id-token"] == idp.current and p["refresh-token"] == "rt-1"
        assert not (tmp_path / "config.lock").exists()
        # still valid: no second grant
        assert conn.auth_headers() == hdr and len(idp.grants) == 1
        # the full CLI against an apiserver that accepts only the token of the IdP's next grant
        api.cfg.token = jwt(idp.exp, n=2)
        kc2 = kubeconfig(tmp_path / "config2", api.url, idp.url, jwt(int(time.time()) + 30), refresh="rt-1")
        r = run_check(kc2)  # expires within the 5-minute skew -> refreshed before the LIST
        assert r.returncode == 0, r.stdout + r.stderr
        assert json.loads(r.stdout)["ready_nodes"] == 1 and persisted(kc2)["refresh-token"] == "rt-2"


def test_401_forces_one_refresh_and_retry(tmp_path):
    """An unexpired id-token the apiserver rejects (revoked): the 401 makes the checker refresh once and
    retry the LIST with the new token."""
    with MockIdP() as idp, MockApiServer([fixtures.realistic_node("a")]) as api:
        api.cfg.token = jwt(idp.exp, n=1)  # the token the IdP's first grant mints
        kc = kubeconfig(tmp_path / "config", api.url, idp.url, jwt(idp.exp, sub="revoked"))
        r = run_check(kc)
        assert r.returncode == 0 and json.loads(r.stdout)["ready_nodes"] == 1, r.stdout + r.stderr
        assert len(idp.grants) == 1 and persisted(kc)["id-token"] == api.cfg.token
        auths = [e["auth"] for e in api.log]
        assert auths[0] == "Bearer " + jwt(idp.exp, sub="revoked") and auths[-1] == "Bearer " + api.cfg.token
        # a second 401 after the refresh is final: exit 1 with the reference's error shape
        api.cfg.token = "nobody"
        r = run_check(kc)
        assert r.returncode == 1 and json.loads(r.stdout)["error"].startswith("(401)")
        assert len(idp.grants) == 2  # one refresh per run, never a loop


def test_refused_refresh_is_exit_1_with_the_error_shape(tmp_path):
    with MockIdP(fail="invalid_grant") as idp, MockApiServer([fixtures.realistic_node("a")]) as api:
        kc = kubeconfig(tmp_path / "config", api.url, idp.url, jwt(int(time.time()) - 10))
        r = run_check(kc)
        assert r.returncode == 1 and r.stderr == ""
        err = json.loads(r.stdout)["error"]
        assert err.startswith("OIDC token refresh at " + idp.url + "/token failed: HTTP 400 invalid_grant")
        r = subprocess.run([sys.executable, f"{REPO}/check-gpu-node.py", "--kubeconfig", kc], capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 1 and r.stderr.startswith("에러: OIDC token refresh at ")
        assert persisted(kc)["refresh-token"] == "rt-0"  # nothing written on failure
        assert not (tmp_path / "config.lock").exists()


def test_discovery_failure_keeps_the_old_token(tmp_path):
    with MockIdP(discovery_status=503) as idp, MockApiServer([fixtures.realistic_node("a")]) as api:
        old = jwt(int(time.time()) - 10)
        kc = kubeconfig(tmp_path / "config", api.url, idp.url, old)
        assert K.load_kube_config(kc).auth_headers() == {"Authorization": "Bearer " + old}  # upstream
        assert idp.grants == []


def test_concurrent_checkers_refresh_once(tmp_path):
    """Six checkers start together on one kubeconfig with an expired token and a single-use refresh
    token: one refreshes, the others wait on <kubeconfig>.lock and adopt the token it wrote."""
    with MockIdP() as idp, MockApiServer([fixtures.realistic_node("a")]) as api:
        api.cfg.token = jwt(idp.exp, n=1)
        kc = kubeconfig(tmp_path / "config", api.url, idp.url, jwt(int(time.time()) - 10))
        procs = [subprocess.Popen([sys.executable, f"{REPO}/check-gpu-node.py", "--kubeconfig", kc, "--json"],
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for _ in range(6)]
        outs = [p.communicate(timeout=60) for p in procs]
        assert [p.returncode for p in procs] == [0] * 6, outs
        assert len(idp.grants) == 1, idp.grants
        assert persisted(kc)["refresh-token"] == "rt-1" and persisted(kc)["id-token"] == api.cfg.token
        assert not (tmp_path / "config.lock").exists()
        with open(kc) as f:
            assert f.read().startswith("apiVersion")  # rewritten as YAML (the comment is not kept)


def test_stale_lock_is_broken(tmp_path, monkeypatch):
    lock = tmp_path / "config.lock"
    lock.write_text("")
    old = time.time() - oidc.LOCK_STALE_S - 5
    import os
    os.utime(lock, (old, old))
    with oidc._FileLock(str(tmp_path / "config")) as lk:
        assert lk.held
    assert not lock.exists()
    lock.write_text("")  # a live lock: wait, then give up with a clear error
    monkeypatch.setattr(oidc, "LOCK_WAIT_S", 0.05)
    with pytest.raises(ConfigException, match="kubeconfig is locked"):
        with oidc._FileLock(str(tmp_path / "config")):
            pass
