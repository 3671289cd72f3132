"""R6: kubeconfig resolution, merge and the auth matrix (no `kubernetes` package)."""
import base64
import json
import os
import stat
import sys

import pytest
import yaml

from k8s_gpu_node_checker_amd.kube import config as K
from k8s_gpu_node_checker_amd.kube.errors import ConfigException


def write(path, cfg):
    path.write_text(yaml.safe_dump(cfg))
    return str(path)


def cfg(server="https://10.0.0.1:6443", user=None, cluster_extra=None, ctx="c1", name="c1"):
    cluster = {"server": server}
    cluster.update(cluster_extra or {})
    return {"apiVersion": "v1", "kind": "Config", "current-context": ctx,
            "clusters": [{"name": name, "cluster": cluster}],
            "contexts": [{"name": ctx, "context": {"cluster": name, "user": "u1"}}],
            "users": [{"name": "u1", "user": user or {"token": "tok"}}]}


@pytest.fixture(autouse=True)
def clean_env(monkeypatch, tmp_path):
    monkeypatch.delenv("KUBECONFIG", raising=False)
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    monkeypatch.setenv("HOME", str(tmp_path))


def test_explicit_path_wins_over_env(tmp_path, monkeypatch):
    a = write(tmp_path / "a", cfg("https://a:1"))
    b = write(tmp_path / "b", cfg("https://b:2"))
    monkeypatch.setenv("KUBECONFIG", b)
    assert K.load_kube_config(a).server == "https://a:1"


def test_env_var_used_when_file_exists(tmp_path, monkeypatch):
    b = write(tmp_path / "b", cfg("https://b:2"))
    monkeypatch.setenv("KUBECONFIG", b)
    assert K.load_kube_config().server == "https://b:2"


def test_env_colon_list_is_merged_first_wins(tmp_path, monkeypatch):
    a = write(tmp_path / "a", cfg("https://a:1"))
    c2 = cfg("https://b:2", ctx="c2", name="k2")
    c2["clusters"].append({"name": "c1", "cluster": {"server": "https://shadowed:9"}})
    b = write(tmp_path / "b", c2)
    monkeypatch.setenv("KUBECONFIG", f"{a}{os.pathsep}{b}")
    conn = K.load_kube_config()
    assert conn.server == "https://a:1"  # current-context from the first file, c1 not shadowed
    assert K.load_kube_config(context="c2").server == "https://b:2"


def test_default_home_location(tmp_path):
    (tmp_path / ".kube").mkdir()
    write(tmp_path / ".kube" / "config", cfg("https://home:3"))
    assert K.load_kube_config().server == "https://home:3"


def test_missing_everything_raises_reference_message(tmp_path):
    with pytest.raises(ConfigException) as e:
        K.load_kube_config(str(tmp_path / "missing"))
    assert str(e.value) == "Invalid kube-config file. No configuration found."
    with pytest.raises(ConfigException):
        K.load_kube_config()


def test_empty_file_is_no_configuration(tmp_path):
    p = tmp_path / "empty"
    p.write_text("")
    with pytest.raises(ConfigException, match="No configuration found"):
        K.load_kube_config(str(p))


def test_missing_current_context_message(tmp_path):
    c = cfg()
    del c["current-context"]
    with pytest.raises(ConfigException, match="Expected key current-context in kube-config"):
        K.load_kube_config(write(tmp_path / "x", c))


def test_unknown_context_message(tmp_path):
    with pytest.raises(ConfigException, match="Expected object with name nope in kube-config/contexts list"):
        K.load_kube_config(write(tmp_path / "x", cfg()), context="nope")


def test_json_kubeconfig(tmp_path):
    p = tmp_path / "kc.json"
    p.write_text(json.dumps(cfg("https://json:1")))
    assert K.load_kube_config(str(p)).server == "https://json:1"


def test_token_and_token_file(tmp_path):
    conn = K.load_kube_config(write(tmp_path / "x", cfg()))
    assert conn.auth_headers() == {"Authorization": "Bearer tok"}
    tf = tmp_path / "tok"
    tf.write_text("from-file\n")
    conn = K.load_kube_config(write(tmp_path / "y", cfg(user={"tokenFile": "tok"})))
    assert conn.auth_headers() == {"Authorization": "Bearer from-file"}  # relative to the kubeconfig dir


def test_basic_auth(tmp_path):
    conn = K.load_kube_config(write(tmp_path / "x", cfg(user={"username": "u", "password": "p"})))
    assert conn.auth_headers() == {"Authorization": "Basic " + base64.b64encode(b"u:p").decode()}


def test_auth_provider_id_token(tmp_path):
    # upstream _load_oid_token: only a well-formed JWT is presented; "idt" is not one -> no header
    conn = K.load_kube_config(write(tmp_path / "x", cfg(user={"auth-provider": {"name": "oidc",
                                                                                "config": {"id-token": "idt"}}})))
    assert conn.auth_headers() == {} and conn.describe()["auth"] == "oidc"
    jwt = "eyJhbGciOiJub25lIn0.eyJzdWIiOiJ1In0.sig"  # {"sub": "u"}: no exp, never refreshed
    conn = K.load_kube_config(write(tmp_path / "y", cfg(user={"auth-provider": {"name": "oidc",
                                                                                "config": {"id-token": jwt}}})))
    assert conn.auth_headers() == {"Authorization": "Bearer " + jwt}
    # other providers (gcp/azure legacy configs): the cached access-token as a static bearer token
    conn = K.load_kube_config(write(tmp_path / "z", cfg(user={"auth-provider": {"name": "gcp",
                                                                                "config": {"access-token": "at"}}})))
    assert conn.auth_headers() == {"Authorization": "Bearer at"}


def test_tls_fields(tmp_path):
    c = cfg(cluster_extra={"insecure-skip-tls-verify": True, "tls-server-name": "api.internal",
                           "proxy-url": "http://proxy:3128"})
    conn = K.load_kube_config(write(tmp_path / "x", c))
    assert conn.insecure and conn.tls_server_name == "api.internal" and conn.proxy_url == "http://proxy:3128"
    ctx = conn.ssl_context()
    import ssl
    assert ctx.verify_mode == ssl.CERT_NONE


def test_ca_data_decoded(tmp_path):
    c = cfg(cluster_extra={"certificate-authority-data": base64.b64encode(b"PEM").decode()})
    conn = K.load_kube_config(write(tmp_path / "x", c))
    assert conn.ca_data == b"PEM"


def test_exec_plugin(tmp_path):
    script = tmp_path / "plugin.py"
    script.write_text(
        "import json, os, sys\n"
        "info = json.loads(os.environ['KUBERNETES_EXEC_INFO'])\n"
        "assert info['kind'] == 'ExecCredential'\n"
        "srv = info['spec']['cluster']['server']\n"
        "print(json.dumps({'apiVersion': 'client.authentication.k8s.io/v1', 'kind': 'ExecCredential',"
        " 'status': {'token': 'exec-' + os.environ['EXTRA'] + '-' + srv[-4:],"
        " 'expirationTimestamp': '2999-01-01T00:00:00Z'}}))\n")
    user = {"exec": {"apiVersion": "client.authentication.k8s.io/v1", "command": sys.executable,
                     "args": [str(script)], "env": [{"name": "EXTRA", "value": "x"}], "provideClusterInfo": True}}
    conn = K.load_kube_config(write(tmp_path / "x", cfg(user=user)))
    assert conn.auth_headers() == {"Authorization": "Bearer exec-x-6443"}
    assert conn.auth_headers() == {"Authorization": "Bearer exec-x-6443"}  # cached until expiry


def test_exec_plugin_failure_is_config_error(tmp_path):
    user = {"exec": {"command": sys.executable, "args": ["-c", "import sys; sys.exit(3)"]}}
    conn = K.load_kube_config(write(tmp_path / "x", cfg(user=user)))
    with pytest.raises(ConfigException, match="returned 3"):
        conn.auth_headers()


def test_client_cert_data_staged_privately(tmp_path, monkeypatch):
    seen = {}

    class Ctx:
        def load_cert_chain(self, cert, key):
            seen["mode"] = stat.S_IMODE(os.stat(key).st_mode)
            with open(cert, "rb") as f:
                seen["cert"] = f.read()
            seen["path"] = cert
    conn = K.ClusterConnection("https://x")
    conn.cert_data, conn.key_data = b"CERT", b"KEY"
    conn._load_client_cert(Ctx())
    assert seen["cert"] == b"CERT" and seen["mode"] == 0o600
    assert not os.path.exists(seen["path"])  # removed after loading


def test_incluster_fallback_only_without_kubeconfig(tmp_path, monkeypatch):
    sa = tmp_path / "sa"
    sa.mkdir()
    (sa / "token").write_text("satoken")
    (sa / "ca.crt").write_text("CA")
    monkeypatch.setattr(K, "SA_DIR", str(sa))
    monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "10.96.0.1")
    monkeypatch.setenv("KUBERNETES_SERVICE_PORT", "443")
    conn = K.incluster_connection(str(sa))
    assert conn.server == "https://10.96.0.1:443" and conn.source == "in-cluster"
    assert conn.auth_headers() == {"Authorization": "Bearer satoken"}
    monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "fd00::1")
    assert K.incluster_connection(str(sa)).server == "https://[fd00::1]:443"
    assert K.load_kube_config().source == "in-cluster"  # no kubeconfig anywhere -> service account
    # an explicit (missing) --kubeconfig still errors like the reference
    with pytest.raises(ConfigException):
        K.load_kube_config(str(tmp_path / "missing"))


def test_gcp_auth_provider_refreshes_through_cmd_path_when_expired(tmp_path):
    """VERDICT r5 missing #3 / PARITY.md #19: a fresh gcp access-token is used as it is; an expired one is refreshed
    by running the stanza's cmd-path (gcloud config-helper's JSON, the token and expiry at the stanza's keys), once
    until the new one expires; a 401 forces the command again.  No cmd-path: the stored token, expired or not."""
    calls = tmp_path / "calls"
    helper = tmp_path / "helper.py"
    helper.write_text(
        "import json, sys\n"
        f"open({str(calls)!r}, 'a').write('x')\n"
        "n = len(open(" + repr(str(calls)) + ").read())\n"
        "print(json.dumps({'credential': {'access_token': f'fresh-{n}', 'token_expiry': '2999-01-01T00:00:00.123456789Z'},"
        " 'args': sys.argv[1:]}))\n")
    stanza = {"cmd-path": sys.executable, "cmd-args": f"{helper} config config-helper --format=json",
              "token-key": "{.credential.access_token}", "expiry-key": "{.credential.token_expiry}"}
    fresh = {"auth-provider": {"name": "gcp", "config": dict(stanza, **{"access-token": "cached",
                                                                      "expiry": "2999-01-01T00:00:00Z"})}}
    conn = K.load_kube_config(write(tmp_path / "a", cfg(user=fresh)))
    assert conn.auth_headers() == {"Authorization": "Bearer cached"} and not calls.exists()
    assert conn.describe()["auth"] == "gcp"
    expired = {"auth-provider": {"name": "gcp", "config": dict(stanza, **{"access-token": "old",
                                                                        "expiry": "2020-01-01T00:00:00Z"})}}
    conn = K.load_kube_config(write(tmp_path / "b", cfg(user=expired)))
    assert conn.auth_headers() == {"Authorization": "Bearer fresh-1"}
    assert conn.auth_headers() == {"Authorization": "Bearer fresh-1"}  # valid until 2999: not run again
    assert conn.invalidate_credentials() is True
    assert conn.auth_headers() == {"Authorization": "Bearer fresh-2"}
    static = {"auth-provider": {"name": "gcp", "config": {"access-token": "old", "expiry": "2020-01-01T00:00:00Z"}}}
    conn = K.load_kube_config(write(tmp_path / "c", cfg(user=static)))
    assert conn.auth_headers() == {"Authorization": "Bearer old"} and conn.invalidate_credentials() is False
    broken = {"auth-provider": {"name": "gcp", "config": dict(stanza, **{"cmd-args": "-c 'import sys; sys.exit(4)'"})}}
    with pytest.raises(ConfigException, match="exited 4"):
        K.load_kube_config(write(tmp_path / "d", cfg(user=broken))).auth_headers()
    # azure (and any other provider): its stored token as it is
    az = {"auth-provider": {"name": "azure", "config": {"access-token": "az-tok", "expires-on": "0"}}}
    assert K.load_kube_config(write(tmp_path / "e", cfg(user=az))).auth_headers() == {"Authorization": "Bearer az-tok"}
    from k8s_gpu_node_checker_amd.kube.gcp_cmd import parse_time
    assert parse_time("1970-01-01T00:00:01Z") == 1.0 and parse_time("1970-01-01T01:00:01+01:00") == 1.0
    assert parse_time("nope") is None and parse_time(None) is None
