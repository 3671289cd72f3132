"""notify/webhook.py == ``requests.post`` on the wire.

``requests`` is importable in this image (not a dependency of the package): each case POSTs the same body
through ``requests.post`` and through :func:`webhook.post` to the same sink and compares the outcome (status
and text, or the exception text) and every request the sink saw -- method, path and headers in order, minus
``User-Agent`` (this package names itself) and ``Host`` (the same by construction).
"""
import os

import pytest

from k8s_gpu_node_checker_amd.notify import webhook

requests = pytest.importorskip("requests")


def _run(sink, url, env):
    out = []
    for which in ("requests", "webhook"):
        n0 = len(sink.requests)
        try:
            if which == "requests":
                r = requests.post(url, json={"a": 1}, timeout=10, headers={"Content-Type": "application/json"})
                res = (r.status_code, r.text)
            else:
                r = webhook.post(url, b'{"a": 1}', environ=env)
                res = (r.status, webhook.response_text(r))
        except Exception as e:  # the reference prints str(e) for every failure
            res = ("error", str(e))
        seen = [(q["method"], q["path"], [(k, v) for k, v in q["headers"].items() if k not in ("User-Agent", "Host")],
                 q["body"]) for q in sink.requests[n0:]]
        out.append((res, seen))
    return out


CASES = ["200", "500", "301", "302", "303", "307", "308", "loop", "cookie", "to/localhost/200", "to/localhost/301",
         "a/../b/./200/../200?x=a b#frag", "%7euser/200"]


@pytest.mark.parametrize("path", CASES)
def test_same_requests_and_outcome(sink, path, monkeypatch):
    for k in ("REQUESTS_CA_BUNDLE", "CURL_CA_BUNDLE", "NETRC", "http_proxy", "HTTP_PROXY", "all_proxy", "ALL_PROXY"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("HOME", "/nonexistent-home")
    a, b = _run(sink, sink.url(path), dict(os.environ))
    assert a == b


@pytest.mark.parametrize("userinfo", ["us%40er:p%3Ass@", "user@", "user:@", ":pw@", "u:p@"])
@pytest.mark.parametrize("path", ["200", "to/localhost/200", "301"])
def test_url_credentials(sink, userinfo, path, monkeypatch):
    monkeypatch.delenv("NETRC", raising=False)
    monkeypatch.setenv("HOME", "/nonexistent-home")
    host, port = sink.server_address[:2]
    a, b = _run(sink, f"http://{userinfo}{host}:{port}/{path}", dict(os.environ))
    assert a == b
    if userinfo == "u:p@":
        assert ("Authorization", "Basic dTpw") in b[1][0][2]


@pytest.mark.parametrize("url", ["http://127.0.0.1:99999/x", "http://[::1/x", "http://[::1]:70000/x", "ftp://x/y",
                                 "nohost", "http://", "  http://127.0.0.1:1/x", "http://no-such-host.invalid/x",
                                 "http://.bad/x", "http://127.0.0.1:1/x"])
def test_url_and_connection_errors(sink, url, monkeypatch):
    monkeypatch.setenv("HOME", "/nonexistent-home")
    a, b = _run(sink, url, dict(os.environ))
    assert a == b and a[0][0] == "error"


def test_netrc_wins_over_url_credentials_and_follows_redirects(sink, tmp_path, monkeypatch):
    host, port = sink.server_address[:2]
    rc = tmp_path / "netrc"
    rc.write_text(f"machine {host} login nu password np\nmachine localhost login lu password lp\n")
    monkeypatch.setenv("NETRC", str(rc))
    for url in (f"http://{host}:{port}/200", f"http://x:y@{host}:{port}/200", f"http://{host}:{port}/to/localhost/200"):
        a, b = _run(sink, url, dict(os.environ))
        assert a == b
    rc.write_text("machine garbage\n  login\n")  # malformed: skipped, as requests does
    a, b = _run(sink, f"http://u:p@{host}:{port}/200", dict(os.environ))
    assert a == b


def test_missing_ca_bundle(sink, monkeypatch):
    monkeypatch.setenv("REQUESTS_CA_BUNDLE", "/missing")
    host, port = sink.server_address[:2]
    for url in (f"https://{host}:{port}/x", f"http://{host}:{port}/200"):
        a, b = _run(sink, url, dict(os.environ))
        assert a == b


def test_response_text_encodings():
    from k8s_gpu_node_checker_amd.utils.http import Response
    body = "실패".encode("utf-8")
    for ctype, want in (("text/plain", body.decode("latin-1")), ("text/plain; charset=utf-8", "실패"),
                        ("application/json", "실패"), (None, "실패")):
        hdrs = [("Content-Type", ctype)] if ctype else []
        assert webhook.response_text(Response(500, "x", hdrs, body)) == want


def test_deflate_and_gzip_responses_decoded():
    import zlib
    from k8s_gpu_node_checker_amd.utils.http import _decode_content
    raw = b"server_error"
    assert _decode_content(zlib.compress(raw), "deflate") == raw
    c = zlib.compressobj(wbits=-zlib.MAX_WBITS)
    assert _decode_content(c.compress(raw) + c.flush(), "deflate") == raw
    g = zlib.compressobj(wbits=16 + zlib.MAX_WBITS)
    assert _decode_content(g.compress(raw) + g.flush(), "gzip") == raw


from hypothesis import given, settings, strategies as st  # noqa: E402

_URL_PART = st.lists(st.sampled_from(list("aZ09-._~!$&'()*+,;=:/?@%# é[]") + ["..", "./", "%41", "%zz", "%7e"]),
                     max_size=10).map("".join)


@settings(max_examples=400, deadline=None)
@given(scheme=st.sampled_from(["http://", "https://", "HTTP://", "ftp://", ""]),
       host=st.sampled_from(["127.0.0.1", "Hooks.Slack.com", "localhost", ".x", "[::1]", "a_b", "", "h"]),
       port=st.sampled_from(["", ":80", ":080", ":0", ":65535", ":65536", ":x"]), rest=_URL_PART)
def test_prepare_url_matches_requests(scheme, host, port, rest):
    """The no-regex fast path and the full path both equal requests' PreparedRequest.prepare_url."""
    url = scheme + host + port + ("/" + rest if rest else "")
    try:
        p = requests.models.PreparedRequest()
        p.prepare_url(url, None)
        want = ("ok", p.url)
    except Exception as e:
        want = ("error", str(e))
    try:
        got = ("ok", webhook.prepare_url(url))
    except webhook.RequestError as e:
        got = ("error", str(e))
    assert got == want, url
    fast = webhook._simple(url)
    if fast is not None:
        assert ("ok", fast) == want, url
