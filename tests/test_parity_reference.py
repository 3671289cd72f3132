"""Contract parity: the UNMODIFIED reference script (with test stand-ins for `kubernetes`/`dotenv`,
tests/refstub) and this CLI run against the same mock apiserver / webhook sink; stdout, stderr
classes, exit codes and Slack requests must match (SURVEY §4.3 "contract/parity").

Skipped when /root/reference is not mounted (e.g. on the GPU box).
"""
import json
import os
import re
import ssl
import subprocess
import sys

import pytest

from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
from k8s_gpu_node_checker_amd.testing.webhook_sink import WebhookSink

REF = os.environ.get("K8SGPU_REFERENCE", "/root/reference/check-gpu-node.py")
STUBS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "refstub")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = [pytest.mark.reference,
              pytest.mark.skipif(not os.path.exists(REF), reason="reference script not mounted")]


def _env(extra=None):
    e = {k: v for k, v in os.environ.items() if k not in ("SLACK_WEBHOOK_URL", "KUBECONFIG", "PYTHONPATH")}
    e["COLUMNS"] = "80"
    if extra:
        e.update(extra)
    return e


def run_ref(args, env=None, cwd=None):
    e = _env(env)
    e["PYTHONPATH"] = STUBS
    return subprocess.run([sys.executable, REF] + args, capture_output=True, text=True, env=e, timeout=120, cwd=cwd)


def run_new(args, env=None, cwd=None):
    return subprocess.run([sys.executable, os.path.join(REPO, "check-gpu-node.py")] + args, capture_output=True,
                          text=True, env=_env(env), timeout=120, cwd=cwd)


@pytest.fixture
def cluster(tmp_path, mock_cluster):
    def make(nodes):
        srv = mock_cluster(nodes)
        return write_kubeconfig(str(tmp_path / "kc.yaml"), srv.url)
    return make


CLUSTERS = {**{g: (lambda g=g: fixtures.golden(g)) for g in fixtures.GOLDEN},
            "amd8": lambda: fixtures.cluster(8, "amd"),
            "amd8-2notready": lambda: fixtures.cluster(8, "amd", not_ready=[1, 5]),
            "cpu16": lambda: fixtures.cluster(16, "cpu"),
            "mixed40": lambda: fixtures.cluster(40, "mixed", not_ready=[3])}


@pytest.mark.parametrize("name", sorted(CLUSTERS))
@pytest.mark.parametrize("flags", [[], ["--json"]])
def test_same_output_same_exit_code(cluster, name, flags):
    kc = cluster(CLUSTERS[name]())
    a = run_ref(["--kubeconfig", kc] + flags)
    b = run_new(["--kubeconfig", kc] + flags)
    assert a.returncode == b.returncode, (a.stderr, b.stderr)
    assert a.stdout == b.stdout
    assert a.stderr == b.stderr == ""


@pytest.mark.parametrize("flags", [[], ["--json"]])
def test_large_paged_cluster_identical(cluster, flags):
    """2,500 mixed nodes (every 7th NotReady): the CLI pages the LIST (limit 500, five pages) and scans it natively,
    the reference takes one unpaginated LIST; stdout and exit code are byte-identical."""
    nodes = fixtures.cluster(2500, "mixed", not_ready=list(range(0, 2500, 7)))
    kc = cluster(nodes)
    a, b = run_ref(["--kubeconfig", kc] + flags), run_new(["--kubeconfig", kc] + flags)
    assert (a.returncode, a.stderr) == (b.returncode, b.stderr) == (0, "")
    assert a.stdout == b.stdout and len(a.stdout) > 100_000


def test_help_and_usage_error_identical():
    a, b = run_ref(["--help"]), run_new(["--help"])
    assert (a.returncode, a.stdout) == (b.returncode, b.stdout)
    a, b = run_ref(["--bogus"]), run_new(["--bogus"])
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)


def test_missing_kubeconfig_identical(tmp_path):
    a = run_ref(["--json", "--kubeconfig", str(tmp_path / "missing")])
    b = run_new(["--json", "--kubeconfig", str(tmp_path / "missing")])
    assert (a.returncode, a.stdout) == (b.returncode, b.stdout) == (1, '{"error": "Invalid kube-config file. No configuration found."}\n')


def _slack_case(cluster, sink, mode, extra_flags, nodes):
    kc = cluster(nodes)
    url = sink.url(mode)
    flags = ["--kubeconfig", kc, "--slack-webhook", url, "--slack-retry-delay", "0"] + extra_flags
    before = len(sink.requests)
    a = run_ref(flags)
    mid = len(sink.requests)
    sink.counts.clear()
    b = run_new(flags + ["--slack-retry-policy", "reference"])
    after = len(sink.requests)
    return a, b, sink.requests[before:mid], sink.requests[mid:after]


@pytest.mark.parametrize("mode", ["200", "500", "204", "flaky2", "resetflaky", "reset", "close", "404", "429",
                                  "seq/mix1/close,500,200", "seq/mix2/reset,404,close"])
def test_slack_behaviour_matches(cluster, sink, mode):
    a, b, ra, rb = _slack_case(cluster, sink, mode, [], fixtures.golden("readme"))
    assert a.returncode == b.returncode
    assert a.stdout == b.stdout
    assert len(ra) == len(rb), (mode, a.stderr, b.stderr)
    assert [json.loads(r["body"]) for r in ra] == [json.loads(r["body"]) for r in rb]
    assert ra[0]["headers"]["Content-Length"] == rb[0]["headers"]["Content-Length"]
    assert ra[0]["headers"]["Content-Type"] == rb[0]["headers"]["Content-Type"] == "application/json"
    # stderr: same lines, except the exception repr inside a reset message (requests vs our transport)
    la, lb = a.stderr.splitlines(), b.stderr.splitlines()
    assert len(la) == len(lb), (a.stderr, b.stderr)
    for x, y in zip(la, lb):
        if "Connection aborted" in x or "Connection reset" in x:
            assert x.split(":")[0] == y.split(":")[0] and "Connection aborted" in y
        else:
            assert x == y


def test_slack_only_on_error_gating_matches(cluster, sink):
    for nodes, expect in ((fixtures.golden("readme"), 0), (fixtures.golden("notready"), 1), (fixtures.golden("nogpu"), 1)):
        a, b, ra, rb = _slack_case(cluster, sink, "200", ["--slack-only-on-error"], nodes)
        assert len(ra) == len(rb) == expect
        assert a.stdout == b.stdout and a.returncode == b.returncode


def test_slack_json_mode_suppresses_final_lines(cluster, sink):
    a, b, ra, rb = _slack_case(cluster, sink, "500", ["--json"], fixtures.golden("readme"))
    assert a.stdout == b.stdout
    assert a.stderr == b.stderr
    assert len(ra) == len(rb) == 4


def test_retry_count_zero_and_negative(cluster, sink):
    for n, posts in (("0", 1), ("-1", 0)):
        a, b, ra, rb = _slack_case(cluster, sink, "500", ["--slack-retry-count", n], fixtures.golden("readme"))
        assert len(ra) == len(rb) == posts
        assert a.stderr == b.stderr and a.stdout == b.stdout


def test_env_webhook_and_empty_flag_fallback(cluster, sink):
    kc = cluster(fixtures.golden("readme"))
    env = {"SLACK_WEBHOOK_URL": sink.url("200")}
    a = run_ref(["--kubeconfig", kc, "--slack-webhook", ""], env=env)
    b = run_new(["--kubeconfig", kc, "--slack-webhook", ""], env=env)
    assert a.stdout == b.stdout and a.stdout.startswith("✅ 슬랙 메시지를 성공적으로 전송했습니다.")


# --- differential fuzz: random NodeLists through the unmodified reference and this CLI -------------------------

from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402

_GPU_KEYS = ["nvidia.com/gpu", "amd.com/gpu", "gpu.intel.com/i915", "intel.com/gpu"]
_QTY = st.sampled_from(["0", "1", "2", "8", "16", "1k", "500m", "x", "-2", "007", " 3", "+4", "٣", "1_0", "",
                        "2Gi", "１"])
_TXT = st.text(alphabet=st.sampled_from(list("abz-09._/한글 \"\\") + ["é", " ", "\t"]), max_size=8)


@st.composite
def _fuzz_node(draw, i):
    node = {"metadata": None if draw(st.integers(0, 12)) == 0 else {
                "name": f"n{i}-" + draw(st.text(alphabet=st.sampled_from(list("abc-09한")), max_size=6)),
                "labels": draw(st.one_of(st.none(), st.dictionaries(_TXT, _TXT, max_size=3)))},
            "spec": {"taints": draw(st.one_of(st.none(), st.lists(st.fixed_dictionaries({
                "key": _TXT, "value": st.one_of(st.none(), _TXT),
                "effect": st.sampled_from(["NoSchedule", "NoExecute", "PreferNoSchedule"])}), max_size=2)))},
            "status": None if draw(st.integers(0, 15)) == 0 else {
                "capacity": draw(st.one_of(st.none(), st.dictionaries(st.sampled_from(_GPU_KEYS + ["cpu", "memory"]),
                                                                     _QTY, max_size=4))),
                "conditions": draw(st.one_of(st.none(), st.lists(st.fixed_dictionaries({
                    "type": st.sampled_from(["Ready", "MemoryPressure", "ready"]),
                    "status": st.sampled_from(["True", "False", "Unknown", "true"])}), max_size=3)))}}
    return node


@st.composite
def _fuzz_cluster(draw):
    n = draw(st.integers(0, 5))
    return [draw(_fuzz_node(i)) for i in range(n)]


@settings(max_examples=int(os.environ.get("K8SGPU_FUZZ_EXAMPLES", "25")), deadline=None,
          suppress_health_check=list(HealthCheck))
@given(_fuzz_cluster(), st.booleans())
def test_random_clusters_byte_identical(tmp_path_factory, nodes, as_json):
    """Random NodeLists (odd quantities such as '\\u0663', ' 3', '1k', missing metadata/status/conditions,
    unicode and control characters in labels and taints, lower-case condition strings): stdout and exit code
    of the unmodified reference and of this CLI are identical."""
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import MockApiServer
    d = tmp_path_factory.mktemp("fz")
    with MockApiServer(nodes) as srv:
        kc = write_kubeconfig(str(d / "kc"), srv.url)
        flags = ["--kubeconfig", kc] + (["--json"] if as_json else [])
        a, b = run_ref(flags), run_new(flags)
    assert (a.returncode, a.stdout) == (b.returncode, b.stdout), (nodes, a.stdout, b.stdout, a.stderr[-500:],
                                                                  b.stderr[-500:])


@settings(max_examples=int(os.environ.get("K8SGPU_FUZZ_EXAMPLES", "15")), deadline=None,
          suppress_health_check=list(HealthCheck))
@given(_fuzz_cluster(), st.booleans())
def test_random_clusters_same_slack_message(tmp_path_factory, sink, nodes, only_on_error):
    """The Slack payload (text, username, icon, in requests' ASCII-escaped JSON) and the gating decision for
    random clusters, reference vs this CLI."""
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import MockApiServer
    d = tmp_path_factory.mktemp("fzs")
    with MockApiServer(nodes) as srv:
        kc = write_kubeconfig(str(d / "kc"), srv.url)
        flags = ["--kubeconfig", kc, "--slack-webhook", sink.url("200"), "--slack-username", "fuzz-bot"] + \
            (["--slack-only-on-error"] if only_on_error else [])
        n0 = len(sink.requests)
        a = run_ref(flags)
        n1 = len(sink.requests)
        b = run_new(flags)
        n2 = len(sink.requests)
    ra, rb = sink.requests[n0:n1], sink.requests[n1:n2]
    assert (a.returncode, a.stdout) == (b.returncode, b.stdout)
    assert len(ra) == len(rb) <= 1
    assert [r["body"] for r in ra] == [r["body"] for r in rb]


_STEP = st.sampled_from(["200", "500", "204", "404", "429", "reset", "close"])


@settings(max_examples=int(os.environ.get("K8SGPU_FUZZ_EXAMPLES", "15")), deadline=None,
          suppress_health_check=list(HealthCheck))
@given(st.lists(_STEP, min_size=1, max_size=5), st.integers(-1, 3), st.booleans())
def test_random_webhook_behaviour_same_retry_state_machine(tmp_path_factory, sink, steps, retries, as_json):
    """Scripted webhook answers (any mix of 200 / 204 / 404 / 429 / 500 / TCP reset / close without a
    response) and retry counts: with ``--slack-retry-policy reference`` both programs make the same number of
    POSTs with the same bodies, print the same stdout and the same stderr lines (modulo the transport's
    exception text inside a connection-error line) and exit the same way."""
    import uuid
    d = tmp_path_factory.mktemp("fzw")
    kc = None
    from k8s_gpu_node_checker_amd.testing.mock_apiserver import MockApiServer
    with MockApiServer(fixtures.golden("readme")) as srv:
        kc = write_kubeconfig(str(d / "kc"), srv.url)
        script = ",".join(steps)
        common = ["--kubeconfig", kc, "--slack-retry-count", str(retries), "--slack-retry-delay", "0"] + \
            (["--json"] if as_json else [])
        tag = uuid.uuid4().hex[:8]
        a = run_ref(common + ["--slack-webhook", sink.url(f"seq/{tag}-a/{script}")])
        b = run_new(common + ["--slack-webhook", sink.url(f"seq/{tag}-b/{script}"), "--slack-retry-policy", "reference"])
    ra = [r for r in sink.requests if f"/{tag}-a/" in r["path"]]
    rb = [r for r in sink.requests if f"/{tag}-b/" in r["path"]]
    assert (a.returncode, a.stdout) == (b.returncode, b.stdout), (steps, retries, a.stderr, b.stderr)
    assert len(ra) == len(rb), (steps, retries, a.stderr, b.stderr)
    assert [r["body"] for r in ra] == [r["body"] for r in rb]
    la, lb = a.stderr.splitlines(), b.stderr.splitlines()
    assert len(la) == len(lb), (steps, retries, a.stderr, b.stderr)
    for x, y in zip(la, lb):
        if "Connection aborted" in x or "Connection reset" in x or "RemoteDisconnected" in x:
            assert x.split(":")[0] == y.split(":")[0], (x, y)
        else:
            assert x == y, (steps, retries, x, y)


# --- the Slack transport: what requests.post does beyond a plain POST -------------------------

def _seq(reqs):
    return [(r["method"], r["path"], [(k, v) for k, v in r["headers"].items() if k not in ("User-Agent", "Host")],
             r["body"]) for r in reqs]


def _transport_case(cluster, sink, url, env=None, flags=()):
    kc = cluster(fixtures.golden("readme"))
    args = ["--kubeconfig", kc, "--slack-webhook", url, "--slack-retry-delay", "0"] + list(flags)
    e = {"HOME": "/nonexistent-home"}
    e.update(env or {})
    n0 = len(sink.requests)
    a = run_ref(args, env=e)
    n1 = len(sink.requests)
    b = run_new(args + ["--slack-retry-policy", "reference"], env=e)
    n2 = len(sink.requests)
    return a, b, _seq(sink.requests[n0:n1]), _seq(sink.requests[n1:n2])


@pytest.mark.parametrize("mode", ["301", "302", "303", "307", "308", "loop", "cookie", "to/localhost/200"])
@pytest.mark.parametrize("flags", [[], ["--json"]])
def test_slack_redirects_identical(cluster, sink, mode, flags):
    a, b, ra, rb = _transport_case(cluster, sink, sink.url(mode), flags=flags)
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert ra == rb and ra
    if mode in ("307", "308"):
        assert "✅ 슬랙 메시지를 성공적으로 전송했습니다." in a.stdout or flags


@pytest.mark.parametrize("mode", [
    "loc/302/",                                  # a redirect status without a Location: the 3xx is the answer
    "loc/307/postonly%3Fa%3D1%26b",              # relative, with a query
    "loc/308/%2F%2F127.0.0.1%3A{port}%2F200",    # scheme-relative
    "loc/307/..%2F..%2F200",                     # dot segments above the root
    "loc/301/%2F200%23frag",                     # a fragment (not sent)
    "loc/307/%2F200%3Fq%3D%25E2%259C%2585",      # a percent-encoded query kept as is
    "loc/307/%2Fp%C3%A4th",                      # a raw non-ASCII path (requests re-quotes it)
    "loc/302/ftp%3A%2F%2Fexample.invalid%2Fx",   # a scheme requests has no adapter for
    "loc/307/http%3A%2F%2F127.0.0.1%3A1%2F200",  # a refused connection after the hop
    "loc/303/%2F307",                            # 303 -> GET, then 307 keeps the GET
    "loc/200/%2F500",                            # a Location on a success is not followed
    "locb/307/%2Fp%E4th",                        # a Location that is not UTF-8 (requests' decode error)
    "locb/302/%2F200%FF",
    "locb/307/%2Fp%C3%A4th",                     # raw UTF-8 bytes
])
def test_slack_redirect_targets_identical(cluster, sink, mode):
    port = sink.server_address[1]
    a, b, ra, rb = _transport_case(cluster, sink, sink.url(mode.replace("{port}", str(port))))
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert ra == rb and ra


def _undate(text):
    return re.sub(r"'Date': '[^']*'", "'Date': D", text)


@pytest.mark.parametrize("status", [403, 404, 500])
@pytest.mark.parametrize("flags", [[], ["--json"]])
def test_apiserver_error_status_identical(tmp_path, mock_cluster, status, flags):
    """A LIST answered 403 / 404 / 500: the reference prints the client's ApiException (status, reason, headers,
    body) after `에러: ` (or as the JSON `error`) and exits 1; so does the CLI.  Only the Date header may differ."""
    srv = mock_cluster(fixtures.golden("readme"), status=status)
    kc = write_kubeconfig(str(tmp_path / "kc.yaml"), srv.url)
    a, b = run_ref(["--kubeconfig", kc] + flags), run_new(["--kubeconfig", kc] + flags)
    assert (a.returncode, _undate(a.stdout)) == (b.returncode, _undate(b.stdout)) and a.returncode == 1
    # stderr: identical up to the traceback the text mode prints (its frames name each program's own code)
    ta, tb = a.stderr.split("Traceback"), b.stderr.split("Traceback")
    assert _undate(ta[0]) == _undate(tb[0]) and len(ta) == len(tb)
    if len(ta) > 1:  # the exception's own line: same text after the type name
        assert ta[-1].strip().splitlines()[-1].split(":", 1)[1] == tb[-1].strip().splitlines()[-1].split(":", 1)[1]


def test_apiserver_refused_same_message(tmp_path):
    """No apiserver: both end in an uncaught connection error (exit 1) whose message is urllib3's MaxRetryError
    text; the CLI's URL carries its page size (`?limit=500`, PARITY.md: paging)."""
    kc = write_kubeconfig(str(tmp_path / "kc.yaml"), "http://127.0.0.1:1")
    a, b = run_ref(["--kubeconfig", kc]), run_new(["--kubeconfig", kc])
    assert (a.returncode, a.stdout) == (b.returncode, b.stdout) == (1, "")
    ma = a.stderr.strip().splitlines()[-1].split(": ", 1)[1]
    mb = b.stderr.strip().splitlines()[-1].split(": ", 1)[1]
    assert mb == ma.replace("/api/v1/nodes ", "/api/v1/nodes?limit=500 ")
    assert "Caused by NewConnectionError(" in mb and mb.count("Max retries exceeded") == 1


@pytest.mark.parametrize("url,env", [
    ("http://example.invalid/200", {"HTTP_PROXY": "SINK"}),
    ("http://example.invalid/200", {"http_proxy": "SINK"}),
    ("http://user:pw@example.invalid/200", {"HTTP_PROXY": "SINK"}),   # origin credentials travel to the proxy
    ("http://example.invalid/200", {"ALL_PROXY": "SINK"}),
    ("http://example.invalid:8080/200", {"HTTP_PROXY": "SINK", "NO_PROXY": "example.invalid"}),  # bypassed
])
def test_slack_env_proxies_identical(cluster, sink, url, env):
    """requests' env proxies: the sink is the proxy (it logs the absolute-form target); 127.0.0.1 (the mock
    apiserver, which the reference's stand-in client also reaches through requests) is always in NO_PROXY."""
    e = {k: sink.base_url if v == "SINK" else v for k, v in env.items()}
    e["NO_PROXY"] = ",".join(["127.0.0.1"] + ([e["NO_PROXY"]] if "NO_PROXY" in e else []))
    a, b, ra, rb = _transport_case(cluster, sink, url, env=e)
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert ra == rb


@pytest.mark.parametrize("kind", ["gzip", "deflate", "chunked", "euckr", "latin", "nolength", "octet", "badgzip",
                                  "baddeflate"])
def test_slack_error_body_decoding_identical(cluster, sink, kind):
    """A 500 whose body is compressed, chunked, in another charset, unlabelled or unbounded: the same
    `(HTTP 500): <text>` line (requests decodes Content-Encoding and picks the charset as `Response.text`); one
    labelled compressed but sent plain: requests' ContentDecodingError line, not retried."""
    a, b, ra, rb = _transport_case(cluster, sink, sink.url("body/" + kind), flags=["--slack-retry-count", "1"])
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert ra == rb
    if kind.startswith("bad"):  # requests' ContentDecodingError: one failure line, no retry
        assert len(rb) == 1 and "but failed to decode it." in b.stderr
    else:
        assert ra == rb and "(HTTP 500): " in b.stderr


@pytest.mark.parametrize("kind", ["badstatus", "notahttp", "status99", "longstatus", "longheader", "manyheaders",
                                  "justenoughheaders", "truncated", "badchunk", "truncatedchunk", "prematurechunk",
                                  "chunkext", "twolengths", "samecl", "badcl", "continue", "http10", "empty200",
                                  "resetbody"])
def test_slack_malformed_responses_identical(cluster, sink, kind):
    """Responses that break HTTP one way each: the head http.client refuses ('Connection aborted.', retried), a
    body cut short or badly chunked ('Connection broken: …', not retried), unmatching or invalid lengths, and
    the unusual-but-valid ones (100 Continue, HTTP/1.0, an empty 200)."""
    a, b, ra, rb = _transport_case(cluster, sink, sink.url("raw/" + kind), flags=["--slack-retry-count", "1"])
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert ra == rb


def test_slack_read_timeout_identical(cluster):
    """A webhook slower than requests' 10 s timeout: the same `Read timed out. (read timeout=10)` line (one
    attempt each: about 20 s)."""
    with WebhookSink(slow_s=10.6) as slow:
        a, b, ra, rb = _transport_case(cluster, slow, slow.url("slow"), flags=["--slack-retry-count", "0"])
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert ra == rb and len(ra) == 1 and "Read timed out. (read timeout=10)" in b.stderr


@pytest.mark.parametrize("tmpl", [
    "{b}/200 ", "{b}/2 00", "{b}/200\n", "{b}/200\t", "HTTP://{hp}/200", "{b}", "{b}?x=1", "{b}/200#frag",
    "http://user@{hp}/200", "http://:pw@{hp}/200", "{b}/%zz", "{b}/ä", "  {b}/200", "http://{hp}:/200",
    "http://{hp}/../200", "http:/{hp}/200", "http:{hp}/200", "//{hp}/200", "{hp}/200", "http://{hp}/200?a=%",
    "http://{hp}/a b?c d"])
def test_slack_odd_webhook_urls_identical(cluster, sink, tmpl):
    """Webhook URLs with blanks, control characters, case, missing parts, bad escapes and non-ASCII: requests'
    URL preparation decides where the POST goes (or which error it is), and the CLI decides the same."""
    host, port = sink.server_address[:2]
    url = tmpl.format(b=f"http://{host}:{port}", hp=f"{host}:{port}")
    a, b, ra, rb = _transport_case(cluster, sink, url, flags=["--slack-retry-count", "0"])
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert ra == rb


def test_slack_https_to_a_plain_http_port_identical(cluster, sink):
    """https to a port that speaks plain HTTP: the handshake never completes; requests reports the 10 s socket
    timeout as `Read timed out.` (one attempt each: about 20 s)."""
    host, port = sink.server_address[:2]
    a, b, ra, rb = _transport_case(cluster, sink, f"hTTps://{host}:{port}/200", flags=["--slack-retry-count", "0"])
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert "Read timed out. (read timeout=10)" in b.stderr


class _TLSSink(WebhookSink):
    """The webhook sink behind TLS with the session's self-signed certificate (127.0.0.1 / localhost)."""

    def __init__(self, crt, key):
        super().__init__()
        self.ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        self.ctx.load_cert_chain(crt, key)

    def get_request(self):
        s, addr = super().get_request()
        try:
            return self.ctx.wrap_socket(s, server_side=True), addr
        except (OSError, ssl.SSLError):
            s.close()
            raise


@pytest.fixture
def tls_sink(certs):
    s = _TLSSink(*certs).start()
    yield s
    s.stop()


@pytest.mark.parametrize("host,env", [("127.0.0.1", "REQUESTS_CA_BUNDLE"), ("localhost", "REQUESTS_CA_BUNDLE"),
                                      ("127.0.0.1", None), ("127.0.0.1", "CURL_CA_BUNDLE"),
                                      ("127.0.0.1", "SSL_CERT_FILE")])
def test_slack_https_verification_identical(cluster, tls_sink, certs, host, env):
    """An https webhook: verified against the bundle requests would use (its env variables, else certifi), the
    same success or the same `CERTIFICATE_VERIFY_FAILED` line."""
    url = f"https://{host}:{tls_sink.server_address[1]}/200"
    a, b, ra, rb = _transport_case(cluster, tls_sink, url, env={env: certs[0]} if env else None)
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert ra == rb
    if env == "REQUESTS_CA_BUNDLE":
        assert ra and "✅ 슬랙 메시지를 성공적으로 전송했습니다." in b.stdout
    elif env is None:
        assert not ra and "CERTIFICATE_VERIFY_FAILED" in b.stderr


@pytest.mark.parametrize("proxy,url", [
    ("HTTPS_PROXY=SINK", "https://example.invalid/200"),               # CONNECT refused by the proxy (404)
    ("https_proxy=SINK", "https://example.invalid/200"),
    ("HTTPS_PROXY=http://127.0.0.1:1", "https://example.invalid/200"),  # the proxy itself refuses
    ("HTTP_PROXY=http://127.0.0.1:1", "http://example.invalid:8080/a/b?c=d"),
    ("HTTPS_PROXY=http://no-such-proxy.invalid:3128", "https://example.invalid/200"),  # the proxy does not resolve
    ("HTTP_PROXY=http://no-such-proxy.invalid:3128", "http://example.invalid/200"),
])
def test_slack_proxy_failures_identical(cluster, sink, proxy, url):
    """A proxy that refuses the tunnel, refuses the connection or does not resolve: urllib3's ProxyError text,
    under the target's pool for a tunnel and the proxy's own pool (absolute URL) for a forwarded request."""
    k, v = proxy.split("=", 1)
    e = {k: sink.base_url if v == "SINK" else v, "NO_PROXY": "127.0.0.1"}
    a, b, ra, rb = _transport_case(cluster, sink, url, env=e, flags=["--slack-retry-count", "0"])
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert ra == rb and "ProxyError('Unable to connect to proxy', " in b.stderr


def test_slack_url_credentials_identical(cluster, sink, tmp_path):
    host, port = sink.server_address[:2]
    for url in (f"http://user:pass@{host}:{port}/200", f"http://us%40er:p%3Ass@{host}:{port}/to/localhost/200"):
        a, b, ra, rb = _transport_case(cluster, sink, url)
        assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
        assert ra == rb
        if "user:pass" in url:
            assert ("Authorization", "Basic dXNlcjpwYXNz") in rb[0][2]
        else:  # the cross-host hop drops the credentials
            assert any(k == "Authorization" for k, _ in rb[0][2]) and all(k != "Authorization" for k, _ in rb[1][2])
    rc = tmp_path / "netrc"
    rc.write_text(f"machine {host} login nu password np\n")
    a, b, ra, rb = _transport_case(cluster, sink, f"http://{host}:{port}/200", env={"NETRC": str(rc)})
    assert (a.stdout, a.stderr) == (b.stdout, b.stderr) and ra == rb
    assert ("Authorization", "Basic bnU6bnA=") in rb[0][2]


@pytest.mark.parametrize("url,env", [("http://127.0.0.1:99999/x", None), ("http://[::1/x", None),
                                     ("https://127.0.0.1:1/x", {"REQUESTS_CA_BUNDLE": "/missing"}),
                                     ("http://127.0.0.1:1/x", None), ("ftp://x/y", None)])
@pytest.mark.parametrize("flags", [[], ["--json"]])
def test_slack_transport_errors_identical(cluster, sink, url, env, flags):
    """A malformed URL, a refused connection or a bad CA bundle: one failure line, never a thread traceback."""
    a, b, ra, rb = _transport_case(cluster, sink, url, env=env, flags=flags)
    assert (a.returncode, a.stdout, a.stderr) == (b.returncode, b.stdout, b.stderr)
    assert "Traceback" not in b.stderr and b.stderr.startswith("슬랙 메시지 전송 실패: ")


# --- argparse prefix matching: hidden extension flags must not make a reference abbreviation ambiguous ----------

@pytest.mark.parametrize("args", [
    ["--js"], ["--jso"], ["--kube", "MISSING"], ["--kubec=MISSING", "--json"], ["--slack-o", "--json"], ["--he"],
    ["--h"], ["--slack"], ["--slack-retry"], ["--slack-retry=3"], ["--slack-u", "x", "--js"], ["--json", "--js"],
    ["--slack-username", "--js"], ["--sl", "--json"], ["--k"], ["--j"], ["--", "--js"], ["--slack-w"],
    ["--slack-retry-c", "x"], ["--jsonx"], ["-j"], ["--json=1"]])
def test_abbreviations_behave_as_in_the_reference(args, tmp_path):
    args = [str(tmp_path / "missing") if a == "MISSING" else a for a in args]
    a, b = run_ref(args, cwd=str(tmp_path)), run_new(args, cwd=str(tmp_path))
    assert (a.returncode, a.stdout) == (b.returncode, b.stdout), (a.stderr, b.stderr)
    # stderr: identical, except the traceback frames of the kubeconfig error (the code that raised differs)
    ta, tb = a.stderr.split("Traceback")[0], b.stderr.split("Traceback")[0]
    assert ta == tb
