"""Event-driven monitoring: streaming HTTP reader, the mock apiserver's watch, NodeWatcher, --watch-events."""
import json
import os
import socket
import subprocess
import sys
import threading
import time

import pytest

from k8s_gpu_node_checker_amd.checker import CheckOptions, CheckResult, apply_health
from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
from k8s_gpu_node_checker_amd.kube.watch import NodeWatcher, outcome_signature
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
from k8s_gpu_node_checker_amd.utils.http import Connection, LineStream
from k8s_gpu_node_checker_amd.utils.timing import NullTracer

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _raw_server(script):
    """One-connection TCP server that plays ``script``: a list of bytes (sent) / floats (sleep)."""
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)

    def run():
        c, _ = srv.accept()
        buf = b""
        while b"\r\n\r\n" not in buf:
            buf += c.recv(4096)
        for step in script:
            if isinstance(step, float):
                time.sleep(step)
            else:
                c.sendall(step)
        time.sleep(0.2)
        c.close()
        srv.close()
    threading.Thread(target=run, daemon=True).start()
    return f"http://127.0.0.1:{srv.getsockname()[1]}"


def test_line_stream_chunked_split_records_idle_and_eof():
    head = b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\nContent-Type: application/json\r\n\r\n"
    rec1, rec2 = b'{"a": 1}\n', b'{"b": 2}\n'
    script = [head, b"%x\r\n" % len(rec1) + rec1[:4], 0.05, rec1[4:] + b"\r\n",
              # one chunk carrying the second record split across two chunks, then an idle gap
              b"3\r\n" + rec2[:3] + b"\r\n", b"%x\r\n" % (len(rec2) - 3) + rec2[3:] + b"\r\n", 0.6,
              b"0\r\n\r\n"]
    url = _raw_server(script)
    conn = Connection(url, timeout=5)
    st = conn.open_stream("GET", "/w", {}, read_timeout=0.3)
    assert isinstance(st, LineStream) and st.status == 200
    assert st.next_line() == rec1.strip()
    assert st.next_line() == rec2.strip()
    assert st.next_line() is None  # idle for longer than the read timeout: not an error
    conn.sock.settimeout(5)
    try:
        st.next_line()
        raise AssertionError("expected EOF")
    except EOFError:
        pass
    conn.close()


def test_line_stream_non_2xx_returns_full_response():
    body = b'{"kind":"Status","code":403}'
    url = _raw_server([b"HTTP/1.1 403 Forbidden\r\nContent-Length: %d\r\n\r\n" % len(body) + body])
    c = Connection(url, timeout=5)
    r = c.open_stream("GET", "/w", {})
    assert not isinstance(r, LineStream) and r.status == 403 and r.body == body
    c.close()


def _watch_lines(url, rv, n, extra="", timeout=5.0):
    conn = Connection(url, timeout=timeout)
    st = conn.open_stream("GET", f"/api/v1/nodes?watch=1&resourceVersion={rv}{extra}", {})
    out = []
    while len(out) < n:
        line = st.next_line()
        if line is None:
            break
        out.append(json.loads(line))
    conn.close()
    return out


def test_mock_apiserver_watch_events_bookmarks_and_410(mock_cluster):
    srv = mock_cluster(fixtures.cluster(3, "amd", gpus_per_node=8), bookmark_interval=0.2)
    rv = srv.state.rv
    got = []
    t = threading.Thread(target=lambda: got.extend(_watch_lines(srv.url, rv, 3, "&timeoutSeconds=5")))
    t.start()
    time.sleep(0.2)
    srv.state.patch("mi355x-node-0001", {"metadata": {"labels": {"x": "y"}}})
    srv.state.delete_node("mi355x-node-0002")
    srv.state.add_node(fixtures.realistic_node("mi355x-node-0009"))
    t.join(10)
    assert [e["type"] for e in got] == ["MODIFIED", "DELETED", "ADDED"]
    assert got[0]["object"]["metadata"]["labels"]["x"] == "y"
    rvs = [int(e["object"]["metadata"]["resourceVersion"]) for e in got]
    assert rvs == sorted(rvs) and rvs[0] > rv
    # bookmarks while idle
    bm = _watch_lines(srv.url, srv.state.rv, 1, "&allowWatchBookmarks=true&timeoutSeconds=3")
    assert bm and bm[0]["type"] == "BOOKMARK" and int(bm[0]["object"]["metadata"]["resourceVersion"]) >= rvs[-1]
    # "0": the current state as ADDED events
    init = _watch_lines(srv.url, 0, 3, "&timeoutSeconds=1")
    assert [e["type"] for e in init] == ["ADDED"] * 3
    # a resourceVersion older than the event log: ERROR 410
    srv.state.EVENT_LOG = 1
    srv.state.patch("mi355x-node-0000", {"metadata": {"labels": {"z": "1"}}})
    srv.state.patch("mi355x-node-0000", {"metadata": {"labels": {"z": "2"}}})
    err = _watch_lines(srv.url, rv, 1, "&timeoutSeconds=1")
    assert err[0]["type"] == "ERROR" and err[0]["object"]["code"] == 410


def test_node_view_and_apply_semantics():
    opts = CheckOptions()
    w = NodeWatcher(ClusterConnection("http://127.0.0.1:1"), opts)
    w.apply({"type": "ADDED", "object": fixtures.realistic_node("b", gpu_count=2, index=1)})
    w.apply({"type": "ADDED", "object": fixtures.realistic_node("a", gpu_count=1)})
    w.apply({"type": "ADDED", "object": fixtures.realistic_node("cpu", gpu_key=None)})
    scan = w.view.scan_result()
    assert [n["name"] for n in scan.gpu_nodes] == ["a", "b"] and scan.items_seen == 3
    # a GPU node losing its GPUs leaves the GPU view, a deletion leaves both
    w.apply({"type": "MODIFIED", "object": fixtures.realistic_node("b", gpu_key=None)})
    w.apply({"type": "DELETED", "object": fixtures.realistic_node("cpu", gpu_key=None)})
    scan = w.view.scan_result()
    assert [n["name"] for n in scan.gpu_nodes] == ["a"] and scan.items_seen == 2
    w.apply({"type": "BOOKMARK", "object": {"metadata": {"resourceVersion": "77"}}})
    assert w.rv == "77"
    assert w.apply({"type": "ERROR", "object": {"code": 410}}) is False and w.rv is None
    # copies: gating one result does not leak into the stored view
    scan.gpu_nodes[0]["ready"] = False
    assert w.view.scan_result().gpu_nodes[0]["ready"] is True


def test_native_relist_view_matches_the_event_path_and_counts_unnamed_nodes(mock_cluster):
    """The relist scans pages natively (the one-shot check's scanner) and so learns the GPU nodes and the item
    count, not the CPU nodes' names: the view equals the one built node by node through upserts, and the count
    stays right as unnamed CPU nodes are modified (no double count), deleted, and new ones added."""
    from k8s_gpu_node_checker_amd.kube.client import KubeClient
    from k8s_gpu_node_checker_amd.kube.watch import NodeView, list_resource_version
    nodes = fixtures.cluster(7, "mixed", not_ready=range(2), with_health=True, gpus_per_node=8)
    nodes += [fixtures.realistic_node(f"cpu-{i}", gpu_key=None, index=100 + i) for i in range(3)]
    srv = mock_cluster(nodes)
    opts = CheckOptions(json=True)
    w = NodeWatcher(ClusterConnection(srv.url), opts, page_size=4)
    with KubeClient(ClusterConnection(srv.url)) as kc:
        w.relist(kc)
    assert w.rv is not None and w.rv == str(srv.state.rv)
    ref = NodeView(opts.gpu_source, 1)
    for n in nodes:
        ref.upsert(n)
    a, b = w.view.scan_result(), ref.scan_result()
    assert a.gpu_nodes == b.gpu_nodes and a.ready_gpu_nodes == b.ready_gpu_nodes
    assert [ex.health_condition for ex in a.extras] == [ex.health_condition for ex in b.extras]
    assert a.items_seen == b.items_seen == len(nodes) and w.view.unnamed == 3 + (len(nodes) - 3 - len(a.gpu_nodes))
    w.apply({"type": "MODIFIED", "object": fixtures.realistic_node("cpu-0", gpu_key=None, index=100)})
    assert w.view.scan_result().items_seen == len(nodes)  # named now, not counted twice
    w.apply({"type": "DELETED", "object": fixtures.realistic_node("cpu-1", gpu_key=None, index=101)})
    w.apply({"type": "DELETED", "object": fixtures.realistic_node("cpu-0", gpu_key=None, index=100)})
    w.apply({"type": "ADDED", "object": fixtures.realistic_node("cpu-9", gpu_key=None, index=109)})
    assert w.view.scan_result().items_seen == len(nodes) - 1
    # the list's resourceVersion, with metadata before items or (a proxy's re-encoding) after them
    assert list_resource_version(b'{"kind":"NodeList","metadata":{"resourceVersion":"42","continue":"x"},"items":[]}') == "42"
    assert list_resource_version(b'{"items":[{"metadata":{"resourceVersion":"1"}}],"metadata":{"resourceVersion":"43"}}') == "43"


def _set_ready(srv, name, ready):
    node = srv.state.find(name)
    conds = [dict(c) for c in node["status"]["conditions"]]
    for c in conds:
        if c["type"] == "Ready":
            c["status"] = "True" if ready else "False"
    srv.state.patch(name, {"status": {"conditions": conds}})


def test_node_watcher_reports_only_changes(mock_cluster):
    srv = mock_cluster(fixtures.cluster(3, "amd", gpus_per_node=8, with_health=True), bookmark_interval=0.3)
    opts = CheckOptions(json=True)
    reports = []

    def evaluate(scan):
        return CheckResult(scan, apply_health(scan, opts, NullTracer()), NullTracer())

    w = NodeWatcher(ClusterConnection(srv.url), opts, watch_timeout=2, debounce=0.1)
    t = threading.Thread(target=lambda: w.run(evaluate, reports.append, duration=4.0))
    t.start()
    time.sleep(0.5)
    srv.state.patch("mi355x-node-0000", {"metadata": {"labels": {"unrelated": "change"}}})  # no report
    time.sleep(0.4)
    _set_ready(srv, "mi355x-node-0001", False)  # report 2
    time.sleep(0.4)
    srv.state.delete_node("mi355x-node-0002")  # report 3
    time.sleep(0.4)
    for i in range(3, 6):  # a burst inside the debounce window: one report
        srv.state.add_node(fixtures.realistic_node(f"mi355x-node-{i:04d}", gpu_count=8, index=i))
    t.join(15)
    assert [len(r.ready_gpu_nodes) for r in reports] == [3, 2, 1, 4], [len(r.ready_gpu_nodes) for r in reports]
    assert [r.exit_code for r in reports] == [0, 0, 0, 0]
    assert [n["name"] for n in reports[-1].gpu_nodes] == [f"mi355x-node-{i:04d}" for i in (0, 1, 3, 4, 5)]
    assert len({outcome_signature(r) for r in reports}) == 4
    assert w.relists == 1  # watch re-opened after each timeoutSeconds without a new LIST


def test_node_watcher_relists_after_410(mock_cluster):
    srv = mock_cluster(fixtures.cluster(2, "amd", gpus_per_node=8))
    opts = CheckOptions(json=True, health_policy="off")
    w = NodeWatcher(ClusterConnection(srv.url), opts, watch_timeout=1, debounce=0.05)
    w.rv = "1"  # far older than the log once it is trimmed
    srv.state.EVENT_LOG = 1
    srv.state.patch("mi355x-node-0000", {"metadata": {"labels": {"a": "1"}}})
    srv.state.patch("mi355x-node-0000", {"metadata": {"labels": {"a": "2"}}})
    reports = []
    w.run(lambda scan: CheckResult(scan, [], NullTracer()), reports.append, duration=1.5)
    assert w.relists >= 1 and reports and len(reports[0].gpu_nodes) == 2


def test_cli_watch_events_json(mock_cluster, tmp_path):
    srv = mock_cluster(fixtures.golden("readme"), bookmark_interval=0.2)
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    env = {k: v for k, v in os.environ.items() if k not in ("SLACK_WEBHOOK_URL", "KUBECONFIG")}
    p = subprocess.Popen([sys.executable, os.path.join(REPO, "check-gpu-node.py"), "--kubeconfig", kc, "--json",
                          "--watch-events", "--watch-count", "2", "--watch-duration", "20",
                          "--watch-debounce", "0.1"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         env=env, cwd=str(tmp_path))
    first = []
    while True:
        line = p.stdout.readline()
        assert line, p.stderr.read()
        first.append(line)
        if line == "}\n":
            break
    assert json.loads("".join(first))["ready_nodes"] == 2
    srv.state.set_nodes(fixtures.golden("notready"))
    out, err = p.communicate(timeout=30)
    assert p.returncode == 3, err
    second = json.loads(out)
    assert second["ready_nodes"] == 0 and second["total_nodes"] >= 1


def test_node_watcher_notices_a_heartbeat_going_stale_without_events(mock_cluster):
    """An agent that stops publishing sends no watch event; its AMDGPUHealthy heartbeat only ages.
    The watcher re-evaluates a quiet cluster every ``recheck`` s, so the stale verdict is reported."""
    from k8s_gpu_node_checker_amd.models import health as H
    rep = fixtures.mi355x_probe_report("n", gpus=8)
    cond = fixtures.health_condition(rep, 8)
    # fresh for 1-2 more seconds (max age 2 s; the timestamp has whole seconds), stale within the 6 s run
    cond["lastHeartbeatTime"] = H.format_k8s_time(time.time())
    srv = mock_cluster([fixtures.realistic_node("n", extra_conditions=[cond])])
    opts = CheckOptions(json=True)
    opts.health_policy, opts.probe_max_age, opts.probe_unknown = "require", 2.0, "deny"
    reports = []

    def evaluate(scan):
        return CheckResult(scan, apply_health(scan, opts, NullTracer()), NullTracer())
    w = NodeWatcher(ClusterConnection(srv.url), opts, watch_timeout=30, debounce=0.05, recheck=0.2)
    w.run(evaluate, reports.append, max_reports=2, duration=6.0)
    assert [r.exit_code for r in reports] == [0, 3]
    assert [r.verdicts[0].state for r in reports] == ["healthy", "unknown"]
    assert w.events == 0  # nothing arrived on the stream: the second report came from the recheck


def test_cli_watch_events_slack_on_node_change(mock_cluster, sink, tmp_path):
    """The shipped watcher's flags: one node of three going NotReady (exit stays 0) is one Slack POST, its
    recovery one more; the first report of a healthy cluster sends nothing."""
    srv = mock_cluster(fixtures.cluster(3, "amd", gpus_per_node=8, with_health=True), bookmark_interval=0.2)
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    env = {k: v for k, v in os.environ.items() if k not in ("SLACK_WEBHOOK_URL", "KUBECONFIG")}
    env["SLACK_WEBHOOK_URL"] = sink.url("200")
    p = subprocess.Popen([sys.executable, os.path.join(REPO, "check-gpu-node.py"), "--kubeconfig", kc, "--json",
                          "--watch-events", "--slack-only-on-error", "--slack-on-node-change", "--watch-count", "3",
                          "--watch-duration", "30", "--watch-debounce", "0.1"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, cwd=str(tmp_path))

    def next_report():
        lines = []
        while True:
            line = p.stdout.readline()
            assert line, p.stderr.read()
            lines.append(line)
            if line == "}\n":
                return json.loads("".join(lines))
    assert next_report()["ready_nodes"] == 3
    time.sleep(0.3)
    assert len(sink.requests) == 0
    _set_ready(srv, "mi355x-node-0001", False)
    assert next_report()["ready_nodes"] == 2
    time.sleep(0.3)
    assert len(sink.requests) == 1
    _set_ready(srv, "mi355x-node-0001", True)
    p.communicate(timeout=30)
    assert p.returncode == 0
    assert len(sink.requests) == 2


def _scrape(port):
    from k8s_gpu_node_checker_amd.utils.http import request
    from prometheus_client.parser import text_string_to_metric_families
    r = request(f"http://127.0.0.1:{port}/metrics")
    assert r.status == 200
    return {s.name: s for f in text_string_to_metric_families(r.text) for s in f.samples
            if not s.labels}, r.text


def test_watcher_serves_metrics_that_follow_watch_events(mock_cluster, tmp_path):
    """deploy/watcher.yaml's metrics endpoint (--metrics-listen): the ready-node gauge changes after a watch
    event, without a textfile in between."""
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    srv = mock_cluster(fixtures.golden("readme"), bookmark_interval=0.2)
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    env = {k: v for k, v in os.environ.items() if k not in ("SLACK_WEBHOOK_URL", "KUBECONFIG")}
    p = subprocess.Popen([sys.executable, os.path.join(REPO, "check-gpu-node.py"), "--kubeconfig", kc, "--json",
                          "--watch-events", "--watch-duration", "30", "--watch-debounce", "0.1",
                          "--metrics-listen", f"127.0.0.1:{port}"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, env=env, cwd=str(tmp_path))
    try:
        def ready():
            try:
                return _scrape(port)[0].get("k8s_gpu_checker_ready_gpu_nodes")
            except Exception:  # not listening yet
                return None
        t0 = time.monotonic()
        while time.monotonic() - t0 < 20 and (ready() is None or ready().value != 2):
            time.sleep(0.1)
        samples, text = _scrape(port)
        assert samples["k8s_gpu_checker_ready_gpu_nodes"].value == 2 and samples["k8s_gpu_checker_exit_code"].value == 0
        assert 'k8s_gpu_checker_node_ready{node="gpu-node-1"} 1' in text
        assert "k8s_gpu_checker_leader" not in text  # no --leader-elect: no leader gauge
        srv.state.set_nodes(fixtures.golden("notready"))
        t0 = time.monotonic()
        while time.monotonic() - t0 < 20 and ready().value != 0:
            time.sleep(0.1)
        samples, text = _scrape(port)
        assert samples["k8s_gpu_checker_ready_gpu_nodes"].value == 0 and samples["k8s_gpu_checker_exit_code"].value == 3
        from k8s_gpu_node_checker_amd.utils.http import request
        assert request(f"http://127.0.0.1:{port}/healthz").status == 200
    finally:
        p.terminate()
        p.communicate(timeout=20)


def test_metrics_server_leader_gauge_and_follower_view():
    import types
    from k8s_gpu_node_checker_amd.utils import prom
    node = {"name": "n0", "ready": True, "gpus": 8, "gpu_breakdown": {"amd.com/gpu": 8}}
    res = types.SimpleNamespace(gpu_nodes=[node], ready_gpu_nodes=[node], exit_code=0, verdicts=[], tracer=None)
    srv = prom.MetricsServer("127.0.0.1", 0)
    try:
        assert srv.text() == "\n"  # nothing before the first report
        srv.set_leader(False)
        assert srv.text().splitlines()[-1] == "k8s_gpu_checker_leader 0"
        srv.set_leader(True)
        srv.update(res)
        t = srv.text()
        assert "k8s_gpu_checker_ready_gpu_nodes 1" in t and t.splitlines()[-1] == "k8s_gpu_checker_leader 1"
        srv.set_leader(False)  # lost the Lease: the cluster gauges go, a follower must not serve stale ones
        assert "k8s_gpu_checker_ready_gpu_nodes" not in srv.text()
    finally:
        srv.httpd.server_close()
    assert prom.parse_listen("0.0.0.0:9465") == ("0.0.0.0", 9465)
    assert prom.parse_listen(":9465") == ("0.0.0.0", 9465)
    assert prom.parse_listen("[::1]:9465") == ("::1", 9465)
    with pytest.raises(ValueError):
        prom.parse_listen("9465x")
