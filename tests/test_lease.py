"""Lease-based leader election (kube/lease.py) against the mock apiserver's coordination.k8s.io/v1 Leases, and
the replicated watcher built on it (``check-gpu-node --watch-events --leader-elect``)."""
import json
import os
import subprocess
import sys
import time

import pytest

from k8s_gpu_node_checker_amd.kube.client import KubeClient
from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
from k8s_gpu_node_checker_amd.kube.lease import LeaderElector
from k8s_gpu_node_checker_amd.testing import fixtures

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAST = dict(lease_duration=0.8, renew_deadline=0.5, retry_period=0.1)


def _elector(srv, ident, **kw):
    conn = ClusterConnection(srv.url)
    return LeaderElector(lambda: KubeClient(conn, timeout=2.0, retries=0), "gpu-health", "gpu-node-watcher", ident,
                         **{**FAST, **kw})


def _wait(pred, timeout=5.0):
    t = time.monotonic()
    while time.monotonic() - t < timeout:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_one_of_two_candidates_leads_and_the_other_takes_over_when_it_stops_renewing(mock_cluster):
    srv = mock_cluster(fixtures.cluster(1, "amd"))
    a = _elector(srv, "watcher-a").start()
    assert _wait(a.leading.is_set)
    b = _elector(srv, "watcher-b").start()
    try:
        time.sleep(1.5)  # well past one lease duration: a keeps renewing, so b must not take it
        assert a.is_leader() and not b.leading.is_set()
        lease = srv.leases[("gpu-health", "gpu-node-watcher")]
        assert lease["spec"]["holderIdentity"] == "watcher-a" and lease["spec"]["leaseDurationSeconds"] == 1
        # a loses the apiserver (every lease call fails): it gives leadership up at its renew deadline, and b
        # takes the Lease only after observing it unrenewed for the lease duration -- never both at once
        srv.lease_status = 500
        both = []
        t0 = time.monotonic()
        while not a.lost.is_set() and time.monotonic() - t0 < 2.0:
            both.append(a.is_leader() and b.is_leader())
            time.sleep(0.01)
        assert a.lost.is_set() and not a.is_leader() and not b.leading.is_set()
        srv.lease_status = None
        while not b.leading.is_set() and time.monotonic() - t0 < 5.0:
            both.append(a.is_leader() and b.is_leader())
            time.sleep(0.01)
        assert b.leading.is_set() and not any(both)  # never two leaders
        assert srv.leases[("gpu-health", "gpu-node-watcher")]["spec"]["holderIdentity"] == "watcher-b"
        assert srv.leases[("gpu-health", "gpu-node-watcher")]["spec"]["leaseTransitions"] == 1
    finally:
        a.stop()
        b.stop()


def test_a_stopping_leader_releases_the_lease_for_an_immediate_takeover(mock_cluster):
    srv = mock_cluster(fixtures.cluster(1, "amd"))
    # a long lease: without the release, b would wait 30 s
    a = _elector(srv, "a", lease_duration=30.0, renew_deadline=20.0, retry_period=0.1).start()
    assert _wait(a.leading.is_set)
    b = _elector(srv, "b", lease_duration=30.0, renew_deadline=20.0, retry_period=0.1).start()
    try:
        time.sleep(0.3)
        assert not b.leading.is_set()
        a.stop()
        assert srv.leases[("gpu-health", "gpu-node-watcher")]["spec"]["holderIdentity"] in ("", "b")
        assert _wait(b.leading.is_set, 3.0)
    finally:
        b.stop()


def test_concurrent_writers_resolve_by_resource_version(mock_cluster):
    """Two candidates that both read an expired Lease: the PUT carrying the stale resourceVersion gets 409, so
    exactly one wins the round."""
    srv = mock_cluster(fixtures.cluster(1, "amd"))
    conn = ClusterConnection(srv.url)
    a, b = _elector(srv, "a"), _elector(srv, "b")
    with KubeClient(conn, retries=0) as c:
        assert a.try_acquire_or_renew(c)
        lease = json.loads(c.request("GET", "/apis/coordination.k8s.io/v1/namespaces/gpu-health/leases/"
                                            "gpu-node-watcher").body)
        lease["spec"]["holderIdentity"] = "someone-else"
        stale = json.loads(json.dumps(lease))
        c.request("PUT", "/apis/coordination.k8s.io/v1/namespaces/gpu-health/leases/gpu-node-watcher",
                  json.dumps(lease).encode(), content_type="application/json", idempotent=False)
        from k8s_gpu_node_checker_amd.kube.errors import ApiException
        with pytest.raises(ApiException) as ei:
            c.request("PUT", "/apis/coordination.k8s.io/v1/namespaces/gpu-health/leases/gpu-node-watcher",
                      json.dumps(stale).encode(), content_type="application/json", idempotent=False)
        assert ei.value.status == 409
        # b sees someone-else's fresh record: not yet (it must watch it go unrenewed for the lease duration)
        assert not b.try_acquire_or_renew(c)
        b.clock = lambda: time.monotonic() + 5.0
        assert b.try_acquire_or_renew(c)
        assert srv.leases[("gpu-health", "gpu-node-watcher")]["spec"]["holderIdentity"] == "b"


def test_invalid_timings_are_refused():
    with pytest.raises(ValueError):
        LeaderElector(lambda: None, "ns", "n", "id", lease_duration=1.0, renew_deadline=2.0, retry_period=0.5)


def _watcher(kc, sink_url, ident, extra=()):
    env = dict(os.environ, PYTHONPATH=REPO, SLACK_WEBHOOK_URL=sink_url, POD_NAME=ident)
    return subprocess.Popen([sys.executable, os.path.join(REPO, "check-gpu-node.py"), "--kubeconfig", kc, "--json",
                             "--watch-events", "--watch-debounce", "0.05", "--leader-elect",
                             "--leader-elect-lease", "gpu-health/gpu-node-watcher",
                             "--leader-elect-timing", "0.8,0.5,0.1", *extra],
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)


def _holder(srv):
    return srv.leases.get(("gpu-health", "gpu-node-watcher"), {}).get("spec", {}).get("holderIdentity")


def _stdout_reports(out):
    return [json.loads(x + "\n}") for x in out.split("\n}\n") if x.strip()]


def test_replicated_watchers_report_once_and_fail_over(mock_cluster, sink, tmp_path):
    """Two watcher replicas on one Lease: only the leader reports (one Slack message); when it stops, the
    other takes over, reports the cluster from its own LIST on stdout -- and does not repeat the Slack message
    the old leader delivered (the last-notified outcome is on the Lease)."""
    srv = mock_cluster(fixtures.cluster(2, "amd"))
    kc = srv.kubeconfig(str(tmp_path / "kc"))
    a = _watcher(kc, sink.url("200"), "replica-a")
    try:
        assert _wait(lambda: _holder(srv) == "replica-a", 30.0)
        b = _watcher(kc, sink.url("200"), "replica-b")
        try:
            assert _wait(lambda: len(sink.requests) >= 1, 30.0)
            time.sleep(1.5)
            assert len(sink.requests) == 1  # the leader's first report; b is waiting
            a.terminate()  # SIGTERM: a releases the Lease on the way out
            a.wait(20)
            assert ("PUT", "gpu-node-watcher", "") in srv.lease_writes
            assert _wait(lambda: _holder(srv) == "replica-b", 10.0)
            time.sleep(1.5)
            assert len(sink.requests) == 1  # nothing new to say: not sent again
            srv.state.set_nodes(fixtures.cluster(3, "amd"))  # a change after the takeover is b's to send
            assert _wait(lambda: len(sink.requests) >= 2, 20.0)
            time.sleep(0.5)
        finally:
            b.terminate()
            out_b, err_b = b.communicate(timeout=20)
        assert "resuming the previous leader's notification state" in err_b
        reports = _stdout_reports(out_b)
        assert [r["total_nodes"] for r in reports] == [2, 3]
    finally:
        if a.poll() is None:
            a.kill()
        a.communicate(timeout=20)


def _handover(srv, kc, sink, mode, between):
    """a leads and reports; a stops; ``between()`` changes the cluster while nobody leads; b takes over.
    Returns (Slack POSTs while a led, Slack POSTs after b's first report)."""
    extra = ("--slack-only-on-error", "--slack-on-node-change")
    a = _watcher(kc, sink.url(mode), "replica-a", extra)
    b = None
    try:
        assert _wait(lambda: _holder(srv) == "replica-a", 30.0)
        assert _wait(lambda: srv.leases[("gpu-health", "gpu-node-watcher")]["metadata"].get("annotations"), 10.0)
        time.sleep(0.5)
        first = len(sink.requests)
        a.terminate()
        a.wait(20)
        between()
        b = _watcher(kc, sink.url(mode), "replica-b", extra)
        assert _wait(lambda: _holder(srv) == "replica-b", 20.0)
        time.sleep(2.0)
        return first, len(sink.requests)
    finally:
        for p in (a, b):
            if p is not None:
                if p.poll() is None:
                    p.terminate()
                p.communicate(timeout=20)


def test_failover_does_not_repeat_a_delivered_alert(mock_cluster, sink, tmp_path):
    """a new leader used to start with no memory and re-send the current error alert."""
    srv = mock_cluster(fixtures.golden("notready"))
    kc = srv.kubeconfig(str(tmp_path / "kc"))
    first, after = _handover(srv, kc, sink, "200", lambda: None)
    assert first == 1 and after == 1


def test_a_recovery_during_the_handover_is_announced(mock_cluster, sink, tmp_path):
    srv = mock_cluster(fixtures.golden("notready"))
    kc = srv.kubeconfig(str(tmp_path / "kc"))
    first, after = _handover(srv, kc, sink, "200", lambda: srv.state.set_nodes(fixtures.golden("readme")))
    assert first == 1 and after == 2
    assert "Ready 상태의 GPU 노드: 2개" in json.loads(sink.requests[-1]["body"])["text"]


def test_an_undelivered_alert_is_retried_by_the_next_leader(mock_cluster, sink, tmp_path):
    srv = mock_cluster(fixtures.golden("notready"))
    kc = srv.kubeconfig(str(tmp_path / "kc"))
    first, after = _handover(srv, kc, sink, "500", lambda: None)
    assert first >= 1 and after > first  # a's alert never arrived (HTTP 500): b sends it again


def test_a_watcher_that_cannot_renew_stops_acting_and_exits(mock_cluster, sink, tmp_path):
    """The leader loses the Lease API (every lease call fails) while the node API keeps working: at its renew
    deadline it stops following the cluster and exits (the Deployment restarts it as a candidate), before any
    other replica could take the Lease over."""
    srv = mock_cluster(fixtures.cluster(2, "amd"))
    kc = srv.kubeconfig(str(tmp_path / "kc"))
    a = _watcher(kc, sink.url("ok"), "replica-a")
    try:
        assert _wait(lambda: len(sink.requests) >= 1, 30.0)
        srv.lease_status = 500
        t0 = time.monotonic()
        a.wait(15)
        took = time.monotonic() - t0
        out, err = a.communicate(timeout=10)
        assert "lost gpu-health/gpu-node-watcher" in err, err[-800:]
        assert took < 5.0, took
        assert len(sink.requests) == 1  # nothing reported after leadership was given up
    finally:
        if a.poll() is None:
            a.kill()
            a.communicate(timeout=10)


def test_an_oversized_leader_state_is_not_kept_on_the_lease(mock_cluster):
    from k8s_gpu_node_checker_amd.kube import lease as L
    srv = mock_cluster(fixtures.cluster(1, "amd"))
    a = _elector(srv, "a").start()
    try:
        assert _wait(a.leading.is_set)
        assert a.publish_state({"exit_code": 3, "not_ready": ["n"]}) is True
        assert _wait(lambda: '"not_ready":["n"]' in (srv.leases[("gpu-health", "gpu-node-watcher")]["metadata"]
                                                       .get("annotations") or {}).get(L.STATE_ANNOTATION, ""))
        big = {"exit_code": 3, "not_ready": [f"node-{i:06d}" for i in range(10000)]}
        assert a.publish_state(big) is False
        assert _wait(lambda: srv.leases[("gpu-health", "gpu-node-watcher")]["metadata"]["annotations"]
                     [L.STATE_ANNOTATION] == "{}")
    finally:
        a.stop()


def test_publish_state_wakes_the_renewal_only_on_a_change():
    """the watcher publishes after every evaluation; an unchanged state must not add a Lease write per
    event batch (it rides on the periodic renewal)."""
    e = LeaderElector(lambda: None, "ns", "n", "id", lease_duration=15.0, renew_deadline=10.0, retry_period=2.0)
    assert e.publish_state({"exit_code": 0}) is True and e._wake.is_set()
    e._wake.clear()
    assert e.publish_state({"exit_code": 0}) is True and not e._wake.is_set()
    assert e.publish_state({"exit_code": 3}) is True and e._wake.is_set()
    e._wake.clear()
    big = {"not_ready": ["x" * 100] * 1000}
    assert e.publish_state(big) is False and e._wake.is_set()  # the old state is dropped: a change
    e._wake.clear()
    assert e.publish_state(big) is False and not e._wake.is_set()
