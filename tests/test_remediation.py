"""Remediation signals: the node agent's Events and unhealthy taint (optimistic concurrency against the
mock apiserver), and the checker's ``--require-schedulable`` gate that reads them back."""
import json

import pytest

from k8s_gpu_node_checker_amd import cli
from k8s_gpu_node_checker_amd.agent import agent as A
from k8s_gpu_node_checker_amd.kube.client import KubeClient
from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
from k8s_gpu_node_checker_amd.kube.errors import ApiException
from k8s_gpu_node_checker_amd.models.health import UNHEALTHY_TAINT
from k8s_gpu_node_checker_amd.testing import fixtures

OTHER = {"key": "dedicated", "value": "ml", "effect": "NoSchedule"}


@pytest.fixture
def fixture_report(tmp_path):
    p = tmp_path / "probe.json"
    p.write_text(json.dumps(fixtures.mi355x_probe_report("x", gpus=8)))
    return str(p)


def _bad(ag):
    rep = ag.probe_once()
    rep["gpus"][3]["ecc_uncorrectable"] = 2
    return rep


def test_events_and_taint_follow_verdict_changes(mock_cluster, fixture_report):
    srv = mock_cluster([fixtures.realistic_node("n", taints=[OTHER])])
    ag = A.Agent("n", source="fixture", fixture=fixture_report, taint_unhealthy=True)
    with KubeClient(ClusterConnection(srv.url)) as kc:
        w = ag.publish(kc, ag.probe_once())
        assert not w["event"] and not w["taint"] and srv.k8s_events == []  # healthy at start: no news
        w = ag.publish(kc, _bad(ag))
        assert w["event"] and w["taint"]
        ev = srv.k8s_events[-1]
        assert (ev["type"], ev["reason"]) == ("Warning", "MI355XUnhealthy")
        assert ev["involvedObject"] == {"apiVersion": "v1", "kind": "Node", "name": "n", "uid": "n"}
        assert ev["metadata"]["namespace"] == "default" and ev["metadata"]["name"].startswith("n.mi355x-")
        assert "gpu3: 2 uncorrectable ECC errors" in ev["message"]
        assert kc.get_node("n")["spec"]["taints"] == [OTHER, UNHEALTHY_TAINT]  # the operator's taint is kept
        w = ag.publish(kc, _bad(ag), force=True)  # same verdict (heartbeat): no second event, no taint write
        assert w["condition"] and not w["event"] and not w["taint"] and len(srv.k8s_events) == 1
        w = ag.publish(kc, ag.probe_once())  # recovery
        assert w["event"] and w["taint"]
        ev = srv.k8s_events[-1]
        assert (ev["type"], ev["reason"]) == ("Normal", "MI355XHealthy")
        assert ev["message"] == "8/8 MI355X GPUs healthy (was unhealthy)"
        assert kc.get_node("n")["spec"]["taints"] == [OTHER]
    assert [e["path"] for e in srv.log if e["method"] == "POST"] == ["/api/v1/namespaces/default/events"] * 2


def test_unknown_verdict_leaves_the_taint_alone(mock_cluster, fixture_report):
    srv = mock_cluster([fixtures.realistic_node("n")])
    ag = A.Agent("n", source="fixture", fixture=fixture_report, taint_unhealthy=True, events=False)
    with KubeClient(ClusterConnection(srv.url)) as kc:
        assert ag.publish(kc, _bad(ag))["taint"]
        failed = {"schema": "mi355x-health/v1", "node": "n", "ts": 0, "error": "amdsmi_init: driver not loaded",
                  "gpus": []}
        w = ag.publish(kc, failed)  # probe failure: verdict unknown, scheduling left as it was
        assert w["condition"] and not w["taint"] and not w["event"]
        assert kc.get_node("n")["spec"]["taints"] == [UNHEALTHY_TAINT]
    assert srv.k8s_events == []


def test_agent_restart_clears_a_stale_taint(mock_cluster, fixture_report):
    srv = mock_cluster([fixtures.realistic_node("n", taints=[dict(UNHEALTHY_TAINT), OTHER])])
    ag = A.Agent("n", source="fixture", fixture=fixture_report, taint_unhealthy=True)
    with KubeClient(ClusterConnection(srv.url)) as kc:
        w = ag.publish(kc, ag.probe_once())
        assert w["taint"] and not w["event"]
        assert kc.get_node("n")["spec"]["taints"] == [OTHER]


def test_taint_write_retries_on_conflict_and_refuses_stale_versions(mock_cluster):
    srv = mock_cluster([fixtures.realistic_node("n")], conflict_first=2)
    with KubeClient(ClusterConnection(srv.url), sleep=lambda s: None) as kc:
        assert kc.update_node_taints("n", lambda t: t + [dict(UNHEALTHY_TAINT)]) == [UNHEALTHY_TAINT]
        assert kc.get_node("n")["spec"]["taints"] == [UNHEALTHY_TAINT]
        assert kc.update_node_taints("n", lambda t: None) is None  # nothing to change: no write
        stale = json.dumps({"metadata": {"resourceVersion": "1"}, "spec": {"taints": []}}).encode()
        with pytest.raises(ApiException) as ei:
            kc.request("PATCH", "/api/v1/nodes/n", stale, content_type="application/merge-patch+json")
        assert ei.value.status == 409 and "the object has been modified" in ei.value.body
        assert kc.get_node("n")["spec"]["taints"] == [UNHEALTHY_TAINT]  # the stale write changed nothing
    assert sum(e["method"] == "PATCH" for e in srv.log) == 4  # 2 injected conflicts, the write, the stale one


def test_taint_write_gives_up_after_its_attempts(mock_cluster):
    srv = mock_cluster([fixtures.realistic_node("n")], conflict_first=10)
    with KubeClient(ClusterConnection(srv.url), sleep=lambda s: None) as kc:
        with pytest.raises(ApiException) as ei:
            kc.update_node_taints("n", lambda t: t + [dict(UNHEALTHY_TAINT)], attempts=3)
        assert ei.value.status == 409
    assert sum(e["method"] == "PATCH" for e in srv.log) == 3


def test_event_failure_never_blocks_the_condition(mock_cluster, fixture_report, capsys):
    srv = mock_cluster([fixtures.realistic_node("n")])
    ag = A.Agent("n", source="fixture", fixture=fixture_report)
    with KubeClient(ClusterConnection(srv.url)) as kc:
        def forbidden(ns, ev):
            raise ApiException(403, "Forbidden", body='events is forbidden: User "system:serviceaccount:x"')
        kc.create_event = forbidden
        w = ag.publish(kc, _bad(ag))
        assert w["condition"] and not w["event"]
        hc = [c for c in kc.get_node("n")["status"]["conditions"] if c["type"] == "AMDGPUHealthy"][0]
        assert hc["status"] == "False"
    assert "events is forbidden" in capsys.readouterr().err


def test_agent_flags(mock_cluster, tmp_path):
    bad = tmp_path / "bad.json"
    bad.write_text(json.dumps(fixtures.mi355x_probe_report("x", gpus=8, gpu0={"ecc_uncorrectable": 1})))
    srv = mock_cluster([fixtures.realistic_node("n"), fixtures.realistic_node("m", index=1)])
    kc = srv.kubeconfig(str(tmp_path / "kc"))
    base = ["--source", "fixture", "--fixture", str(bad), "--once", "--kubeconfig", kc]
    assert A.main(["--node", "n", "--taint-unhealthy", "--event-namespace", "gpu-health"] + base) == 0
    assert [e["metadata"]["namespace"] for e in srv.k8s_events] == ["gpu-health"]
    assert UNHEALTHY_TAINT in srv.state.find("n")["spec"]["taints"]
    assert A.main(["--node", "m", "--no-events"] + base) == 0  # default: no taint; events off
    assert len(srv.k8s_events) == 1 and not srv.state.find("m")["spec"].get("taints")


def test_require_schedulable_gate(mock_cluster, run_cli, tmp_path):
    cordoned = fixtures.realistic_node("a")
    cordoned["spec"]["unschedulable"] = True
    tainted = fixtures.realistic_node("b", index=1, taints=[dict(UNHEALTHY_TAINT)])
    srv = mock_cluster([cordoned, tainted])
    kc = srv.kubeconfig(str(tmp_path / "kc"))
    p = run_cli(["--kubeconfig", kc, "--json"])
    assert p.returncode == 0 and json.loads(p.stdout)["ready_nodes"] == 2  # the reference counts both
    p = run_cli(["--kubeconfig", kc, "--json", "--require-schedulable"])
    doc = json.loads(p.stdout)
    assert p.returncode == 3 and doc["ready_nodes"] == 0 and doc["total_nodes"] == 2
    srv.state.patch("a", {"spec": {"unschedulable": None}})  # kubectl uncordon
    p = run_cli(["--kubeconfig", kc, "--json", "--require-schedulable"])
    assert p.returncode == 0 and [n["name"] for n in json.loads(p.stdout)["nodes"] if n["ready"]] == ["a"]
    assert cli.parse_args(["--mi355x"]).require_schedulable


def test_require_schedulable_in_event_watch(mock_cluster, tmp_path, capsys):
    node = fixtures.realistic_node("a")
    node["spec"]["unschedulable"] = True
    srv = mock_cluster([node])
    kc = srv.kubeconfig(str(tmp_path / "kc"))
    rc = cli.main(["--kubeconfig", kc, "--json", "--require-schedulable", "--watch-events", "--watch-count", "1"])
    assert rc == 3 and json.loads(capsys.readouterr().out)["ready_nodes"] == 0


def test_label_node_keeps_inventory_and_verdict_labels(mock_cluster, fixture_report):
    srv = mock_cluster([fixtures.realistic_node("n")])
    ag = A.Agent("n", source="fixture", fixture=fixture_report, label_node=True, events=False)
    with KubeClient(ClusterConnection(srv.url)) as kc:
        w = ag.publish(kc, ag.probe_once())
        assert w["labels"]
        lab = kc.get_node("n")["metadata"]["labels"]
        assert lab["amd.com/mi355x-health"] == "healthy" and lab["amd.com/gpu.count"] == "8"
        assert lab["amd.com/gpu.compute-partition"] == "SPX" and lab["amd.com/gpu.memory-partition"] == "NPS1"
        assert lab["amd.com/gpu.vbios"] == "00175784" and lab["amd.com/gpu.driver"] == "6.18.54"
        assert lab["kubernetes.io/hostname"]  # the node's own labels are untouched
        assert not ag.publish(kc, ag.probe_once())["labels"]  # unchanged: no write
        w = ag.publish(kc, _bad(ag))
        assert w["labels"] and kc.get_node("n")["metadata"]["labels"]["amd.com/mi355x-health"] == "unhealthy"


def test_label_values_are_valid_kubernetes_labels():
    import re
    from hypothesis import given, strategies as st
    ok = re.compile(r"^(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?$")

    @given(st.text(max_size=200))
    def check(v):
        out = A.label_value(v)
        assert len(out) <= 63 and ok.match(out), (v, out)
    check()
    drv = "Linuxversion6.18.54-ant.1(nixbld@localhost)(gcc(GCC)15.3.0,GNUld(GNUBinutils)2.46)#1-ant-oci"
    out = A.label_value(drv)
    assert len(out) == 63 and out.startswith("Linuxversion6.18.54-ant.1nixbldlocalhost")
    # what the MI355X box's in-tree driver reports becomes its kernel release
    rep = fixtures.mi355x_probe_report("n", gpus=1, driver={"name": "amdgpu", "version": drv})
    assert A.node_labels(rep, "healthy")["amd.com/gpu.driver"] == "6.18.54-ant.1"
    rep = fixtures.mi355x_probe_report("n", gpus=2, gpu1={"compute_partition": "CPX"})
    rep.pop("driver")
    lab = A.node_labels(rep, "degraded")
    assert lab["amd.com/gpu.compute-partition"] == "mixed" and lab["amd.com/gpu.driver"] is None


def test_rejected_annotation_never_blocks_the_condition(mock_cluster, fixture_report):
    """A failed annotation / label / taint write is reported, the condition heartbeat still goes out,
    and the failed write is retried at the next publish."""
    srv = mock_cluster([fixtures.realistic_node("n")])
    ag = A.Agent("n", source="fixture", fixture=fixture_report, label_node=True, taint_unhealthy=True)
    with KubeClient(ClusterConnection(srv.url)) as kc:
        real = kc.patch_node_annotations, kc.patch_node_labels

        def too_big(node, ann):
            raise ApiException(422, "Unprocessable Entity", body="metadata.annotations: Too long: must have at most "
                                                                 "262144 bytes")

        def no_labels(node, labels):
            raise ApiException(403, "Forbidden", body="nodes is forbidden")
        kc.patch_node_annotations, kc.patch_node_labels = too_big, no_labels
        with pytest.raises(A.PublishError) as ei:
            ag.publish(kc, _bad(ag))
        assert "annotation: " in str(ei.value) and "Too long" in str(ei.value) and "labels: " in str(ei.value)
        assert ei.value.wrote["condition"] and ei.value.wrote["taint"] and not ei.value.wrote["annotation"]
        hc = [c for c in kc.get_node("n")["status"]["conditions"] if c["type"] == "AMDGPUHealthy"][0]
        assert hc["status"] == "False"
        kc.patch_node_annotations, kc.patch_node_labels = real
        w = ag.publish(kc, _bad(ag))  # same verdict: only the writes that failed go out again
        assert w["annotation"] and w["labels"] and not w["condition"] and not w["taint"]
        assert kc.get_node("n")["metadata"]["labels"]["amd.com/mi355x-health"] == "unhealthy"


def test_probe_that_cannot_run_publishes_unknown(mock_cluster, tmp_path):
    srv = mock_cluster([fixtures.realistic_node("n")])
    ag = A.Agent("n", source="fixture", fixture=str(tmp_path / "gone.json"))
    rep = ag.probe_once()
    assert rep["state"] == "unknown" and rep["error"].startswith("probe: ") and "gone.json" in rep["error"]
    with KubeClient(ClusterConnection(srv.url)) as kc:
        assert ag.publish(kc, rep)["condition"]
        hc = [c for c in kc.get_node("n")["status"]["conditions"] if c["type"] == "AMDGPUHealthy"][0]
        assert hc["status"] == "Unknown"


def test_agent_once_exit_code_reflects_publish(mock_cluster, fixture_report, tmp_path):
    srv = mock_cluster([fixtures.realistic_node("n")])
    kc = srv.kubeconfig(str(tmp_path / "kc"))
    base = ["--source", "fixture", "--fixture", fixture_report, "--once", "--kubeconfig", kc]
    assert A.main(["--node", "n"] + base) == 0
    assert A.main(["--node", "no-such-node"] + base) == 1  # every write 404s
