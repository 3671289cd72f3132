"""GPU-node membership when the device plugin withdraws GPUs.

Under ``--gpu-source allocatable`` (and so ``--mi355x``) a node whose ``amd.com/gpu`` allocatable dropped to 0
while capacity still registers 8 -- a crashed or wedged ROCm device plugin -- stays in the GPU-node set as Not
Ready, with the reason ``device plugin allocates 0 of 8 amd.com/gpu``.  The reference defines membership from
capacity (``check-gpu-node.py:181-196``, ``:220-225``) and reports "GPU nodes exist, none Ready" as exit 3
(``:289-293``); counting allocatable must change the counts, not hide the node.
"""
import json
import os
import socket
import subprocess
import sys
import time
import types

import pytest

from k8s_gpu_node_checker_amd.models.node import (HEALTH_ANNOTATION, HEALTH_CONDITION, NodeExtras, ScanResult,
                                                  classify_node, scan_items, withdrawn_count)
from k8s_gpu_node_checker_amd.models.resources import GPU_RESOURCE_KEYS
from k8s_gpu_node_checker_amd.ops import fastpath
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
from k8s_gpu_node_checker_amd.utils import statefile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = [f"mi355x-node-{i:04d}" for i in range(8)]


def _withdraw(node, n=0, key="amd.com/gpu"):
    node["status"]["allocatable"][key] = str(n)
    return node


def _healthy_cluster(withdrawn=()):
    nodes = fixtures.cluster(8, "amd", with_health=True)
    for i in withdrawn:
        _withdraw(nodes[i])
    return nodes


# -- the rule ------------------------------------------------------------------------------------------------------

def test_classify_node_membership_rule():
    n = _withdraw(fixtures.realistic_node("w"))
    assert classify_node(n, GPU_RESOURCE_KEYS, "capacity")["gpus"] == 8  # the reference: capacity decides
    info = classify_node(n, GPU_RESOURCE_KEYS, "allocatable")
    assert info["gpus"] == 0 and info["gpu_breakdown"] == {"amd.com/gpu": 0} and info["ready"] is False
    # allocatable without the key at all: still a member, empty breakdown
    del n["status"]["allocatable"]["amd.com/gpu"]
    info = classify_node(n, GPU_RESOURCE_KEYS, "allocatable")
    assert info is not None and info["gpus"] == 0 and info["gpu_breakdown"] == {} and not info["ready"]
    # a node with neither: not a GPU node under either source
    cpu = fixtures.realistic_node("cpu", gpu_key=None)
    assert classify_node(cpu, GPU_RESOURCE_KEYS, "capacity") is None
    assert classify_node(cpu, GPU_RESOURCE_KEYS, "allocatable") is None
    # capacity 0 everywhere (the reference's "only-zero" edge): excluded, as before
    z = fixtures.realistic_node("z", gpu_count=0)
    assert classify_node(z, GPU_RESOURCE_KEYS, "allocatable") is None
    # partly withdrawn: counts from allocatable, Ready untouched
    p = _withdraw(fixtures.realistic_node("p"), 6)
    info = classify_node(p, GPU_RESOURCE_KEYS, "allocatable")
    assert info["gpus"] == 6 and info["ready"] is True


def test_withdrawn_count():
    assert withdrawn_count({"amd.com/gpu": 8}, {"amd.com/gpu": 0}) == 8
    assert withdrawn_count({"amd.com/gpu": 8}, {}) == 8
    assert withdrawn_count({"amd.com/gpu": 8}, {"amd.com/gpu": 1}) == 0
    assert withdrawn_count({}, {}) == 0
    assert withdrawn_count({"amd.com/gpu": 0}, {"amd.com/gpu": 0}) == 0


@pytest.mark.skipif(fastpath.ext() is None, reason="native fast path not built")
@pytest.mark.parametrize("src", ["capacity", "allocatable"])
def test_native_scanner_applies_the_same_rule(src):
    nodes = _healthy_cluster(withdrawn=(2, 5))
    del nodes[5]["status"]["allocatable"]["amd.com/gpu"]
    nodes += fixtures.cluster(3, "cpu") + [_withdraw(fixtures.realistic_node("nv", "nvidia.com/gpu", index=40),
                                                               key="nvidia.com/gpu")]
    body = json.dumps(fixtures.node_list(nodes)).encode()
    ext = fastpath.ext()
    a = ScanResult()
    ext.scan_nodelist(body, a, GPU_RESOURCE_KEYS, src == "allocatable", True, HEALTH_ANNOTATION, NodeExtras,
                      HEALTH_CONDITION, 1)
    b = scan_items(nodes, None, GPU_RESOURCE_KEYS, src, True, 1)
    assert json.dumps([a.gpu_nodes, a.ready_gpu_nodes, a.items_seen], ensure_ascii=False) == \
        json.dumps([b.gpu_nodes, b.ready_gpu_nodes, b.items_seen], ensure_ascii=False)
    assert len(a.gpu_nodes) == 9  # 8 amd + the withdrawn nvidia node, under both sources
    want_ready = 9 if src == "capacity" else 6
    assert len(a.ready_gpu_nodes) == want_ready
    # extras keep the kubelet's Ready condition: withdrawal is not a kubelet verdict
    assert all(e.ready_condition for e in a.extras)


# -- the CLI (done-when (a) and (b)) --------------------------------------------------------------------------------

def test_mi355x_one_withdrawn_node_of_eight_is_listed_not_ready(run_cli, mock_cluster, tmp_path):
    srv = mock_cluster(_healthy_cluster(withdrawn=(3,)))
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    p = run_cli(["--kubeconfig", kc, "--mi355x", "--json"])
    assert p.returncode == 0, p.stderr
    doc = json.loads(p.stdout)
    assert doc["total_nodes"] == 8 and doc["ready_nodes"] == 7
    assert [n["name"] for n in doc["nodes"]] == NAMES
    w = doc["nodes"][3]
    assert w["ready"] is False and w["gpus"] == 0 and w["gpu_breakdown"] == {"amd.com/gpu": 0}
    # text mode and Slack carry the reason
    p = run_cli(["--kubeconfig", kc, "--mi355x"])
    assert p.returncode == 0 and "mi355x-node-0003  False  0" in p.stdout


def test_mi355x_fleet_entirely_withdrawn_exits_3_not_2(run_cli, mock_cluster, sink, tmp_path):
    srv = mock_cluster(_healthy_cluster(withdrawn=range(8)))
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    p = run_cli(["--kubeconfig", kc, "--mi355x", "--json"])
    assert p.returncode == 3, p.stdout
    doc = json.loads(p.stdout)
    assert doc["total_nodes"] == 8 and doc["ready_nodes"] == 0
    p = run_cli(["--kubeconfig", kc, "--mi355x", "--slack-only-on-error", "--slack-webhook", sink.url("200")])
    assert p.returncode == 3
    assert p.stdout.splitlines()[1] == "⚠️ GPU 노드는 8개 있으나, Ready 상태 노드는 없습니다."
    text = sink.payloads()[-1]["text"]
    assert "`mi355x-node-0000`: ❌ Not Ready, GPU: 0 (amd.com/gpu:0)" in text
    assert "device plugin allocates 0 of 8 amd.com/gpu" in text
    # the reference's own rule (capacity) still counts them Ready: the default is unchanged
    p = run_cli(["--kubeconfig", kc, "--json"])
    assert p.returncode == 0 and json.loads(p.stdout)["ready_nodes"] == 8


def test_explain_names_the_device_plugin(run_cli, mock_cluster, tmp_path):
    srv = mock_cluster(_healthy_cluster(withdrawn=(1,)))
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    p = run_cli(["--kubeconfig", kc, "--mi355x", "--explain", NAMES[1]])
    assert "device plugin allocates 0 of 8 amd.com/gpu" in p.stdout, p.stdout + p.stderr


# -- Slack de-dup (done-when (c)) -----------------------------------------------------------------------------------

def _cronjob_args(tmp_path, kc):
    import yaml
    with open(os.path.join(REPO, "deploy", "cronjob.yaml"), encoding="utf-8") as f:
        cmd = yaml.safe_load(f)["spec"]["jobTemplate"]["spec"]["template"]["spec"]["containers"][0]["command"]
    assert cmd[0] == "check-gpu-node" and "--mi355x" in cmd and "--slack-on-node-change" in cmd
    args = [a for a in cmd[1:] if a != "--in-cluster"]
    args[args.index("/state/last.json")] = str(tmp_path / "last.json")
    return args + ["--kubeconfig", kc]


def test_shipped_cronjob_alerts_once_for_8_to_0_allocatable_and_once_for_recovery(run_cli, mock_cluster, sink,
                                                                                 tmp_path):
    srv = mock_cluster(_healthy_cluster())
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    args = _cronjob_args(tmp_path, kc)
    env = {"SLACK_WEBHOOK_URL": sink.url("200")}
    for _ in range(2):
        assert run_cli(args, env=env).returncode == 0
    assert len(sink.requests) == 0
    srv.state.set_nodes(_healthy_cluster(withdrawn=range(8)))
    for _ in range(3):
        p = run_cli(args, env=env)
        assert p.returncode == 3, p.stdout + p.stderr
    assert len(sink.requests) == 1
    assert "device plugin allocates 0 of 8 amd.com/gpu" in sink.payloads()[0]["text"]
    srv.state.set_nodes(_healthy_cluster())
    for _ in range(2):
        assert run_cli(args, env=env).returncode == 0
    assert len(sink.requests) == 2  # the recovery, once
    assert sink.payloads()[1]["text"].startswith("✅")


def test_node_leaving_the_gpu_set_notifies_with_node_change(run_cli, mock_cluster, sink, tmp_path):
    """A node that is simply gone (deleted, or its capacity deregistered) is in no not-Ready list: the member
    comparison catches it."""
    nodes = _healthy_cluster()
    srv = mock_cluster(nodes)
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    args = _cronjob_args(tmp_path, kc)
    env = {"SLACK_WEBHOOK_URL": sink.url("200")}
    assert run_cli(args, env=env).returncode == 0
    assert statefile.load(str(tmp_path / "last.json"))["gpu_nodes"] == NAMES
    srv.state.set_nodes(nodes[:3] + nodes[4:])
    for _ in range(2):
        assert run_cli(args, env=env).returncode == 0
    assert len(sink.requests) == 1
    srv.state.set_nodes(nodes)
    assert run_cli(args, env=env).returncode == 0
    assert len(sink.requests) == 1  # a node joining is not an alert


def _res(exit_code, names, ready=True):
    return types.SimpleNamespace(exit_code=exit_code, gpu_nodes=[{"name": n, "ready": ready, "gpus": 8} for n in names],
                                 ready_gpu_nodes=[], slack_sent=None)


def test_left_gpu_set_rules():
    before = _res(0, ["a", "b", "c"])
    prev = statefile.outcome(before)
    assert prev["gpu_nodes"] == ["a", "b", "c"] and prev["gpu_count"] == 3
    assert statefile.left_gpu_set(prev, _res(0, ["a", "c"]))
    assert not statefile.left_gpu_set(prev, _res(0, ["a", "b", "c", "d"]))
    assert statefile.should_notify(prev, _res(0, ["a", "c"]), True, on_node_change=True)
    assert not statefile.should_notify(prev, _res(0, ["a", "c"]), True, on_node_change=False)
    # compacted state (no names, no sketch: the last resort for a huge fleet's Lease): digest + count decide
    big = statefile.outcome(_res(0, [f"n{i}" for i in range(1001)]))
    small = {k: v for k, v in big.items() if k != "gpu_nodes"}
    assert statefile.left_gpu_set(small, _res(0, [f"n{i}" for i in range(1000)]))
    assert not statefile.left_gpu_set(small, _res(0, [f"n{i}" for i in range(1001)]))
    assert statefile.compact(prev) is prev and statefile.compact(big) is big  # short names: fits as it is
    # a state file from before the member list: no opinion
    assert not statefile.left_gpu_set({"exit_code": 0, "not_ready": []}, _res(0, ["a"]))


# -- watcher metrics (done-when (d)) --------------------------------------------------------------------------------

def _scrape(port):
    from k8s_gpu_node_checker_amd.utils.http import request
    r = request(f"http://127.0.0.1:{port}/metrics")
    assert r.status == 200
    return r.text


def test_watcher_metrics_keep_a_withdrawn_nodes_series_at_zero(mock_cluster, tmp_path):
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    srv = mock_cluster(_healthy_cluster(), bookmark_interval=0.2)
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    env = {k: v for k, v in os.environ.items() if k not in ("SLACK_WEBHOOK_URL", "KUBECONFIG")}
    p = subprocess.Popen([sys.executable, os.path.join(REPO, "check-gpu-node.py"), "--kubeconfig", kc, "--json",
                          "--mi355x", "--watch-events", "--watch-duration", "30", "--watch-debounce", "0.1",
                          "--metrics-listen", f"127.0.0.1:{port}"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, env=env, cwd=str(tmp_path))
    series = f'k8s_gpu_checker_node_ready{{node="{NAMES[2]}"}}'

    def wait_for(needle):
        t0 = time.monotonic()
        while time.monotonic() - t0 < 20:
            try:
                text = _scrape(port)
                if needle in text:
                    return text
            except Exception:  # not listening yet
                pass
            time.sleep(0.1)
        raise AssertionError(f"{needle!r} never appeared")
    try:
        wait_for(series + " 1")
        srv.state.patch(NAMES[2], {"status": {"allocatable": {"amd.com/gpu": "0"}}})
        text = wait_for(series + " 0")
        assert "k8s_gpu_checker_gpu_nodes 8" in text and "k8s_gpu_checker_ready_gpu_nodes 7" in text
        srv.state.patch(NAMES[2], {"status": {"allocatable": {"amd.com/gpu": "8"}}})
        wait_for(series + " 1")
    finally:
        p.terminate()
        p.communicate(timeout=30)


def _long_names(n, start=0):
    # real node names: 40-70 characters (cloud instance DNS names)
    return [f"ip-10-{i // 250}-{i % 250}-{i}.us-west-2.compute.internal.mi355x-gpu-pool-a-zone-1" for i in range(start, start + n)]


def test_compaction_is_by_size_and_keeps_departures_hidden_by_growth():
    """1,001 realistic names exceed the Lease's 64 KiB as a list; VERDICT r5 #6: a compacted state must
    still see one node leave while two join.  The compacted outcome fits, carries a hash sketch, and the watcher's
    gate sends exactly one node-change alert for that move."""
    names = _long_names(1001)
    prev = statefile.outcome(_res(0, names))
    assert len(json.dumps(prev, sort_keys=True, separators=(",", ":"))) > statefile.STATE_MAX_BYTES
    small = statefile.compact(prev)
    assert len(json.dumps(small, sort_keys=True, separators=(",", ":"))) <= statefile.STATE_MAX_BYTES
    assert "gpu_nodes" not in small and small["gpu_sketch"].startswith("8:") and small["gpu_count"] == 1001
    moved = names[1:] + _long_names(2, start=5000)  # node 0 leaves, two new ones join: the set grew
    assert statefile.left_gpu_set(small, _res(0, moved))
    alerts = 0
    state = small
    for res in (_res(0, moved), _res(0, moved), _res(0, moved)):
        if statefile.should_notify(state, res, True, on_node_change=True):
            alerts += 1
        state = statefile.compact(statefile.outcome(res))
    assert alerts == 1
    assert not statefile.left_gpu_set(small, _res(0, names + _long_names(1, start=9000)))  # growth alone: no alert
    # the sketch survives the state file / Lease round trip and a corrupt one is dropped, not trusted
    assert statefile.sketch_members(small["gpu_sketch"])[0] == 8
    assert statefile.sketch_members("8:???") is None and statefile.sketch_members("8:AAAA") is None and statefile.sketch_members("3:AAAA") is None


def test_compaction_narrows_then_drops_the_sketch_then_digests_not_ready():
    names = _long_names(7000)
    prev = statefile.outcome(_res(0, names))
    small = statefile.compact(prev)
    assert small["gpu_sketch"].startswith("4:")  # 8-byte hashes of 7,000 names do not fit, 4-byte ones do
    assert statefile.left_gpu_set(small, _res(0, names[1:]))
    huge = statefile.outcome(_res(0, _long_names(20000)))
    assert "gpu_sketch" not in statefile.compact(huge) and "members" in statefile.compact(huge)
    # thousands of not-Ready names: their digest and count stand in, and a change is still seen
    down = statefile.outcome(_res(3, _long_names(2000), ready=False))
    tiny = statefile.compact(down)
    assert "not_ready" not in tiny and tiny["not_ready_count"] == 2000
    assert len(json.dumps(tiny, sort_keys=True, separators=(",", ":"))) <= statefile.STATE_MAX_BYTES
    assert not statefile.should_notify(tiny, _res(3, _long_names(2000), ready=False), True, on_node_change=True)
    assert statefile.should_notify(tiny, _res(3, _long_names(1999), ready=False), True, on_node_change=True)
