"""``--probe-endpoint 'http://{pod_ip}:9464/probe'`` reaches the agents the shipped manifests deploy.

The agent DaemonSet listens on the pod network only, so the fan-out addresses it through the EndpointSlices
of the agents' headless Service (``deploy/daemonset.yaml``), read with the namespaced Role in
``deploy/rbac.yaml``.  These tests take the Service, port, RBAC and documented template from the real
manifests, serve matching EndpointSlices from the mock apiserver and run the checker against mock agents
bound to those pod addresses (127.0.0.x).  Reference: each verdict belongs to the node it was read for
(``/root/reference/check-gpu-node.py:199-212``).
"""
import json
import os
import re
import types

import pytest
import yaml

from k8s_gpu_node_checker_amd import cli
from k8s_gpu_node_checker_amd.agent import agent as A
from k8s_gpu_node_checker_amd.parallel import fanout
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.mock_apiserver import endpoint_slice, write_kubeconfig

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _docs(*rel):
    with open(os.path.join(REPO, "deploy", *rel), encoding="utf-8") as f:
        return [d for d in yaml.safe_load_all(f) if d]


def _agent_service():
    """(namespace, name, port) of the agents' Service, checked against the DaemonSet it fronts."""
    docs = _docs("daemonset.yaml")
    ds = next(d for d in docs if d["kind"] == "DaemonSet")
    svc = next(d for d in docs if d["kind"] == "Service")
    pod = ds["spec"]["template"]
    assert svc["metadata"]["namespace"] == ds["metadata"]["namespace"]
    assert svc["spec"]["selector"].items() <= pod["metadata"]["labels"].items()
    c = pod["spec"]["containers"][0]
    ports = {p["name"]: p["containerPort"] for p in c["ports"]}
    [sp] = svc["spec"]["ports"]
    port = ports[sp["targetPort"]]
    # the agent really listens on that port on every pod address
    args = A.build_parser().parse_args(c["command"][1:])
    assert args.listen == f"0.0.0.0:{port}"
    assert not pod["spec"].get("hostNetwork") and "hostPort" not in c["ports"][0]
    return svc["metadata"]["namespace"], svc["metadata"]["name"], port


def test_manifests_wire_the_pod_ip_source_end_to_end():
    ns, name, port = _agent_service()
    # the checker's default --probe-service is that Service
    assert cli.parse_args([]).probe_service == f"{ns}/{name}"
    # the checker's ServiceAccount may list EndpointSlices in that namespace (and nothing more is added)
    rbac = _docs("rbac.yaml")
    roles = {d["metadata"]["name"]: d for d in rbac if d["kind"] == "Role"}
    grants = set()
    for b in (d for d in rbac if d["kind"] == "RoleBinding"):
        if {"kind": "ServiceAccount", "name": "gpu-node-checker", "namespace": ns} not in b["subjects"]:
            continue
        role = roles[b["roleRef"]["name"]]
        assert role["metadata"]["namespace"] == b["metadata"]["namespace"] == ns
        grants |= {(g, r, v) for rule in role["rules"] for g in rule["apiGroups"] for r in rule["resources"]
                   for v in rule["verbs"]}
    assert grants == {("discovery.k8s.io", "endpointslices", "list")}
    # the documented template is the one that reaches the agents
    with open(os.path.join(REPO, "README.md"), encoding="utf-8") as f:
        readme = f.read()
    assert f"--probe-endpoint 'http://{{pod_ip}}:{port}/probe'" in readme
    assert "'http://{ip}:9464/probe'" not in readme


def test_agent_addresses_prefers_ready_then_live_endpoints():
    slices = [
        endpoint_slice("gpu-health", "svc", [{"node": "a", "ip": "10.0.0.9", "ready": False, "terminating": True},
                                             {"node": "b", "ip": "10.0.1.2", "ready": False}]),
        endpoint_slice("gpu-health", "svc", [{"node": "a", "ip": "10.0.0.3", "ready": True},
                                             {"node": "b", "ip": "10.0.1.1", "ready": False},
                                             {"node": "c", "ip": "fd00::7"}], name="svc-2"),
        {"endpoints": [{"addresses": [], "nodeName": "d"}, {"addresses": ["10.9.9.9"]}, "junk"]},
    ]
    assert fanout.agent_addresses(slices) == {"a": "10.0.0.3", "b": "10.0.1.1", "c": "fd00::7"}
    scan = types.SimpleNamespace(gpu_nodes=[{"name": n} for n in "abcd"],
                                 extras=[types.SimpleNamespace(internal_ip=None)] * 4)
    t = fanout.build_targets(scan, "http://{pod_ip}:9464/probe", fanout.agent_addresses(slices))
    assert [x["url"] for x in t] == ["http://10.0.0.3:9464/probe", "http://10.0.1.1:9464/probe",
                                     "http://[fd00::7]:9464/probe", ""]
    assert t[3]["error"] == "no agent endpoint on this node"
    t = fanout.build_targets(scan, "http://{pod_ip}:9464/probe", None, "(403) Forbidden")
    assert all(x["error"] == "agent endpoints unavailable: (403) Forbidden" for x in t)


@pytest.fixture
def pod_network(fixture_report_factory):
    """Mock agents on 127.0.0.2-4 (one port), as the DaemonSet's pods a, b, c; b reports an ECC fault."""
    servers = []
    port = 0
    for i, name in enumerate("abc"):
        ag = A.Agent(name, source="fixture", fixture=fixture_report_factory(name))
        rep = ag.probe_once()
        if name == "b":
            rep["gpus"][0]["ecc_uncorrectable"] = 3
        srv = A.serve(ag, f"127.0.0.{i + 2}", port)
        port = srv.server_address[1]
        servers.append(srv)
    yield port
    for s in servers:
        s.shutdown()
        s.server_close()


@pytest.fixture
def fixture_report_factory(tmp_path):
    def make(name):
        p = tmp_path / f"probe-{name}.json"
        p.write_text(json.dumps(fixtures.mi355x_probe_report(name, gpus=8)))
        return str(p)
    return make


def _cluster(mock_cluster, ns, name, port, status=None):
    nodes = []
    for i, n in enumerate("abcd"):
        node = fixtures.realistic_node(n, "amd.com/gpu", 8, index=i)
        # the InternalIP reaches nothing: only {pod_ip} can find the agents
        node["status"]["addresses"][0]["address"] = "127.0.0.1"
        nodes.append(node)
    srv = mock_cluster(nodes)
    # two slices, as the EndpointSlice controller splits large Services; a stale terminating pod on node a
    srv.endpoint_slices = [
        endpoint_slice(ns, name, [{"node": "a", "ip": "127.0.0.9", "ready": False, "terminating": True},
                                  {"node": "a", "ip": "127.0.0.2", "ready": True},
                                  {"node": "b", "ip": "127.0.0.3", "ready": True}], port=port, name=f"{name}-x1"),
        endpoint_slice(ns, name, [{"node": "c", "ip": "127.0.0.4"}], port=port, name=f"{name}-x2"),
        # another Service's slice in the namespace, and one of the same name elsewhere: neither is read
        endpoint_slice(ns, "other", [{"node": "d", "ip": "127.0.0.5", "ready": True}], port=port),
        endpoint_slice("default", name, [{"node": "d", "ip": "127.0.0.6", "ready": True}], port=port),
    ]
    srv.endpoint_slices_status = status
    return srv


def test_pod_ip_fanout_reaches_each_nodes_own_agent(pod_network, mock_cluster, run_cli, tmp_path):
    ns, name, _ = _agent_service()
    port = pod_network
    srv = _cluster(mock_cluster, ns, name, port)
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    # --page-size 1: the EndpointSlice LIST is paged like the node LIST
    p = run_cli(["--kubeconfig", kc, "--mi355x", "--json-extended", "--probe-unknown", "deny", "--page-size", "1",
                 "--probe-endpoint", f"http://{{pod_ip}}:{port}/probe", "--probe-timeout", "2"])
    doc = json.loads(p.stdout)
    health = {n["name"]: n["health"] for n in doc["mi355x"]["nodes"]}
    assert {k: v["state"] for k, v in health.items()} == {"a": "healthy", "b": "unhealthy", "c": "healthy",
                                                          "d": "unknown"}
    assert any("no agent endpoint" in r for r in health["d"].get("reasons", [])), health["d"]
    assert not any("report is for node" in r for v in health.values() for r in v.get("reasons", []))
    assert [n["ready"] for n in doc["nodes"]] == [True, False, True, False]
    assert p.returncode == 0
    paths = [e["path"] for e in srv.log if "endpointslices" in e["path"]]
    assert paths and all(pth.startswith(f"/apis/discovery.k8s.io/v1/namespaces/{ns}/endpointslices?") for pth in paths)
    assert len(paths) == 2  # two slices of this Service at one per page


def test_pod_ip_fanout_without_rbac_makes_nodes_unknown_not_wrong(pod_network, mock_cluster, run_cli, tmp_path):
    ns, name, _ = _agent_service()
    srv = _cluster(mock_cluster, ns, name, pod_network, status=403)
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    p = run_cli(["--kubeconfig", kc, "--mi355x", "--json-extended", "--probe-unknown", "deny",
                 "--probe-endpoint", f"http://{{pod_ip}}:{pod_network}/probe"])
    doc = json.loads(p.stdout)
    for n in doc["mi355x"]["nodes"]:
        assert n["health"]["state"] == "unknown"
        assert any(re.search(r"agent endpoints unavailable: \(403\)", r) for r in n["health"]["reasons"]), n
    assert p.returncode == 3


def test_probe_service_flag_selects_another_service(pod_network, mock_cluster, run_cli, tmp_path):
    srv = _cluster(mock_cluster, "monitoring", "gpu-agents", pod_network)
    kc = write_kubeconfig(str(tmp_path / "kc"), srv.url)
    p = run_cli(["--kubeconfig", kc, "--mi355x", "--json-extended", "--probe-service", "monitoring/gpu-agents",
                 "--probe-endpoint", f"http://{{pod_ip}}:{pod_network}/probe"])
    states = [n["health"]["state"] for n in json.loads(p.stdout)["mi355x"]["nodes"]]
    assert states == ["healthy", "unhealthy", "healthy", "unknown"]


def test_watch_mode_reuses_fetched_reports_and_endpoints_within_the_ttl(pod_network, mock_cluster, monkeypatch):
    """--watch-events re-evaluates the fleet on every batch of node events: with a ProbeCache the agents' reports
    and the EndpointSlices are fetched once per TTL, a failed fetch is retried at once, and after the TTL
    everything is fetched again."""
    from k8s_gpu_node_checker_amd.checker import CheckOptions, apply_health, scan_cluster
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    from k8s_gpu_node_checker_amd.models import health as H
    from k8s_gpu_node_checker_amd.parallel import fanout
    from k8s_gpu_node_checker_amd.utils.timing import NullTracer
    ns, name, _ = _agent_service()
    port = pod_network
    srv = _cluster(mock_cluster, ns, name, port)
    cluster = ClusterConnection(srv.url)
    fetched = []
    real = fanout.fetch_all

    async def counting(targets, *a, **kw):
        fetched.extend(t["name"] for t in targets if not t.get("error"))
        return await real(targets, *a, **kw)
    monkeypatch.setattr(fanout, "fetch_all", counting)
    cache = fanout.ProbeCache(ttl=60.0)
    opts = CheckOptions(probe_endpoint=f"http://{{pod_ip}}:{port}/probe", health_policy="require",
                        probe_cache=cache)

    def evaluate():
        scan = scan_cluster(cluster, opts, NullTracer())
        return {n["name"]: v.state for n, v in zip(scan.gpu_nodes, apply_health(scan, opts, NullTracer(), [], cluster))}
    first = evaluate()
    assert first == {"a": H.HEALTHY, "b": H.UNHEALTHY, "c": H.HEALTHY, "d": H.UNKNOWN}
    assert sorted(fetched) == ["a", "b", "c"]  # d has no endpoint: nothing to fetch
    slices = len([e for e in srv.log if "endpointslices" in e["path"]])
    fetched.clear()
    assert evaluate() == first
    assert fetched == [] and cache.reused == 3  # all three from the cache
    assert len([e for e in srv.log if "endpointslices" in e["path"]]) == slices  # no second EndpointSlice LIST
    cache.ttl = 0.0  # expired: everything again
    assert evaluate() == first and sorted(fetched) == ["a", "b", "c"]
    from k8s_gpu_node_checker_amd import cli
    assert cli.parse_args(["--probe-cache-ttl", "5"]).probe_cache_ttl == 5.0


def test_probe_cache_forgets_entries_well_past_the_ttl():
    from k8s_gpu_node_checker_amd.parallel.fanout import ProbeCache
    c = ProbeCache(ttl=10.0)
    t = {"name": "a", "url": "http://10.0.0.1:9464/probe"}
    c.put(t, {"node": "a"}, now=0.0)
    c.put({"name": "b", "url": "u"}, {"error": "x"}, now=0.0)  # a failed fetch is not kept
    assert c.get(t, now=5.0) == {"node": "a"} and c.get({"name": "b", "url": "u"}, now=5.0) is None
    assert c.get(t, now=10.0) is None  # expired, still held
    c.prune(now=39.0)
    assert len(c._reports) == 1
    c.prune(now=40.0)
    assert c._reports == {}


def test_fetched_reports_are_slimmed_before_they_are_cached():
    """a --watch-events checker keeps every agent's /probe report in its ProbeCache; the
    agent-only per-test fields (per-XCD/CU maps, burn-in rows, wall time) are dropped as for annotations."""
    import http.server
    import threading
    from k8s_gpu_node_checker_amd.models.node import DIAG_AGENT_ONLY
    from k8s_gpu_node_checker_amd.parallel import fanout
    rep = fixtures.mi355x_probe_report("a", gpus=2)
    for g in rep["gpus"]:
        g["diag"] = {"mfma": {"pass": True, "map": {"cus": 256}, "kinds": {"bf16": {}}, "wall_s": 1.0, "rates": {}}}
    body = json.dumps(rep).encode()

    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        target = {"name": "a", "url": f"http://127.0.0.1:{srv.server_address[1]}/probe"}
        out = fanout.run_coroutine(fanout.fetch_all([target], 4, 5.0))
    finally:
        srv.shutdown()
        srv.server_close()
    got = out[0]
    assert got["node"] == "a" and all(g["diag"]["mfma"]["pass"] for g in got["gpus"])
    assert not any(k in g["diag"]["mfma"] for g in got["gpus"] for k in DIAG_AGENT_ONLY)
    cache = fanout.ProbeCache(ttl=10.0)
    cache.put(target, got, now=0.0)
    assert "map" not in cache.get(target, now=1.0)["gpus"][0]["diag"]["mfma"]
