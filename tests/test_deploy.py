"""deploy/: every manifest parses, and every container command is accepted by the CLI it runs."""
import glob
import os

import pytest
import yaml

from k8s_gpu_node_checker_amd import cli
from k8s_gpu_node_checker_amd.agent import agent

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MANIFESTS = sorted(glob.glob(os.path.join(REPO, "deploy", "*.yaml")))


def _read(path):
    with open(path, encoding="utf-8") as f:
        return f.read()


def _containers(doc):
    spec = doc.get("spec") or {}
    if doc["kind"] == "CronJob":
        spec = spec["jobTemplate"]["spec"]
    pod = (spec.get("template") or {}).get("spec") or {}
    return pod.get("containers") or []


@pytest.mark.parametrize("path", MANIFESTS, ids=os.path.basename)
def test_manifest_commands_parse(path):
    docs = [d for d in yaml.safe_load_all(_read(path)) if d]
    assert docs and all("kind" in d and "apiVersion" in d for d in docs)
    for d in docs:
        for c in _containers(d):
            cmd = c["command"]
            if cmd[0] == "check-gpu-node":
                cli.parse_args(cmd[1:])
            elif cmd[0] == "k8s-gpu-node-agent":
                agent.build_parser().parse_args(cmd[1:])
            else:
                raise AssertionError(f"unknown entry point {cmd[0]}")


def test_rbac_matches_what_the_code_calls():
    verbs = {}
    for path in MANIFESTS:
        for d in yaml.safe_load_all(_read(path)):
            if d and d["kind"] == "ClusterRole":
                verbs[d["metadata"]["name"]] = {(r, v) for rule in d["rules"] for r in rule["resources"]
                                                for v in rule["verbs"]}
    assert verbs["gpu-node-checker"] == {("nodes", "get"), ("nodes", "list")}  # the reference's contract
    assert ("nodes/status", "patch") in verbs["mi355x-node-agent"] and ("nodes", "patch") in verbs["mi355x-node-agent"]
    assert {("nodes", "get"), ("events", "create")} <= verbs["mi355x-node-agent"]  # taint read-modify-write, events
    assert ("nodes", "watch") in verbs["gpu-node-watcher"]


def test_replicated_watcher_has_the_lease_rbac_its_elector_uses():
    """deploy/watcher.yaml runs 2 replicas with --leader-elect: the Role grants exactly what kube/lease.py calls
    (GET and PUT of the named Lease, POST to create it) in the namespace of the Lease the command names."""
    docs = [d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "watcher.yaml"))) if d]
    dep = next(d for d in docs if d["kind"] == "Deployment")
    cmd = dep["spec"]["template"]["spec"]["containers"][0]["command"]
    args = cli.parse_args(cmd[1:])
    assert dep["spec"]["replicas"] >= 2 and args.leader_elect and args.watch_events
    ns, name = args.leader_elect_lease.split("/")
    env = {e["name"]: e for e in dep["spec"]["template"]["spec"]["containers"][0]["env"]}
    assert env["POD_NAME"]["valueFrom"]["fieldRef"]["fieldPath"] == "metadata.name"
    role = next(d for d in docs if d["kind"] == "Role")
    binding = next(d for d in docs if d["kind"] == "RoleBinding")
    assert role["metadata"]["namespace"] == ns == binding["metadata"]["namespace"]
    assert binding["roleRef"]["name"] == role["metadata"]["name"]
    assert {(s["name"], s["namespace"]) for s in binding["subjects"]} == {
        (dep["spec"]["template"]["spec"]["serviceAccountName"], dep["metadata"]["namespace"])}
    grants = {(v, n) for r in role["rules"] for v in r["verbs"] for n in (r.get("resourceNames") or ["*"])
              if r["resources"] == ["leases"] and r["apiGroups"] == ["coordination.k8s.io"]}
    assert grants == {("get", name), ("update", name), ("create", "*")}


def test_manifests_are_self_consistent():
    """Everything a workload references (namespace, ServiceAccount, PVC) is defined in deploy/, and the
    kustomization lists every manifest."""
    docs = [d for path in MANIFESTS for d in yaml.safe_load_all(_read(path)) if d]
    defined = {(d["kind"], (d.get("metadata") or {}).get("namespace"), d["metadata"]["name"])
               for d in docs if d["kind"] != "Kustomization"}
    namespaces = {name for kind, _, name in defined if kind == "Namespace"}
    for d in docs:
        if d["kind"] in ("Kustomization", "Namespace", "ValidatingAdmissionPolicy",
                         "ValidatingAdmissionPolicyBinding") or d["kind"].startswith("Cluster"):
            continue  # cluster-scoped
        ns = d["metadata"]["namespace"]
        assert ns in namespaces, (d["kind"], d["metadata"]["name"])
        spec = d.get("spec") or {}
        if d["kind"] == "CronJob":
            spec = spec["jobTemplate"]["spec"]
        pod = (spec.get("template") or {}).get("spec")
        if not pod:
            continue
        assert ("ServiceAccount", ns, pod["serviceAccountName"]) in defined, pod["serviceAccountName"]
        for v in pod.get("volumes") or []:
            if "persistentVolumeClaim" in v:
                assert ("PersistentVolumeClaim", ns, v["persistentVolumeClaim"]["claimName"]) in defined
    kust = yaml.safe_load(_read(os.path.join(REPO, "deploy", "kustomization.yaml")))
    assert sorted(kust["resources"]) == sorted(os.path.basename(p) for p in MANIFESTS
                                               if not p.endswith("kustomization.yaml"))


def _pods():
    for path in MANIFESTS:
        for d in yaml.safe_load_all(_read(path)):
            if not d or d["kind"] not in ("DaemonSet", "Deployment", "CronJob", "Job"):
                continue
            spec = d["spec"]["jobTemplate"]["spec"] if d["kind"] == "CronJob" else d["spec"]
            yield os.path.basename(path), spec["template"]["spec"]


def test_gpu_device_access_is_real():
    """A container that mounts /dev/kfd must be able to open it: hostPath device mounts add no
    device-cgroup rule, so it is privileged, or it requests the GPU from the device plugin (which adds the
    rule) and runs in the render/video groups (the unprivileged DaemonSet could not)."""
    seen = 0
    for name, pod in _pods():
        vols = {v["name"]: v for v in pod.get("volumes") or []}
        for c in pod["containers"]:
            mounts = {m["mountPath"]: m["name"] for m in c.get("volumeMounts") or []}
            if "/dev/kfd" not in mounts:
                continue
            seen += 1
            assert vols[mounts["/dev/kfd"]]["hostPath"]["path"] == "/dev/kfd"
            sc = c.get("securityContext") or {}
            if sc.get("privileged"):
                continue
            limits = (c.get("resources") or {}).get("limits") or {}
            groups = set((pod.get("securityContext") or {}).get("supplementalGroups") or [])
            assert any(k.startswith("amd.com/gpu") for k in limits), (name, c["name"])
            assert groups, (name, c["name"], "needs the render/video GIDs")
    assert seen, "no container mounts /dev/kfd"


def test_agent_daemonset_sees_host_pids_and_kubelet_allocations():
    [(name, pod)] = [(n, p) for n, p in _pods() if p["containers"][0]["command"][0] == "k8s-gpu-node-agent"]
    assert pod.get("hostPID") is True
    c = pod["containers"][0]
    args = agent.build_parser().parse_args(c["command"][1:])
    sock = args.pod_resources_socket
    assert sock and args.diag_when == "idle"
    mounted = {m["mountPath"] for m in c["volumeMounts"]}
    assert os.path.dirname(sock) in mounted
    vols = {v["name"]: v for v in pod["volumes"]}
    pr = [m for m in c["volumeMounts"] if m["mountPath"] == os.path.dirname(sock)][0]
    assert vols[pr["name"]]["hostPath"]["path"] == os.path.dirname(sock)
    sc = c["securityContext"]
    assert sc.get("readOnlyRootFilesystem") is True and "/tmp" in mounted  # HIP / amd-smi scratch on tmpfs


def _rich_report():
    """A report carrying every field the agent turns into a metric."""
    from k8s_gpu_node_checker_amd.testing import fixtures
    r = fixtures.mi355x_probe_report("n", gpus=2)
    r["state"] = "healthy"
    g = r["gpus"][0]
    g.update(xgmi_error=0, xgmi_kb=[[1, 2]] * 1, cper={"fatal": 0, "uncorrected": 0, "corrected": 1},
             ecc_blocks={"umc": {"ce": 1, "ue": 0, "de": 0}}, gfx_activity=0,
             throttle={"s": 60, "thermal_pct": 0.0, "power_pct": 1.0, "prochot_pct": 0.0},
             diag={"gemm": {"pass": True, "tflops": 1200.0, "fraction": 0.98, "checksum_bad_tiles": 0,
                            "peers": {"gpus": 2, "ratio": {"tflops": 1.01}},
                            "baseline": {"ratio": {"tflops": 0.99}, "runs": 5}},
                   "gemm_fp8": {"pass": True, "tflops": 2300.0, "checksum_bad_tiles": 0},
                   "mfma": {"pass": True, "kinds": {"bf16": {"tflops": 1900.0, "errors": 0}}},
                   "hbm": {"pass": True, "copy_tbs": 6.4, "read_tbs": 7.0},
                   "hbm_xcd": {"pass": True, "read_tbs": 6.1, "errors": 0, "alone_tbs": {"0": 1.3}},
                   "memtest": {"pass": True, "errors": 0}}, bad_pages=3, bad_pages_pending=1,
             bad_pages_unreservable=0, bad_page_threshold=2048, ecc_ce_per_h=1.5)
    r["fabric"] = {"p2p": {"pass": True, "median_gbps": 50.0, "min_gbps": 48.0},
                   "rccl": {"pass": True, "best_busbw_by_op": {"all_reduce": 300.0}}}
    r["diag_node"] = {"findings": [{"test": "hbm", "metric": "copy_tbs", "median_fraction": 0.9,
                                    "min_fraction": 0.89, "max_fraction": 0.91, "gpus": 2, "below_floor": False}]}
    return r


def test_monitoring_rules_use_metrics_the_agent_emits():
    import re

    from prometheus_client.parser import text_string_to_metric_families
    docs = [d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "monitoring", "monitoring.yaml"))) if d]
    kinds = {d["kind"] for d in docs}
    assert kinds == {"ServiceMonitor", "PrometheusRule"}
    assert {d["metadata"]["name"] for d in docs if d["kind"] == "ServiceMonitor"} == {"mi355x-node-agent",
                                                                                      "gpu-node-watcher"}
    fams = {f.name: f for f in text_string_to_metric_families(agent._metrics(_rich_report()))}
    fams.update(_watcher_families())
    labels = {name: set().union(*(set(s.labels) for s in f.samples)) | {"node"} for name, f in fams.items()}
    rules = [r for d in docs if d["kind"] == "PrometheusRule" for grp in d["spec"]["groups"] for r in grp["rules"]]
    assert len(rules) >= 10
    for r in rules:
        names = set(re.findall(r"\b(?:mi355x|k8s_gpu_checker)_[a-z0-9_]+", r["expr"]))
        assert names, r["alert"]
        for n in names:
            assert n in fams, (r["alert"], n)
        # every label a summary prints exists on the alert's series: a label of its metric(s), the
        # relabelled `node`, or a label the expression aggregates by
        have = set().union(*(labels[n] for n in names))
        outer = re.match(r"\s*count by \(([^)]*)\)", r["expr"])
        if outer:
            have = {x.strip() for x in outer.group(1).split(",")}
        for lbl in re.findall(r"\$labels\.([a-z_]+)", r["annotations"]["summary"]):
            assert lbl in have, (r["alert"], lbl, have)
    # the Service and ServiceMonitor find the DaemonSet's pods and its metrics port
    base = [d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "daemonset.yaml"))) if d]
    ds = next(d for d in base if d["kind"] == "DaemonSet")
    pod_labels = ds["spec"]["template"]["metadata"]["labels"]
    port_names = {p["name"] for c in ds["spec"]["template"]["spec"]["containers"] for p in c.get("ports", [])}
    svc = next(d for d in base if d["kind"] == "Service")
    assert svc["spec"]["selector"].items() <= pod_labels.items()
    assert {p["targetPort"] for p in svc["spec"]["ports"]} <= port_names
    sm = next(d for d in docs if d["kind"] == "ServiceMonitor" and d["metadata"]["name"] == "mi355x-node-agent")
    assert sm["spec"]["selector"]["matchLabels"].items() <= svc["metadata"]["labels"].items()
    assert {e["port"] for e in sm["spec"]["endpoints"]} <= {p["name"] for p in svc["spec"]["ports"]}


def _watcher_families():
    """The metric families the event watcher's /metrics serves (leader: report gauges + leader gauge)."""
    import types

    from prometheus_client.parser import text_string_to_metric_families
    from k8s_gpu_node_checker_amd.models import health as H
    from k8s_gpu_node_checker_amd.utils import prom
    node = {"name": "n0", "ready": True, "gpus": 8, "gpu_breakdown": {"amd.com/gpu": 8}}
    fleet = {"gemm@[4096, 4096, 4096]/tflops": {"nodes": 3, "median_fraction": 0.97, "min_fraction": 0.95,
                                                "max_fraction": 0.99, "platform_shortfall": False, "outliers": []}}
    res = types.SimpleNamespace(gpu_nodes=[node], ready_gpu_nodes=[node], exit_code=0,
                                verdicts=[H.Verdict(H.HEALTHY)], tracer=None, fleet_diag=fleet)
    srv = prom.MetricsServer("127.0.0.1", 0)
    try:
        srv.update(res)
        srv.set_leader(True)
        srv.update(res)
        return {f.name: f for f in text_string_to_metric_families(srv.text())}
    finally:
        srv.httpd.server_close()


def _all_deploy_docs():
    for path in sorted(glob.glob(os.path.join(REPO, "deploy", "**", "*.yaml"), recursive=True)):
        for d in yaml.safe_load_all(_read(path)):
            if isinstance(d, dict) and "kind" in d:
                yield os.path.relpath(path, REPO), d


def _pod_of(doc):
    spec = doc.get("spec") or {}
    if doc["kind"] == "CronJob":
        spec = spec["jobTemplate"]["spec"]
    return spec.get("template")


def test_every_metrics_output_in_deploy_has_a_consumer():
    """Each metrics output a workload in deploy/ produces is read by something: an HTTP /metrics port is behind
    a Service that a ServiceMonitor scrapes on that port; a --prometheus-textfile is on a volume another
    container of the pod (a node-exporter) mounts.  No metrics written into the void."""
    # kustomize patches (deploy/level2/) amend a base workload checked here in full: not workloads of their own
    patches = {os.path.normpath(os.path.join(os.path.dirname(p), x["path"]))
               for p, d in _all_deploy_docs() if d["kind"] == "Kustomization" for x in d.get("patches") or []}
    docs = [(p, d) for p, d in _all_deploy_docs() if p not in patches]
    services = [d for _, d in docs if d["kind"] == "Service"]
    monitors = [d for _, d in docs if d["kind"] == "ServiceMonitor"]
    outputs = 0
    for path, d in docs:
        tpl = _pod_of(d) if d["kind"] in ("DaemonSet", "Deployment", "CronJob", "Job") else None
        if not tpl or "containers" not in (tpl.get("spec") or {}):
            continue
        pod, labels, ns = tpl["spec"], (tpl.get("metadata") or {}).get("labels") or {}, d["metadata"].get("namespace")
        for c in pod["containers"]:
            cmd = c.get("command") or []
            ports, textfiles = [], []
            if cmd and cmd[0] == "k8s-gpu-node-agent":
                a = agent.build_parser().parse_args(cmd[1:])
                if "http" in a.publish.split(","):
                    ports.append(int(a.listen.rpartition(":")[2]))
            elif cmd and cmd[0] == "check-gpu-node":
                a = cli.parse_args(cmd[1:])
                if a.metrics_listen:
                    ports.append(int(a.metrics_listen.rpartition(":")[2]))
                if a.prometheus_textfile:
                    textfiles.append(a.prometheus_textfile)
            for port in ports:
                outputs += 1
                named = {p["containerPort"]: p.get("name") for p in c.get("ports") or []}
                assert port in named, (path, c["name"], port)
                scraped = False
                for svc in services:
                    if svc["metadata"].get("namespace") != ns or not svc["spec"].get("selector"):
                        continue
                    if not svc["spec"]["selector"].items() <= labels.items():
                        continue
                    sports = [p["name"] for p in svc["spec"]["ports"] if p.get("targetPort") in (port, named[port])]
                    for sm in monitors:
                        if (sm["spec"]["selector"]["matchLabels"].items() <= (svc["metadata"].get("labels") or {}).items()
                                and any(e["port"] in sports for e in sm["spec"]["endpoints"])):
                            scraped = True
                assert scraped, f"{path}: {c['name']} serves /metrics on {port} but no ServiceMonitor scrapes it"
            for tf in textfiles:
                outputs += 1
                mine = [m for m in c.get("volumeMounts") or [] if tf.startswith(m["mountPath"].rstrip("/") + "/")]
                assert mine, (path, tf, "textfile not on a volume")
                readers = [o for o in pod["containers"] if o is not c
                           and any(m["name"] == mine[0]["name"] for m in o.get("volumeMounts") or [])]
                assert readers, f"{path}: {c['name']} writes {tf} but no container of the pod reads it"
    assert outputs >= 2  # the agent's /metrics and the watcher's


def test_grafana_dashboard_queries_series_that_exist():
    """deploy/monitoring/dashboard.yaml (generated by tools/make_dashboard.py): valid dashboard JSON with unique
    panel ids, listed in the monitoring kustomization, and every metric it queries is one the agent's /metrics or
    the checker's textfile emits (so no panel is silently empty), with every label its legends use."""
    import json
    import re
    import subprocess
    import sys
    import types

    from prometheus_client.parser import text_string_to_metric_families
    from k8s_gpu_node_checker_amd.utils import prom
    path = os.path.join(REPO, "deploy", "monitoring", "dashboard.yaml")
    before = _read(path)
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "make_dashboard.py")], check=True, capture_output=True)
    assert _read(path) == before, "deploy/monitoring/dashboard.yaml is stale: run tools/make_dashboard.py"
    cm = yaml.safe_load(before)
    assert cm["kind"] == "ConfigMap" and cm["metadata"]["labels"]["grafana_dashboard"] == "1"
    assert "dashboard.yaml" in yaml.safe_load(_read(os.path.join(REPO, "deploy", "monitoring",
                                                                 "kustomization.yaml")))["resources"]
    dash = json.loads(cm["data"]["mi355x-node-health.json"])
    ids = [p["id"] for p in dash["panels"]]
    assert len(ids) == len(set(ids)) and dash["uid"] == "mi355x-node-health"
    fams = {f.name: f for f in text_string_to_metric_families(agent._metrics(_rich_report()))}
    node = {"name": "n0", "ready": True, "gpus": 8, "gpu_breakdown": {"amd.com/gpu": 8}}
    fleet = {"gemm@[4096, 4096, 4096]/tflops": {"nodes": 3, "median_fraction": 0.97, "min_fraction": 0.95,
                                                "max_fraction": 0.99, "platform_shortfall": False, "outliers": []}}
    res = types.SimpleNamespace(gpu_nodes=[node], ready_gpu_nodes=[node], exit_code=0, verdicts=[], tracer=None,
                                fleet_diag=fleet)
    fams.update({f.name: f for f in text_string_to_metric_families("\n".join(prom.render(res)) + "\n")})
    queried = 0
    for p in dash["panels"]:
        for t in p.get("targets", []):
            for name in re.findall(r"\b((?:mi355x|k8s_gpu_checker)_[a-z0-9_]+)", t["expr"]):
                assert name in fams, (p["title"], name)
                queried += 1
                have = set().union(*(set(s.labels) for s in fams[name].samples)) | {"node"}
                for lbl in re.findall(r"\{\{(\w+)\}\}", t["legendFormat"]):
                    assert lbl in have, (p["title"], lbl)
    assert queried >= 25


def test_agent_metrics_carry_the_verdict_state():
    from prometheus_client.parser import text_string_to_metric_families
    r = _rich_report()
    r["state"] = "degraded"
    fams = {f.name: f for f in text_string_to_metric_families(agent._metrics(r))}
    assert {s.labels["state"]: s.value for s in fams["mi355x_node_health"].samples} == {
        "healthy": 0, "degraded": 1, "unhealthy": 0, "unknown": 0}


def test_image_carries_every_third_party_runtime_import():
    """Every non-stdlib module the package imports is either installed in the image's runtime stage or is
    optional by design (torch: bench / torchrun collectives; amdsmi: the Python probe fallback, shipped by
    ROCm itself; charset_normalizer: the guess of an undeclared webhook-error encoding, as requests makes it,
    with a UTF-8/latin-1 fallback; prometheus_client / requests: tests and tools only)."""
    import ast
    import sys
    pkg = os.path.join(REPO, "k8s_gpu_node_checker_amd")
    mods = set()
    for root, _, files in os.walk(pkg):
        if "testing" in root.split(os.sep):
            continue
        for f in files:
            if f.endswith(".py"):
                tree = ast.parse(_read(os.path.join(root, f)))
                for n in ast.walk(tree):
                    if isinstance(n, ast.Import):
                        mods |= {a.name.split(".")[0] for a in n.names}
                    elif isinstance(n, ast.ImportFrom) and n.level == 0 and n.module:
                        mods.add(n.module.split(".")[0])
    third = {m for m in mods if m not in sys.stdlib_module_names and m != "k8s_gpu_node_checker_amd"}
    # the runtime stage copies the build stage's venv: third-party modules are whatever its pip install names
    lines = [ln for ln in _read(os.path.join(REPO, "deploy", "Dockerfile")).splitlines() if not ln.lstrip().startswith("#")]
    pip = " ".join(ln for ln in lines if "/opt/venv/bin/pip install" in ln)
    assert "COPY --from=build /opt/venv /opt/venv" in lines
    installed = {"yaml": "PyYAML" in pip, "grpc": "grpcio" in pip}
    optional = {"torch", "amdsmi", "charset_normalizer"}
    assert third <= set(installed) | optional, third - set(installed) - optional
    assert all(installed[m] for m in third & set(installed)), installed


def test_agent_port_network_policy_selects_the_agent_and_its_port():
    pol = next(d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "monitoring", "networkpolicy.yaml")))
               if d)
    ds = next(d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "daemonset.yaml"))) if d)
    pod = ds["spec"]["template"]
    assert pol["metadata"]["namespace"] == ds["metadata"]["namespace"]
    assert pol["spec"]["podSelector"]["matchLabels"].items() <= pod["metadata"]["labels"].items()
    assert not pod["spec"].get("hostNetwork")  # a host-network pod would ignore the policy
    ports = {p["name"] for c in pod["spec"]["containers"] for p in c.get("ports", [])}
    assert {p["port"] for r in pol["spec"]["ingress"] for p in r["ports"]} <= ports
    kust = yaml.safe_load(_read(os.path.join(REPO, "deploy", "monitoring", "kustomization.yaml")))
    assert "networkpolicy.yaml" in kust["resources"]


# --- the agent's write authority is scoped to its own Node (deploy/agent-policy.yaml) ------------------------

import copy  # noqa: E402

from k8s_gpu_node_checker_amd.models import health as H  # noqa: E402
from k8s_gpu_node_checker_amd.models.node import HEALTH_ANNOTATION  # noqa: E402
from k8s_gpu_node_checker_amd.testing import cel, fixtures  # noqa: E402

AGENT_USER = "system:serviceaccount:gpu-health:mi355x-node-agent"


def _policy():
    docs = [d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "agent-policy.yaml"))) if d]
    pol = next(d for d in docs if d["kind"] == "ValidatingAdmissionPolicy")
    binding = next(d for d in docs if d["kind"] == "ValidatingAdmissionPolicyBinding")
    return pol, binding


def _req(resource="nodes", sub="", user=AGENT_USER, node_claim="gpu-a", op="UPDATE"):
    extra = {} if node_claim is None else {"authentication.kubernetes.io/node-name": [node_claim]}
    return {"operation": op, "resource": {"group": "", "version": "v1", "resource": resource}, "subResource": sub,
            "userInfo": {"username": user, "extra": extra}}


def _node(name="gpu-a"):
    return fixtures.realistic_node(name, gpu_count=8)


def _admit(req, new, old):
    pol, _ = _policy()
    return cel.admit(pol, req, new, old)


def test_policy_is_bound_to_the_agent_service_account_and_names_the_node_claim():
    pol, binding = _policy()
    assert binding["spec"]["policyName"] == pol["metadata"]["name"] and binding["spec"]["validationActions"] == ["Deny"]
    assert pol["spec"]["failurePolicy"] == "Fail"
    mc = " ".join(m["expression"] for m in pol["spec"]["matchConditions"])
    assert AGENT_USER in mc
    sa = next(d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "rbac.yaml")))
              if d and d["kind"] == "ServiceAccount" and d["metadata"]["name"] == "mi355x-node-agent")
    assert AGENT_USER == f"system:serviceaccount:{sa['metadata']['namespace']}:{sa['metadata']['name']}"
    assert "authentication.kubernetes.io/node-name" in yaml.safe_dump(pol)
    rules = {(r, o) for rr in pol["spec"]["matchConstraints"]["resourceRules"] for r in rr["resources"]
             for o in rr["operations"]}
    assert {("nodes", "UPDATE"), ("nodes/status", "UPDATE"), ("events", "CREATE")} <= rules
    kust = yaml.safe_load(_read(os.path.join(REPO, "deploy", "kustomization.yaml")))
    assert "agent-policy.yaml" in kust["resources"]


def test_policy_admits_every_write_the_agent_makes_to_its_own_node():
    old = _node()
    ann = copy.deepcopy(old)
    ann["metadata"]["annotations"][HEALTH_ANNOTATION] = '{"schema":"mi355x-health/v1"}'
    assert _admit(_req(), ann, old) == (True, "")
    lab = copy.deepcopy(old)
    lab["metadata"]["labels"].update({"amd.com/mi355x-health": "healthy", "amd.com/gpu.count": "8"})
    del lab["metadata"]["labels"]["amd.com/gpu.family"]  # an amd.com/ label the agent removes
    assert _admit(_req(), lab, old) == (True, "")
    tainted = copy.deepcopy(old)
    tainted["spec"]["taints"] = list(old["spec"].get("taints") or []) + [dict(H.UNHEALTHY_TAINT)]
    assert _admit(_req(), tainted, old) == (True, "")
    assert _admit(_req(), old, tainted) == (True, "")  # and removes it again
    st = copy.deepcopy(old)
    st["status"]["conditions"] = old["status"]["conditions"] + [
        {"type": H.HEALTH_CONDITION, "status": "True", "reason": "MI355XHealthy", "message": "8/8"}]
    assert _admit(_req(sub="status"), st, old) == (True, "")
    ev = {"involvedObject": {"kind": "Node", "name": "gpu-a"}, "reason": "MI355XUnhealthy"}
    assert _admit(_req(resource="events", op="CREATE"), ev, None) == (True, "")


def test_policy_refuses_writes_to_other_nodes_and_other_fields():
    old = _node()
    ann = copy.deepcopy(old)
    ann["metadata"]["annotations"][HEALTH_ANNOTATION] = "{}"
    # a compromised agent on gpu-b writing gpu-a's verdict
    ok, msg = _admit(_req(node_claim="gpu-b"), ann, old)
    assert ok is False and msg == "the MI355X node agent on gpu-b may only write its own Node, not gpu-a"
    ok, msg = _admit(_req(node_claim=None), ann, old)  # a token without the claim: fail closed
    assert ok is False and "node-name claim" in msg
    bad = copy.deepcopy(old)
    bad["metadata"]["labels"]["pool"] = "inference"
    assert _admit(_req(), bad, old) == (False, "the MI355X node agent may only change amd.com/ labels")
    bad = copy.deepcopy(old)
    del bad["metadata"]["labels"]["pool"]
    assert _admit(_req(), bad, old)[0] is False
    bad = copy.deepcopy(old)
    bad["metadata"]["annotations"]["node.alpha.kubernetes.io/ttl"] = "30"
    assert _admit(_req(), bad, old) == (False, "the MI355X node agent may only change the amd.com/mi355x-health "
                                               "annotation")
    bad = copy.deepcopy(old)
    bad["spec"]["taints"] = [{"key": "dedicated", "value": "x", "effect": "NoExecute"}]
    assert _admit(_req(), bad, old)[1] == "the MI355X node agent may only add or remove the amd.com/gpu-unhealthy taint"
    bad = copy.deepcopy(old)
    bad["spec"]["unschedulable"] = True
    assert _admit(_req(), bad, old)[1] == ("the MI355X node agent may only change the amd.com/gpu-unhealthy taint in a "
                                           "Node's spec (no cordon, no re-addressing)")
    bad = copy.deepcopy(old)
    bad["status"]["conditions"][0] = dict(bad["status"]["conditions"][0], status="Unknown")  # the kubelet's Ready
    assert _admit(_req(sub="status"), bad, old)[0] is False
    bad = copy.deepcopy(old)
    bad["status"]["capacity"]["amd.com/gpu"] = "0"
    assert _admit(_req(sub="status"), bad, old)[0] is False
    ev = {"involvedObject": {"kind": "Node", "name": "gpu-z"}, "reason": "MI355XHealthy"}
    assert _admit(_req(resource="events", op="CREATE"), ev, None) == (
        False, "the MI355X node agent may only post Events about its own Node")
    # other users are not this policy's business (the kubelet, an operator)
    assert _admit(_req(user="system:node:gpu-a"), bad, old) == (None, "")


def _full_node():
    """A Node carrying every optional spec / status / metadata field the policy guards."""
    n = _node()
    n["metadata"]["finalizers"] = ["example.com/decommission"]
    n["metadata"]["ownerReferences"] = [{"apiVersion": "example.com/v1", "kind": "Machine", "name": "m-1",
                                         "uid": "0000-1111"}]
    n["spec"]["configSource"] = {"configMap": {"name": "kubelet", "namespace": "kube-system",
                                               "kubeletConfigKey": "kubelet"}}
    n["spec"]["externalID"] = "i-0123456789"
    n["status"]["phase"] = "Running"
    n["status"]["volumesInUse"] = ["kubernetes.io/csi/ebs.csi.aws.com^vol-1"]
    n["status"]["volumesAttached"] = [{"name": "kubernetes.io/csi/ebs.csi.aws.com^vol-1", "devicePath": ""}]
    n["status"]["config"] = {"active": {"configMap": {"name": "kubelet", "namespace": "kube-system"}}}
    n["status"]["runtimeHandlers"] = [{"name": "runc", "features": {"recursiveReadOnlyMounts": True}}]
    n["status"]["features"] = {"supplementalGroupsPolicy": True}
    return n


def _drop(path):
    def f(n):
        obj = n
        for k in path[:-1]:
            obj = obj[k]
        del obj[path[-1]]
    return f


SPEC_MSG = "the MI355X node agent may only change the amd.com/gpu-unhealthy taint in a Node's spec (no cordon, no re-addressing)"
STATUS_MSG = "the MI355X node agent may only change its AMDGPUHealthy condition in a Node's status"
META_MSG = "the MI355X node agent may not change a Node's finalizers or ownerReferences"
GUARDED = [  # (subresource, field, mutation, refusal): one refused agent write per guarded field
    ("status", "addresses", lambda n: n["status"]["addresses"][0].update(address="10.66.0.1"), STATUS_MSG),
    ("status", "nodeInfo", lambda n: n["status"]["nodeInfo"].update(kubeletVersion="v1.99.0"), STATUS_MSG),
    ("status", "daemonEndpoints", lambda n: n["status"]["daemonEndpoints"]["kubeletEndpoint"].update(Port=1),
     STATUS_MSG),
    ("status", "images", lambda n: n["status"]["images"].pop(), STATUS_MSG),
    ("status", "volumesInUse", _drop(["status", "volumesInUse"]), STATUS_MSG),
    ("status", "volumesAttached", lambda n: n["status"]["volumesAttached"].append({"name": "x", "devicePath": ""}),
     STATUS_MSG),
    ("status", "phase", lambda n: n["status"].update(phase="Terminated"), STATUS_MSG),
    ("status", "config", _drop(["status", "config"]), STATUS_MSG),
    ("status", "runtimeHandlers", lambda n: n["status"]["runtimeHandlers"][0].update(name="kata"), STATUS_MSG),
    ("status", "features", lambda n: n["status"]["features"].update(supplementalGroupsPolicy=False), STATUS_MSG),
    ("status", "capacity", lambda n: n["status"]["capacity"].update(cpu="1"), STATUS_MSG),
    ("status", "allocatable", _drop(["status", "allocatable"]), STATUS_MSG),
    ("", "podCIDR", lambda n: n["spec"].update(podCIDR="10.0.0.0/8"), SPEC_MSG),
    ("", "podCIDRs", lambda n: n["spec"]["podCIDRs"].append("fd00::/64"), SPEC_MSG),
    ("", "providerID", _drop(["spec", "providerID"]), SPEC_MSG),
    ("", "configSource", lambda n: n["spec"]["configSource"]["configMap"].update(name="evil"), SPEC_MSG),
    ("", "externalID", lambda n: n["spec"].update(externalID="i-other"), SPEC_MSG),
    ("", "unschedulable", lambda n: n["spec"].update(unschedulable=True), SPEC_MSG),
    ("", "finalizers", lambda n: n["metadata"].update(finalizers=[]), META_MSG),
    ("status", "finalizers", _drop(["metadata", "finalizers"]), META_MSG),
    ("", "ownerReferences", lambda n: n["metadata"]["ownerReferences"].append(
        {"apiVersion": "v1", "kind": "Pod", "name": "p", "uid": "u"}), META_MSG),
]


@pytest.mark.parametrize("sub,field,mutate,msg", GUARDED, ids=[f"{s or 'main'}-{f}" for s, f, _, _ in GUARDED])
def test_policy_refuses_a_write_to_every_guarded_field(sub, field, mutate, msg):
    old = _full_node()
    assert _admit(_req(sub=sub), copy.deepcopy(old), old) == (True, "")  # the unchanged node is admitted
    new = copy.deepcopy(old)
    mutate(new)
    assert new != old
    assert _admit(_req(sub=sub), new, old) == (False, msg)
    # a field that was absent and appears is refused as well
    if field in ("phase", "externalID", "features"):
        where = "status" if sub == "status" else "spec"
        bare = copy.deepcopy(old)
        del bare[where][field]
        assert _admit(_req(sub=sub), old, bare) == (False, msg)


def test_policy_header_names_every_guarded_field():
    text = _read(os.path.join(REPO, "deploy", "agent-policy.yaml"))
    header = text.split("apiVersion:")[0]
    for _, field, _, _ in GUARDED:
        assert field in header, field


class _RecordingClient:
    """The agent's KubeClient against the mock apiserver; each node write is recorded as (subresource, merged
    Node after, Node before) -- what admission sees -- and each Event as posted."""

    def __init__(self, kc, srv, node):
        self.kc, self.srv, self.node = kc, srv, node
        self.writes = []
        self.events = []
        self.calls = []

    def _snap(self):
        return copy.deepcopy(self.srv.state.find(self.node))

    def __getattr__(self, name):
        fn = getattr(self.kc, name)
        sub = {"patch_node_condition": "status", "patch_node_annotations": "", "patch_node_labels": "",
               "update_node_taints": ""}.get(name)
        if name == "create_event":
            def post(namespace, ev, *a, **kw):
                self.events.append(copy.deepcopy(ev))
                return fn(namespace, ev, *a, **kw)
            return post
        if sub is None:
            return fn

        def write(*a, **kw):
            before = self._snap()
            out = fn(*a, **kw)
            self.calls.append(name)
            self.writes.append((sub, self._snap(), before))
            return out
        return write


def test_policy_admits_the_agents_real_patches_replayed_through_the_apiserver(mock_cluster):
    """The agent's own condition, annotation (JSON and gzip), label, taint and Event writes -- healthy, then
    an uncorrectable ECC error (unhealthy: taint added, labels and condition flip), then recovered -- on a Node
    carrying every guarded field: each merged result is admitted."""
    from k8s_gpu_node_checker_amd.kube.client import KubeClient
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    srv = mock_cluster([_full_node()])
    healthy = fixtures.mi355x_probe_report("gpu-a", gpus=8)
    sick = copy.deepcopy(healthy)
    sick["gpus"][2]["ecc_uncorrectable"] = 4
    kinds = set()
    for encoding in ("json", "gzip"):
        ag = agent.Agent("gpu-a", source="fixture", label_node=True, taint_unhealthy=True,
                         annotation_encoding=encoding, expect_gpus=8)
        with KubeClient(ClusterConnection(srv.url)) as kc:
            rec = _RecordingClient(kc, srv, "gpu-a")
            for rep in (healthy, sick, healthy):
                rep = dict(rep, ts=__import__("time").time())
                ag.publish(rec, rep, force=True)
        assert set(rec.calls) == {"patch_node_condition", "patch_node_annotations", "patch_node_labels",
                                  "update_node_taints"}, rec.calls
        for sub, new, old in rec.writes:
            assert new != old or sub == ""
            assert _admit(_req(sub=sub), new, old) == (True, ""), (sub, encoding)
            kinds.add(sub)
        for ev in rec.events:
            assert _admit(_req(resource="events", op="CREATE"), ev, None) == (True, "")
        assert len(rec.events) >= 2
    assert kinds == {"", "status"}
    final = srv.state.find("gpu-a")
    assert final["metadata"]["finalizers"] == ["example.com/decommission"]
    assert not any(t["key"] == H.UNHEALTHY_TAINT["key"] for t in final["spec"].get("taints") or [])


def test_cel_subset_semantics():
    e = cel.eval_expr
    assert e("[1, 2, 3].filter(x, x > 1) == [2, 3]", {}) is True
    assert e("{'a': 1, 'b': 2}.all(k, k.startsWith('a') || k == 'b')", {}) is True
    assert e("has(o.a) && o.a.b == 1 ? 'y' : 'n'", {"o": {"a": {"b": 1}}}) == "y"
    assert e("has(o.x) ? 1 : 2", {"o": {}}) == 2
    assert e("o.x == 1 || true", {"o": {}}) is True  # commutative with errors
    with pytest.raises(cel.CelError):
        e("o.x == 1 && true", {"o": {}})
    assert e("'k' in m && size(m['k']) == 2", {"m": {"k": ["a", "b"]}}) is True
    assert e("true == 1", {}) is False


# --- memory limits from the measured budget ---------------------------------------------------

def _mib(q):
    units = {"Ki": 1 / 1024, "Mi": 1, "Gi": 1024}
    for u, f in units.items():
        if q.endswith(u):
            return float(q[:-2]) * f
    return float(q) / (1 << 20)


def _agent_container(doc):
    return next(c for c in doc["spec"]["template"]["spec"]["containers"] if c["name"] == "agent")


def test_daemonset_memory_limit_covers_the_budget_of_an_eight_gpu_node():
    ds = next(d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "daemonset.yaml"))) if d)
    c = _agent_container(ds)
    level = int(c["command"][c["command"].index("--diag-level") + 1])
    assert level == 1
    args = agent.build_parser().parse_args(c["command"][1:])
    assert args.diag_isolation == "process"  # the budget below is the process-isolation one
    assert _mib(c["resources"]["limits"]["memory"]) >= agent.memory_budget_mib(8, level, parallel=args.diag_parallel)
    # the request is what stays resident (measured), not a first-launch cost
    req = _mib(c["resources"]["requests"]["memory"])
    assert agent.MEM_RESIDENT_MIB <= req <= 2 * agent.MEM_RESIDENT_MIB
    # the measured one-GPU figures (profiles/agent_soak_isolated_l{1,2}_r06_mi355x.json)
    assert agent.memory_budget_mib(1, 1) == 65 + 493 and agent.memory_budget_mib(1, 2) == 65 + 1128
    assert agent.memory_budget_mib(8, 1, parallel=2) == 65 + 2 * 493  # children at once, not devices, count
    assert agent.memory_budget_mib(8, 2, rccl=True, parallel=4) == 65 + 2712 + 7 * 682  # the fabric child bounds it
    assert agent.memory_budget_mib(1, 2, rccl=True) >= agent.memory_budget_mib(1, 2)


def test_level2_overlay_keeps_the_comgr_cache_and_sizes_both_containers():
    base = os.path.join(REPO, "deploy", "level2")
    kust = yaml.safe_load(_read(os.path.join(base, "kustomization.yaml")))
    assert kust["resources"] == ["../"] and kust["patches"][0]["path"] == "daemonset-level2.yaml"
    patch = yaml.safe_load(_read(os.path.join(base, "daemonset-level2.yaml")))
    c = _agent_container(patch)
    agent.build_parser().parse_args(c["command"][1:])
    assert c["command"][c["command"].index("--diag-level") + 1] == "2"
    args = agent.build_parser().parse_args(c["command"][1:])
    assert _mib(c["resources"]["limits"]["memory"]) >= agent.memory_budget_mib(8, 2, rccl=True,
                                                                               parallel=args.diag_parallel)
    assert agent.MEM_RESIDENT_MIB <= _mib(c["resources"]["requests"]["memory"]) <= 2 * agent.MEM_RESIDENT_MIB
    init = patch["spec"]["template"]["spec"]["initContainers"][0]
    assert init["command"][0] == "mi355x-fabric"
    from k8s_gpu_node_checker_amd.ops import fabric
    fabric.main.__code__  # the console script's target exists
    assert '"mi355x-fabric = k8s_gpu_node_checker_amd.ops.fabric:main"' in _read(os.path.join(REPO, "setup.py"))
    assert _mib(init["resources"]["limits"]["memory"]) >= agent.MEM_RCCL_COLD_PEAK_MIB
    for ctr in (c, init):
        env = {e["name"]: e["value"] for e in ctr["env"]}
        mount = next(m["mountPath"] for m in ctr["volumeMounts"] if m["name"] == "comgr-cache")
        assert env["AMD_COMGR_CACHE_DIR"].startswith(mount)
    vol = next(v for v in patch["spec"]["template"]["spec"]["volumes"] if v["name"] == "comgr-cache")
    assert vol["hostPath"]["type"] == "DirectoryOrCreate"


def test_agent_baseline_file_is_on_a_writable_host_volume():
    """--diag-baseline-file must sit on a mounted hostPath (the root filesystem is read-only) so each GPU's
    self-baseline survives agent restarts; the level-2 overlay keeps the same file."""
    ds = next(d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "daemonset.yaml"))) if d)
    pod = ds["spec"]["template"]["spec"]
    c = pod["containers"][0]
    overlay = yaml.safe_load(_read(os.path.join(REPO, "deploy", "level2", "daemonset-level2.yaml")))
    for cmd in (c["command"], _agent_container(overlay)["command"]):
        path = agent.build_parser().parse_args(cmd[1:]).diag_baseline_file
        assert path == "/var/lib/mi355x-node-agent/baseline.json"
        mount = next(m for m in c["volumeMounts"] if m["mountPath"] == os.path.dirname(path))
        assert not mount.get("readOnly")
        vol = next(v for v in pod["volumes"] if v["name"] == mount["name"])
        assert vol["hostPath"] == {"path": os.path.dirname(path), "type": "DirectoryOrCreate"}


def test_every_alert_has_a_runbook_section():
    """RUNBOOK.md has a section per alert of deploy/monitoring/monitoring.yaml, and no section for an alert that
    is gone."""
    import re
    docs = list(yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "monitoring", "monitoring.yaml"))))
    alerts = {r["alert"] for d in docs if d and d["kind"] == "PrometheusRule" for g in d["spec"]["groups"]
              for r in g["rules"]}
    sections = set(re.findall(r"^## (\S+)\s*$", _read(os.path.join(REPO, "RUNBOOK.md")), re.M))
    assert alerts and alerts == sections, (alerts - sections, sections - alerts)


def test_mtls_overlay_serves_the_agent_over_tls_and_documents_a_checker_that_reads_it():
    """deploy/mtls/: the agent's command is the base command plus the three TLS flags, whose files are on the
    mounted Secret; the kubelet probes switch to HTTPS; the checker command the overlay documents parses, uses
    {pod_ip} over https and verifies against the Service's DNS name."""
    import re
    import shlex
    base = os.path.join(REPO, "deploy", "mtls")
    kust_text = _read(os.path.join(base, "kustomization.yaml"))
    kust = yaml.safe_load(kust_text)
    assert kust["resources"] == ["../"] and kust["patches"][0]["path"] == "daemonset-mtls.yaml"
    patch = yaml.safe_load(_read(os.path.join(base, "daemonset-mtls.yaml")))
    c = _agent_container(patch)
    ds = next(d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "daemonset.yaml"))) if d)
    base_cmd = ds["spec"]["template"]["spec"]["containers"][0]["command"]
    assert c["command"][:len(base_cmd)] == base_cmd  # nothing else of the agent changes
    a = agent.build_parser().parse_args(c["command"][1:])
    mount = next(m for m in c["volumeMounts"] if m["name"] == "tls")
    for path in (a.tls_cert_file, a.tls_key_file, a.tls_client_ca):
        assert path and os.path.dirname(path) == mount["mountPath"]
    vol = next(v for v in patch["spec"]["template"]["spec"]["volumes"] if v["name"] == "tls")
    assert vol["secret"]["secretName"] == "mi355x-node-agent-tls" and mount["readOnly"]
    for probe in ("readinessProbe", "livenessProbe"):
        assert c[probe]["httpGet"]["scheme"] == "HTTPS" and c[probe]["httpGet"]["path"] == "/healthz"
    # the documented checker command
    doc = " ".join(ln.lstrip("# ").rstrip("\\ ") for ln in kust_text.splitlines() if ln.startswith("#"))
    m = re.search(r"(check-gpu-node --mi355x .*?--probe-client-key \S+)", doc)
    assert m, doc
    from k8s_gpu_node_checker_amd import cli
    args = cli.parse_args(shlex.split(m.group(1))[1:])
    assert args.probe_endpoint == "https://{pod_ip}:9464/probe"
    svc = next(d for d in yaml.safe_load_all(_read(os.path.join(REPO, "deploy", "daemonset.yaml")))
               if d and d["kind"] == "Service")
    assert args.probe_tls_server_name == f"{svc['metadata']['name']}.{svc['metadata']['namespace']}.svc"
    assert args.probe_ca and args.probe_client_cert and args.probe_client_key


def test_monitoring_mtls_overlay_scrapes_the_tls_agents():
    """deploy/monitoring/mtls/: the agents' ServiceMonitor endpoint is the base one (port, path, interval,
    relabelings -- the list is replaced whole, CRD lists do not merge) plus https and a tlsConfig naming the same
    Service DNS name as deploy/mtls/."""
    base_dir = os.path.join(REPO, "deploy", "monitoring")
    kust = yaml.safe_load(_read(os.path.join(base_dir, "mtls", "kustomization.yaml")))
    assert kust["resources"] == ["../"] and kust["patches"][0]["path"] == "servicemonitor-mtls.yaml"
    patch = yaml.safe_load(_read(os.path.join(base_dir, "mtls", "servicemonitor-mtls.yaml")))
    base = next(d for d in yaml.safe_load_all(_read(os.path.join(base_dir, "monitoring.yaml")))
                if d and d["kind"] == "ServiceMonitor" and d["metadata"]["name"] == patch["metadata"]["name"])
    (ep,), (base_ep,) = patch["spec"]["endpoints"], base["spec"]["endpoints"]
    assert {k: v for k, v in ep.items() if k not in ("scheme", "tlsConfig")} == base_ep
    assert ep["scheme"] == "https"
    tls = ep["tlsConfig"]
    assert tls["serverName"] == "mi355x-node-agent.gpu-health.svc"
    assert tls["ca"]["secret"]["key"] == "ca.crt" and tls["cert"]["secret"]["key"] == "tls.crt"
    assert tls["keySecret"]["key"] == "tls.key"
    assert "mi355x-node-agent.gpu-health.svc" in _read(os.path.join(REPO, "deploy", "mtls", "kustomization.yaml"))
