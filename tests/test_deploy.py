"""deploy/: every manifest parses, and every container command is accepted by the CLI it runs."""
import glob
import os

import pytest
import yaml

from k8s_gpu_node_checker_amd import cli
from k8s_gpu_node_checker_amd.agent import agent

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MANIFESTS = sorted(glob.glob(os.path.join(REPO, "deploy", "*.yaml")))


def _containers(doc):
    spec = doc.get("spec") or {}
    if doc["kind"] == "CronJob":
        spec = spec["jobTemplate"]["spec"]
    pod = (spec.get("template") or {}).get("spec") or {}
    return pod.get("containers") or []


@pytest.mark.parametrize("path", MANIFESTS, ids=os.path.basename)
def test_manifest_commands_parse(path):
    docs = [d for d in yaml.safe_load_all(open(path)) if d]
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
        for d in yaml.safe_load_all(open(path)):
            if d and d["kind"] == "ClusterRole":
                verbs[d["metadata"]["name"]] = {(r, v) for rule in d["rules"] for r in rule["resources"]
                                                for v in rule["verbs"]}
    assert verbs["gpu-node-checker"] == {("nodes", "get"), ("nodes", "list")}  # the reference's contract
    assert ("nodes/status", "patch") in verbs["mi355x-node-agent"] and ("nodes", "patch") in verbs["mi355x-node-agent"]
    assert {("nodes", "get"), ("events", "create")} <= verbs["mi355x-node-agent"]  # taint read-modify-write, events
    assert ("nodes", "watch") in verbs["gpu-node-watcher"]


def test_manifests_are_self_consistent():
    """Everything a workload references (namespace, ServiceAccount, PVC) is defined in deploy/, and the
    kustomization lists every manifest."""
    docs = [d for path in MANIFESTS for d in yaml.safe_load_all(open(path)) if d]
    defined = {(d["kind"], (d.get("metadata") or {}).get("namespace"), d["metadata"]["name"])
               for d in docs if d["kind"] != "Kustomization"}
    namespaces = {name for kind, _, name in defined if kind == "Namespace"}
    for d in docs:
        if d["kind"] in ("Kustomization", "Namespace") or d["kind"].startswith("Cluster"):
            continue
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
    kust = yaml.safe_load(open(os.path.join(REPO, "deploy", "kustomization.yaml")))
    assert sorted(kust["resources"]) == sorted(os.path.basename(p) for p in MANIFESTS
                                               if not p.endswith("kustomization.yaml"))
