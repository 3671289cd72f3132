"""``check-gpu-node --explain NODE``: one node's Ready verdict, its AMDGPUHealthy condition and the GPU
rows of its report, with the reference's exit codes applied to that node."""
import json

from k8s_gpu_node_checker_amd.models import health as H
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig


def _cluster(mock_cluster, tmp_path):
    bad = fixtures.mi355x_probe_report("bad", gpus=8, gpu3={"ecc_uncorrectable": 2,
                                                            "ecc_blocks": {"umc": {"ce": 0, "ue": 2, "de": 0}},
                                                            "fw": dict(fixtures.MI355X_FW, pm=0x04560000)})
    good = fixtures.mi355x_probe_report("good", gpus=8)
    nodes = [fixtures.realistic_node("good", index=0, annotations=fixtures.health_annotation(good, "gzip"),
                                     extra_conditions=[fixtures.health_condition(good, 8)]),
             fixtures.realistic_node("bad", index=1, annotations=fixtures.health_annotation(bad),
                                     extra_conditions=[fixtures.health_condition(bad, 8)]),
             fixtures.realistic_node("plain", index=2),
             fixtures.realistic_node("cpu", gpu_key=None, index=3)]
    return write_kubeconfig(str(tmp_path / "kc"), mock_cluster(nodes).url)


def test_explain_unhealthy_node(run_cli, mock_cluster, tmp_path):
    kc = _cluster(mock_cluster, tmp_path)
    p = run_cli(["--kubeconfig", kc, "--explain", "bad"])
    assert p.returncode == 3, p.stdout + p.stderr
    out = p.stdout
    assert out.startswith("node bad: Ready=True  GPUs 8 (amd.com/gpu:8)")
    assert "AMDGPUHealthy=False (MI355XUnhealthy" in out
    assert "MI355X verdict: unhealthy, 7/8 GPUs ok" in out
    assert "  reason: gpu3: 2 uncorrectable ECC errors (umc 2)" in out
    row3 = next(ln for ln in out.splitlines() if ln.startswith("  3 "))
    assert "0000:35:00.0" in row3 and "2/0" in row3 and row3.endswith("2 uncorrectable ECC errors (umc 2)")
    assert "  node: firmware differs across GPUs: pm: gpu0-2,4-7 " in out  # a node-level finding naming a GPU span is kept
    assert out.rstrip().endswith("=> counts as Ready: no")


def test_explain_healthy_plain_and_missing(run_cli, mock_cluster, tmp_path):
    kc = _cluster(mock_cluster, tmp_path)
    p = run_cli(["--kubeconfig", kc, "--explain", "good"])
    assert p.returncode == 0 and "MI355X verdict: healthy, 8/8 GPUs ok" in p.stdout
    assert "labels: amd.com/gpu.family=MI355X" in p.stdout  # the agent's --label-node labels, when present
    assert "report: probe fixture" in p.stdout and "driver 6.18.54" in p.stdout  # gzip annotation read
    rows = [ln for ln in p.stdout.splitlines() if ln.startswith("  ") and ln.split()[0].isdigit()]
    assert len(rows) == 8 and all(r.endswith("ok") for r in rows)
    p = run_cli(["--kubeconfig", kc, "--explain", "plain"])  # no agent: the reference's Ready rule
    assert p.returncode == 0 and "AMDGPUHealthy: not published" in p.stdout and "verdict: none" in p.stdout
    p = run_cli(["--kubeconfig", kc, "--explain", "plain", "--mi355x"])  # the probe is required there
    assert p.returncode == 3 and "verdict: unknown" in p.stdout
    p = run_cli(["--kubeconfig", kc, "--explain", "cpu"])
    assert p.returncode == 2 and "not a GPU node" in p.stdout
    p = run_cli(["--kubeconfig", str(tmp_path / "missing"), "--explain", "x", "--json"])
    assert p.returncode == 1 and "error" in json.loads(p.stdout)
    assert H.HEALTH_CONDITION == "AMDGPUHealthy"


def test_explain_json(run_cli, mock_cluster, tmp_path):
    kc = _cluster(mock_cluster, tmp_path)
    p = run_cli(["--kubeconfig", kc, "--explain", "bad", "--json"])
    assert p.returncode == 3
    d = json.loads(p.stdout)
    assert d["node"] == "bad" and d["gpu_node"] and not d["counts_as_ready"] and d["gpus"] == 8
    assert d["verdict"]["state"] == "unhealthy" and d["health_condition"]["status"] == "False"
    g3 = d["report"]["gpus"][3]
    assert g3["bdf"] == "0000:35:00.0" and g3["ecc_uncorrectable"] == 2
    assert g3["findings"][0] == "2 uncorrectable ECC errors (umc 2)"
    assert d["report"]["node_findings"][0].startswith("firmware differs across GPUs: pm: gpu0-2,4-7 ")
    p = run_cli(["--kubeconfig", kc, "--explain", "cpu", "--json"])
    assert p.returncode == 2 and json.loads(p.stdout)["gpu_node"] is False


def test_fleet_summary(run_cli, mock_cluster, tmp_path):
    kc = _cluster(mock_cluster, tmp_path)
    p = run_cli(["--kubeconfig", kc, "--fleet"])
    assert p.returncode == 0, p.stderr  # good and plain count as Ready
    lines = p.stdout.splitlines()
    assert lines[0] == "GPU nodes: 3, counting as Ready: 2"
    assert lines[1] == "MI355X verdicts: 1 healthy, 1 unhealthy; 1 without a verdict"
    assert lines[2] == "  bad: unhealthy (not Ready)  gpu3: 2 uncorrectable ECC errors (umc 2)"
    assert "versions across 2 reporting nodes (mixed: pm):" in p.stdout
    assert "  driver: 6.18.54 x2" in p.stdout and "  pm: 04.86.00.00 x1, 04.86.15.106 x2" in lines


def test_fleet_summary_json(run_cli, mock_cluster, tmp_path):
    kc = _cluster(mock_cluster, tmp_path)
    p = run_cli(["--kubeconfig", kc, "--fleet", "--json"])
    d = json.loads(p.stdout)
    assert p.returncode == 0 and d["total_nodes"] == 3 and d["ready_nodes"] == 2
    assert d["verdicts"] == {"healthy": 1, "unhealthy": 1} and d["without_verdict"] == 1
    assert [a["name"] for a in d["attention"]] == ["bad"] and d["attention"][0]["reasons"][0].startswith("gpu3:")
    assert d["fleet"]["mixed"] == ["pm"]
