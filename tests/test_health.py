"""MI355X health model + Ready gate + CLI integration (SURVEY §5 failure detection, §7.1)."""
import json
import time

import pytest

from k8s_gpu_node_checker_amd.models import health as H
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig


def rep(**kw):
    return fixtures.mi355x_probe_report("n", gpus=8, **kw)


def test_measured_mi355x_report_is_healthy():
    v = H.evaluate_report(rep(), 8)
    assert v.state == H.HEALTHY and v.gpus_ok == 8 and v.ok
    assert v.short() == "MI355X 8/8 healthy"


@pytest.mark.parametrize("override,needle", [
    ({"gfx": "gfx942"}, "not gfx950"),
    ({"vram_type": 3}, "not HBM3E"),
    ({"vram_mb": 196000}, "VRAM"),
    ({"ecc_uncorrectable": 2}, "uncorrectable ECC"),
    ({"xgmi": "XUUUUUDU"}, "xGMI link(s) down"),
    ({"xgmi": "XUUUUUXX"}, "5/7 xGMI links up"),
    ({"kfd": False}, "no KFD node"),
    ({"cus": 240}, "240 CUs"),
    ({"bad_pages": 100}, "retired pages"),
    ({"error": "AMDSMI_STATUS_NO_PERM"}, "probe error"),
    ({"diag": {"gemm": {"pass": False, "detail": "120 TFLOP/s"}}}, "diag gemm failed"),
    ({"market_name": "AMD Radeon Graphics", "product_name": "Other", "vbios_name": "x", "device_id": "0x1234"},
     "not MI355X"),
])
def test_failures(override, needle):
    v = H.evaluate_report(rep(gpu3=override), 8)
    assert v.state == H.UNHEALTHY
    assert any(needle in r for r in v.reasons), v.reasons
    assert v.gpus_ok == 7


def test_identity_survives_generic_market_name():
    g = dict(rep()["gpus"][0], market_name="AMD Radeon Graphics")
    assert H.is_mi35x(g)
    g.update(product_name="", vbios_name="")
    assert H.is_mi35x(g)  # device id 0x75a3


@pytest.mark.parametrize("override,needle", [({"ecc_deferred": 1}, "deferred"), ({"ecc_correctable": 5000}, "correctable"),
                                            ({"bad_pages": 3}, "retired pages"), ({"hotspot_c": 104}, "hotspot"),
                                            ({"pcie_width": 8, "pcie_max_width": 16}, "PCIe link x8 of x16"),
                                            ({"pcie_replays": 20000}, "PCIe replays")])
def test_warnings_degrade_but_stay_ok(override, needle):
    v = H.evaluate_report(rep(gpu0=override), 8)
    assert v.state == H.DEGRADED and v.ok
    assert any(needle in w for w in v.warnings)


def test_partition_modes_scale_vram_expectation():
    nps2 = {f"gpu{i}": {"vram_mb": 147448, "memory_partition": "NPS2"} for i in range(8)}  # the whole board
    v = H.evaluate_report(rep(**nps2), 8)
    assert v.state == H.HEALTHY
    assert H.evaluate_report(rep(gpu0={"vram_mb": 147448}), 8).state == H.UNHEALTHY


def test_missing_gpus_vs_capacity():
    v = H.evaluate_report(fixtures.mi355x_probe_report("n", gpus=7), 8)
    assert v.state == H.UNHEALTHY and "7 of 8 GPUs visible" in v.reasons[-1]


def test_unknown_states():
    assert H.evaluate_report(None, 8).state == H.UNKNOWN
    assert H.evaluate_report(rep(ts=time.time() - 10000), 8).state == H.UNKNOWN
    assert H.evaluate_report(rep(error="AMDSMI_STATUS_DRIVER_NOT_LOADED"), 8).state == H.UNKNOWN
    assert H.evaluate_report({"schema": "other/v9"}, 8).state == H.UNKNOWN
    assert H.parse_annotation("{not json")["error"] == "annotation is not JSON"


def test_xgmi_check_can_be_disabled():
    exp = H.HealthExpectations(xgmi_links=0)
    assert H.evaluate_report(rep(gpu0={"xgmi": "XXXXXXXX"}), 8, exp).state == H.HEALTHY


def test_gate_policies():
    bad = H.Verdict(H.UNHEALTHY)
    unk = H.Verdict(H.UNKNOWN)
    good = H.Verdict(H.HEALTHY)
    assert H.gate_ready(True, bad, "off", True) is True
    assert H.gate_ready(True, bad, "auto", True) is False
    assert H.gate_ready(True, good, "auto", True) is True
    assert H.gate_ready(True, None, "auto", True) is True
    assert H.gate_ready(True, None, "require", True) is False
    assert H.gate_ready(True, unk, "auto", True, unknown_ok=True) is True
    assert H.gate_ready(True, unk, "auto", True, unknown_ok=False) is False
    assert H.gate_ready(False, good, "auto", True) is False
    assert H.gate_ready(True, bad, "require", False) is True  # non-AMD GPU nodes are not gated


def _cluster(mock_cluster, tmp_path, nodes):
    srv = mock_cluster(nodes)
    return write_kubeconfig(str(tmp_path / "kc"), srv.url)


def test_cli_without_annotations_is_reference_behaviour(run_cli, mock_cluster, tmp_path):
    kc = _cluster(mock_cluster, tmp_path, fixtures.cluster(3, "amd"))
    for policy in ("off", "auto"):
        p = run_cli(["--kubeconfig", kc, "--json", "--health-policy", policy])
        assert p.returncode == 0 and json.loads(p.stdout)["ready_nodes"] == 3


def test_cli_unhealthy_annotation_flips_ready_and_exit_code(run_cli, mock_cluster, tmp_path):
    bad = fixtures.mi355x_probe_report("mi355x-node-0000", gpus=8, gpu2={"ecc_uncorrectable": 7})
    nodes = [fixtures.realistic_node("mi355x-node-0000", annotations=fixtures.health_annotation(bad))]
    kc = _cluster(mock_cluster, tmp_path, nodes)
    p = run_cli(["--kubeconfig", kc, "--json"])
    assert p.returncode == 3
    doc = json.loads(p.stdout)
    assert doc["ready_nodes"] == 0 and doc["nodes"][0]["ready"] is False
    assert set(doc) == {"total_nodes", "ready_nodes", "nodes"}  # schema unchanged
    p = run_cli(["--kubeconfig", kc, "--json", "--health-policy", "off"])
    assert p.returncode == 0


def test_cli_require_policy_and_mi355x_preset(run_cli, mock_cluster, tmp_path):
    good = fixtures.mi355x_probe_report("a", gpus=8)
    nodes = [fixtures.realistic_node("a", annotations=fixtures.health_annotation(good), index=0),
             fixtures.realistic_node("b", index=1),  # no probe report
             fixtures.realistic_node("c", index=2, allocatable_gpus=0,
                                     annotations=fixtures.health_annotation(fixtures.mi355x_probe_report("c")))]
    kc = _cluster(mock_cluster, tmp_path, nodes)
    p = run_cli(["--kubeconfig", kc, "--json", "--health-policy", "require"])
    doc = json.loads(p.stdout)
    assert [n["ready"] for n in doc["nodes"]] == [True, False, True]
    p = run_cli(["--kubeconfig", kc, "--json-extended", "--mi355x"])  # allocatable-based + require
    doc = json.loads(p.stdout)
    # c's device plugin withdrew all 8 GPUs (allocatable 0): it stays a GPU node, Not Ready, with the reason
    assert [n["name"] for n in doc["nodes"]] == ["a", "b", "c"]
    assert [n["ready"] for n in doc["nodes"]] == [True, False, False]
    assert doc["nodes"][2]["gpus"] == 0 and doc["nodes"][2]["gpu_breakdown"] == {"amd.com/gpu": 0}
    h = doc["mi355x"]["nodes"][2]["health"]
    assert h["state"] == "unhealthy" and h["reasons"][0] == "device plugin allocates 0 of 8 amd.com/gpu"


def test_cli_health_in_slack_and_extended_json(run_cli, mock_cluster, sink, tmp_path):
    bad = fixtures.mi355x_probe_report("mi355x-node-0000", gpus=8, gpu0={"xgmi": "XUUUDUUU"})
    nodes = [fixtures.realistic_node("mi355x-node-0000", annotations=fixtures.health_annotation(bad))]
    kc = _cluster(mock_cluster, tmp_path, nodes)
    p = run_cli(["--kubeconfig", kc, "--json-extended", "--slack-webhook", sink.url("200")])
    doc = json.loads(p.stdout)
    h = doc["mi355x"]["nodes"][0]["health"]
    assert h["state"] == "unhealthy" and "xGMI" in h["reasons"][0]
    text = sink.payloads()[-1]["text"]
    assert "❌ Not Ready" in text and "[MI355X unhealthy: gpu0: 1 xGMI link(s) down (XUUUDUUU)]" in text


def test_condition_roundtrip():
    now = 1_800_000_000.0
    good = H.evaluate_report(rep(ts=now), 8, now=now)
    c = H.condition_for(good, now=now)
    assert c["type"] == "AMDGPUHealthy" and c["status"] == "True" and c["reason"] == "MI355XHealthy"
    assert c["lastHeartbeatTime"] == "2027-01-15T08:00:00Z" and H.parse_k8s_time(c["lastHeartbeatTime"]) == now
    v = H.verdict_from_condition((c["status"], c["reason"], c["message"], now), 900, now + 10)
    assert v.state == H.HEALTHY and v.ok
    bad = H.evaluate_report(rep(ts=now, gpu1={"ecc_uncorrectable": 1}), 8, now=now)
    c2 = H.condition_for(bad, now=now + 60, previous=c)
    assert c2["status"] == "False" and c2["lastTransitionTime"] == "2027-01-15T08:01:00Z"
    v = H.verdict_from_condition((c2["status"], c2["reason"], c2["message"], now + 60), 900, now + 70)
    assert v.state == H.UNHEALTHY and "uncorrectable" in v.reasons[0]
    c3 = H.condition_for(good, now=now + 120, previous=H.condition_for(good, now=now))
    assert c3["lastTransitionTime"] == c["lastTransitionTime"]  # unchanged status keeps the transition
    deg = H.evaluate_report(rep(ts=now, gpu0={"ecc_deferred": 2}), 8, now=now)
    v = H.verdict_from_condition(tuple(H.condition_for(deg, now=now)[k] for k in ("status", "reason", "message")) + (now,),
                                 900, now)
    assert v.state == H.DEGRADED and v.ok
    assert H.verdict_from_condition(("True", "MI355XHealthy", "", now - 5000), 900, now).state == H.UNKNOWN
    # a heartbeat from further in the future than the max age (an agent clock ahead by hours) is not fresh
    fut = H.verdict_from_condition(("True", "MI355XHealthy", "", now + 5000), 900, now)
    assert fut.state == H.UNKNOWN and "in the future" in fut.reasons[0]
    assert H.verdict_from_condition(("True", "MI355XHealthy", "", now + 60), 900, now).state == H.HEALTHY
    assert H.verdict_from_condition(("Unknown", "MI355XProbeFailed", "no driver", now), 900, now).state == H.UNKNOWN


def test_cli_condition_path_and_reeval(run_cli, mock_cluster, tmp_path):
    # condition says healthy, but the report fails a stricter --xgmi-links 8: non-default checker
    # thresholds re-evaluate the annotation by themselves (the condition cannot honour them)
    rep8 = fixtures.mi355x_probe_report("a", gpus=8)
    cond = fixtures.health_condition(rep8, 8)
    nodes = [fixtures.realistic_node("a", annotations=fixtures.health_annotation(rep8), extra_conditions=[cond])]
    kc = _cluster(mock_cluster, tmp_path, nodes)
    p = run_cli(["--kubeconfig", kc, "--json"])
    assert p.returncode == 0 and p.stderr == ""  # condition path: the agent's verdict
    p = run_cli(["--kubeconfig", kc, "--json", "--xgmi-links", "8"])
    assert p.returncode == 3 and p.stderr == ""
    p = run_cli(["--kubeconfig", kc, "--json", "--xgmi-links", "8", "--health-reeval"])
    assert p.returncode == 3  # re-evaluated with the checker's thresholds


def test_cli_custom_thresholds_without_annotation_warn(run_cli, mock_cluster, tmp_path):
    rep8 = fixtures.mi355x_probe_report("a", gpus=8)
    nodes = [fixtures.realistic_node("a", extra_conditions=[fixtures.health_condition(rep8, 8)])]
    kc = _cluster(mock_cluster, tmp_path, nodes)
    p = run_cli(["--kubeconfig", kc, "--json", "--xgmi-links", "8"])
    assert p.returncode == 0 and json.loads(p.stdout)["ready_nodes"] == 1
    assert "--xgmi-links 8" in p.stderr and "not applied" in p.stderr and "a" in p.stderr


def _seven_of_eight_cluster(mock_cluster, tmp_path, with_annotation=True):
    """VERDICT r1 scenario: amd.com/gpu capacity 8, amd-smi on the node sees 7, and the agent (which
    did not know the node's count) published AMDGPUHealthy=True for its 7 healthy GPUs."""
    rep7 = fixtures.mi355x_probe_report("n7", gpus=7)
    cond = fixtures.health_condition(rep7, 0)
    assert cond["status"] == "True" and cond["message"] == "7/7 MI355X GPUs healthy"
    ann = fixtures.health_annotation(rep7) if with_annotation else None
    nodes = [fixtures.realistic_node("n7", gpu_count=8, annotations=ann, extra_conditions=[cond])]
    return _cluster(mock_cluster, tmp_path, nodes)


@pytest.mark.parametrize("flags", [[], ["--mi355x"], ["--health-reeval"], ["--health-policy", "require"]])
def test_cli_missing_gpu_is_not_ready_on_every_path(run_cli, mock_cluster, tmp_path, flags):
    kc = _seven_of_eight_cluster(mock_cluster, tmp_path)
    p = run_cli(["--kubeconfig", kc, "--json"] + flags)
    assert p.returncode == 3, (flags, p.stdout, p.stderr)
    assert json.loads(p.stdout)["nodes"][0]["ready"] is False


def test_cli_missing_gpu_condition_only_extended_json(run_cli, mock_cluster, tmp_path):
    kc = _seven_of_eight_cluster(mock_cluster, tmp_path, with_annotation=False)
    p = run_cli(["--kubeconfig", kc, "--json-extended"])
    assert p.returncode == 3
    h = json.loads(p.stdout)["mi355x"]["nodes"][0]["health"]
    assert h["state"] == "unhealthy" and h["gpus_seen"] == 7 and h["gpus_ok"] == 7
    assert h["reasons"][0] == "7 of 8 GPUs visible to amd-smi"


def test_condition_message_counts_roundtrip():
    now = 1_800_000_000.0
    for r, exp_state in ((rep(ts=now), H.HEALTHY), (rep(ts=now, gpu0={"ecc_deferred": 2}), H.DEGRADED),
                         (rep(ts=now, gpu5={"ecc_uncorrectable": 3}), H.UNHEALTHY)):
        v = H.evaluate_report(r, 8, now=now)
        c = H.condition_for(v, now=now)
        assert H.parse_condition_counts(c["message"]) == (v.gpus_ok, v.gpus_seen)
        back = H.verdict_from_condition((c["status"], c["reason"], c["message"], now), 900, now, expected_gpus=8)
        assert back.state == exp_state and (back.gpus_ok, back.gpus_seen) == (v.gpus_ok, v.gpus_seen)
        assert back.reasons == v.reasons or back.reasons == ["; ".join(v.reasons)]
    # an older agent's message carries no counts: nothing to cross-check, the verdict stands
    assert H.parse_condition_counts("gpu3: 2 uncorrectable ECC errors") is None
    v = H.verdict_from_condition(("True", "MI355XHealthy", "all good", now), 900, now, expected_gpus=8)
    assert v.state == H.HEALTHY
    # more GPUs seen than registered (device plugin lagging) is not a failure
    c = H.condition_for(H.evaluate_report(rep(ts=now), 0, now=now), now=now)
    assert H.verdict_from_condition((c["status"], c["reason"], c["message"], now), 900, now, 4).state == H.HEALTHY
    # probe failure: no counts in the message
    u = H.condition_for(H.evaluate_report(rep(ts=now, error="AMDSMI_STATUS_DRIVER_NOT_LOADED"), 8, now=now), now=now)
    assert u["message"] == "probe failed: AMDSMI_STATUS_DRIVER_NOT_LOADED"


def test_cli_unhealthy_condition_without_annotation(run_cli, mock_cluster, tmp_path):
    bad = H.condition_for(H.Verdict(H.UNHEALTHY, ["gpu3: 2 uncorrectable ECC errors"]))
    nodes = [fixtures.realistic_node("a", extra_conditions=[bad]), fixtures.realistic_node("b", index=1)]
    kc = _cluster(mock_cluster, tmp_path, nodes)
    p = run_cli(["--kubeconfig", kc, "--json"])
    assert [n["ready"] for n in json.loads(p.stdout)["nodes"]] == [False, True] and p.returncode == 0


def test_fabric_failure_makes_the_node_unhealthy():
    from k8s_gpu_node_checker_amd.models import health as H
    from k8s_gpu_node_checker_amd.testing import fixtures
    rep = fixtures.mi355x_probe_report("n", gpus=8)
    rep["fabric"] = {"p2p": {"pass": True, "median_gbps": 48.0, "min_gbps": 45.1, "detail": ""}}
    assert H.evaluate_report(rep, 8).state == H.HEALTHY
    rep["fabric"]["p2p"] = {"pass": False, "detail": "3->5 11.2 GB/s"}
    v = H.evaluate_report(rep, 8)
    assert v.state == H.UNHEALTHY and v.reasons == ["xGMI p2p failed (3->5 11.2 GB/s)"]


def test_p2p_matrix_flags_slow_corrupting_and_non_peer_pairs(monkeypatch):
    from k8s_gpu_node_checker_amd.ops import diag
    fake = {(0, 1): (50.0, 0, True), (1, 0): (49.0, 0, True), (0, 2): (51.0, 0, True),
            (2, 0): (12.0, 0, True), (1, 2): (50.5, 7, True), (2, 1): (48.0, 0, False)}

    def p2p_copy(a, b, mib=256, iters=5):
        g, e, p = fake[(a, b)]
        return {"src": a, "dst": b, "gbps": g, "errors": e, "peer": p}
    monkeypatch.setattr(diag, "p2p_copy", p2p_copy)

    def p2p_fan(src, dsts, mib=256, iters=5):  # every link of src at once: the pair rates again
        return {"src": src, "total_gbps": sum(fake[(src, d)][0] for d in dsts),
                "to": [{"dst": d, "gbps": fake[(src, d)][0], "errors": 0, "peer": True} for d in dsts]}
    monkeypatch.setattr(diag, "p2p_fan", p2p_fan)
    m = diag.p2p_matrix([0, 1, 2])
    assert not m["pass"] and len(m["pairs"]) == 6 and m["median_gbps"] == 50.0 and m["min_gbps"] == 12.0
    assert "2->0 12.0 GB/s" in m["detail"] and "1->2 7 bad words" in m["detail"] and "2->1 no peer access" in m["detail"]
    assert "fan 2->0 12.0 GB/s with every link of 2 busy" in m["detail"] and m["fan"]["sources"] == 3
    for k in list(fake):
        fake[k] = (50.0, 0, True)
    assert diag.p2p_matrix([0, 1, 2])["pass"]
    assert diag.p2p_matrix([0])["skipped"] and diag.p2p_matrix([0])["pass"]


def test_pcie_full_width_and_idle_speed_are_healthy():
    # the link may idle at a lower speed (power management); only a narrower width is a finding
    v = H.evaluate_report(rep(gpu0={"pcie_width": 16, "pcie_max_width": 16, "pcie_speed_mts": 2500,
                                    "pcie_max_speed_mts": 32000, "pcie_replays": 3}), 8)
    assert v.state == H.HEALTHY, v.warnings


@pytest.mark.parametrize("override,needle", [
    ({"hbm_temp_c": 97}, "HBM 97 C"),
    ({"power_cap_w": 1000, "power_cap_default_w": 1400}, "power cap 1000 W of 1400 W default"),
    ({"throttle": {"s": 60.0, "thermal_pct": 25.0, "power_pct": 0.0, "prochot_pct": 0.0}}, "thermally throttled"),
    ({"throttle": {"s": 60.0, "thermal_pct": 0.0, "power_pct": 0.0, "prochot_pct": 3.0}}, "PROCHOT"),
])
def test_telemetry_warnings(override, needle):
    v = H.evaluate_report(rep(gpu2=override), 8)
    assert v.state == H.DEGRADED and v.ok
    assert any(needle in w for w in v.warnings), v.warnings


def test_power_throttling_alone_is_the_normal_operating_point():
    # package-power tracking under MFMA load is how an MI355X runs (profiles/telemetry_mi355x.json: 6.5 %
    # of a level-2 diagnostic burst); it is reported, never a warning
    v = H.evaluate_report(rep(gpu0={"throttle": {"s": 60.0, "thermal_pct": 0.0, "power_pct": 80.0,
                                                 "prochot_pct": 0.0}}), 8)
    assert v.state == H.HEALTHY


def test_throttle_window_from_accumulators():
    a = {"n": 1000, "prochot": 0, "ppt": 50, "socket_thm": 10, "vr_thm": 30, "hbm_thm": 0}
    b = {"n": 2000, "prochot": 5, "ppt": 350, "socket_thm": 60, "vr_thm": 230, "hbm_thm": 0}
    w = H.throttle_window(a, b, 12.34)
    assert w == {"s": 12.3, "thermal_pct": 20.0, "power_pct": 30.0, "prochot_pct": 0.5}
    assert H.throttle_window(None, b, 1.0) is None
    assert H.throttle_window(b, a, 1.0) is None            # counter went backwards: driver reload
    assert H.throttle_window(a, dict(b, ppt=10), 1.0).get("power_pct") is None
    assert H.throttle_window({"n": 1}, {"n": 5}, 1.0) is None  # no residency fields at all


def test_condition_counts_parser_matches_its_regex():
    import re

    from hypothesis import given, settings
    from hypothesis import strategies as st
    rx = re.compile(r"^(\d+)/(\d+) MI355X GPUs (?:healthy|ok)\b")

    @settings(max_examples=500, deadline=None)
    @given(st.from_regex(r"[0-9٣x/ ]{0,4}/?[0-9 ]{0,3} MI355X GPUs (healthy|ok|okay|heal)[ _;!a-zé]{0,3}",
                         fullmatch=True) | st.text(max_size=30))
    def check(msg):
        m = rx.match(msg)
        assert H.parse_condition_counts(msg) == ((int(m.group(1)), int(m.group(2))) if m else None), msg
    check()


def test_allocatable_below_capacity_is_a_degraded_hint(run_cli, mock_cluster, tmp_path):
    """the device plugin withholding GPUs (allocatable < capacity) is a health hint: a node
    whose agent says healthy becomes degraded (still Ready), and the hint names the counts."""
    r8 = fixtures.mi355x_probe_report("a", gpus=8)
    nodes = [fixtures.realistic_node("a", index=0, allocatable_gpus=7, extra_conditions=[fixtures.health_condition(r8, 8)]),
             fixtures.realistic_node("b", index=1, extra_conditions=[fixtures.health_condition(r8, 8)])]
    kc = _cluster(mock_cluster, tmp_path, nodes)
    p = run_cli(["--kubeconfig", kc, "--json-extended"])
    assert p.returncode == 0, p.stderr
    doc = json.loads(p.stdout)
    assert [n["ready"] for n in doc["nodes"]] == [True, True]
    h = [n["health"] for n in doc["mi355x"]["nodes"]]
    assert h[0]["state"] == "degraded" and h[0]["warnings"] == ["device plugin allocates 7 of 8 amd.com/gpu"]
    assert h[1]["state"] == "healthy"
    # --mi355x counts allocatable GPUs: the node is still a GPU node with 7
    p = run_cli(["--kubeconfig", kc, "--json", "--mi355x"])
    assert json.loads(p.stdout)["nodes"][0]["gpus"] == 7


def test_partitions_are_judged_on_down_links_only():
    exp = H.HealthExpectations()  # 7 links per GPU
    for part in ("CPX", "DPX"):
        assert H.evaluate_report(rep(gpu0={"xgmi": "XXXXXXXX", "compute_partition": part}), 8, exp).state \
            != H.UNHEALTHY
        assert "xGMI link(s) down" in " ".join(
            H.evaluate_report(rep(gpu0={"xgmi": "XUUUDUUU", "compute_partition": part}), 8, exp).reasons)
    assert H.evaluate_report(rep(gpu0={"xgmi": "XXXXXXXX"}), 8, exp).state == H.UNHEALTHY  # SPX: all 7 must be Up


@pytest.mark.parametrize("mutate,needle", [
    (lambda r: r.update(gpus=5), "gpus is a JSON int"),
    (lambda r: r.update(gpus="abc"), "gpus is a JSON str"),
    (lambda r: r["gpus"][2].update(fw=[1, "a"], power_cap_w="x", throttle_acc={"n": "x"}), None),
    (lambda r: r.update(ts=float("nan")), "probe report has no timestamp"),
    (lambda r: r.update(ts=float("inf")), "probe report has no timestamp"),
    (lambda r: r.update(ts=time.time() + 3600), "in the future (clock skew?)"),
])
def test_a_malformed_report_is_unknown_not_an_exception(mutate, needle):
    """A report is untrusted JSON (an agent endpoint, an annotation): fields of the wrong type never raise out of
    the verdict, and a report dated further in the future than a report may be old does not count as fresh."""
    r = rep()
    mutate(r)
    v = H.evaluate_report(r, 8)
    if needle is None:
        assert v.state in (H.UNKNOWN, H.UNHEALTHY, H.DEGRADED, H.HEALTHY)
    else:
        assert v.state == H.UNKNOWN and any(needle in x for x in v.reasons), v.to_dict()
    assert H.evaluate_report([1, 2], 8).state == H.UNKNOWN
    assert H.report_gpus({"gpus": 5}) == [] and H.report_gpus(None) == []


def test_hostile_annotations_are_probe_errors_not_crashes_or_memory():
    """A report annotation nested deeper than the JSON parser's stack, or a gzip member that inflates past
    MAX_REPORT_BYTES (~1000x from a 256 KiB annotation), is a probe error (verdict unknown), bounded in time and
    memory; a report of two gzip members still parses."""
    import base64
    import gzip
    for raw in ("[" * 200000, '{"a":' * 100000):
        doc = H.parse_annotation(raw)
        assert doc["error"] == "annotation is not JSON"
        assert H.evaluate_report(doc, 8).state == H.UNKNOWN
    bomb = H.GZIP_PREFIX + base64.b64encode(gzip.compress(b" " * (64 << 20) + b"{}")).decode()
    assert len(bomb) < 256 << 10
    t = time.perf_counter()
    doc = H.parse_annotation(bomb)
    assert doc["error"] == f"annotation decompresses to more than {H.MAX_REPORT_BYTES} bytes"
    assert time.perf_counter() - t < 1.0
    multi = H.GZIP_PREFIX + base64.b64encode(gzip.compress(b" " * (8 << 20)) + gzip.compress(b"{}")).decode()
    assert "more than" in H.parse_annotation(multi)["error"]
    two = H.GZIP_PREFIX + base64.b64encode(gzip.compress(b'{"a":') + gzip.compress(b"1}")).decode()
    assert H.parse_annotation(two) == {"a": 1}


def test_cli_survives_a_deeply_nested_annotation(run_cli, mock_cluster, tmp_path):
    """One node's hostile annotation makes that node unknown -- not Ready under --mi355x -- and the check
    completes (exit 0: one GPU node is Ready) with the other node judged as usual."""
    good = fixtures.mi355x_probe_report("a", gpus=8)
    nodes = [fixtures.realistic_node("a", annotations=fixtures.health_annotation(good), index=0),
             fixtures.realistic_node("b", index=1, annotations={fixtures.HEALTH_ANNOTATION: "[" * 100000})]
    kc = _cluster(mock_cluster, tmp_path, nodes)
    p = run_cli(["--kubeconfig", kc, "--json", "--mi355x"])
    assert p.returncode == 0, p.stderr
    doc = json.loads(p.stdout)
    assert [n["ready"] for n in doc["nodes"]] == [True, False] and doc["ready_nodes"] == 1


@pytest.mark.parametrize("args", [["--json-extended", "--mi355x"], ["--health-reeval", "--json-extended"],
                                  ["--fleet", "--json"], ["--explain", "b", "--json"], ["--explain", "c"]])
def test_every_report_path_survives_hostile_annotations(run_cli, mock_cluster, tmp_path, args):
    """Deep nesting, a wrong-typed ``gpus`` and a JSON array as the annotation: every report-reading path of the
    CLI (health gate, re-evaluation, --fleet, --explain) completes without a traceback."""
    bad_types = fixtures.mi355x_probe_report("c", gpus=8)
    bad_types["gpus"] = 5
    nodes = [fixtures.realistic_node("a", index=0,
                                     annotations=fixtures.health_annotation(fixtures.mi355x_probe_report("a", gpus=8))),
             fixtures.realistic_node("b", index=1, annotations={fixtures.HEALTH_ANNOTATION: "[" * 100000}),
             fixtures.realistic_node("c", index=2, annotations={fixtures.HEALTH_ANNOTATION: json.dumps(bad_types)}),
             fixtures.realistic_node("d", index=3, annotations={fixtures.HEALTH_ANNOTATION: "[1, 2]"})]
    kc = _cluster(mock_cluster, tmp_path, nodes)
    p = run_cli(["--kubeconfig", kc] + args)
    assert "Traceback" not in p.stderr and p.returncode in (0, 3), p.stderr[-2000:]
