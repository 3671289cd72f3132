"""Firmware consistency, per-block ECC and the xGMI error status (probe fields beyond SURVEY §7.1).

The reference sees none of this (``check-gpu-node.py:172-196`` reads Ready and capacity only); these
are the fleet failure modes an MI355X node has besides a dead GPU: a half-applied firmware update,
HBM errors attributed to the memory controller vs the xGMI PHYs, a link that retried traffic.
"""
import json

from k8s_gpu_node_checker_amd.checker import CheckOptions, fleet_versions, run_check
from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
from k8s_gpu_node_checker_amd.models import health as H
from k8s_gpu_node_checker_amd.models.node import NodeExtras
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig


def rep(**kw):
    return fixtures.mi355x_probe_report("n", gpus=8, **kw)


def test_fixture_with_firmware_is_healthy():
    v = H.evaluate_report(rep(), 8)
    assert v.state == H.HEALTHY and not v.warnings, v.to_dict()


def test_uncorrectable_ecc_names_the_blocks():
    blocks = {"umc": {"ce": 4, "ue": 3, "de": 0}, "xgmi_wafl": {"ce": 0, "ue": 1, "de": 0}}
    v = H.evaluate_report(rep(gpu5={"ecc_uncorrectable": 4, "ecc_correctable": 4, "ecc_blocks": blocks}), 8)
    assert v.state == H.UNHEALTHY
    assert v.reasons == ["gpu5: 4 uncorrectable ECC errors (umc 3, xgmi_wafl 1)"]
    # the same totals from an agent without the per-block read keep the plain message
    v = H.evaluate_report(rep(gpu5={"ecc_uncorrectable": 4}), 8)
    assert v.reasons == ["gpu5: 4 uncorrectable ECC errors"]


def test_correctable_and_deferred_warnings_name_the_blocks():
    blocks = {"xgmi_wafl": {"ce": 5000, "ue": 0, "de": 0}, "umc": {"ce": 1, "ue": 0, "de": 2}}
    v = H.evaluate_report(rep(gpu1={"ecc_correctable": 5001, "ecc_deferred": 2, "ecc_blocks": blocks}), 8)
    assert v.state == H.DEGRADED
    assert "gpu1: 2 deferred ECC errors (umc 2)" in v.warnings
    assert "gpu1: 5001 correctable ECC errors (xgmi_wafl 5000, umc 1)" in v.warnings


def test_xgmi_error_status_degrades_unless_links_are_not_checked():
    v = H.evaluate_report(rep(gpu2={"xgmi_error": 2}, gpu6={"xgmi_error": 1}), 8)
    assert v.state == H.DEGRADED and v.ok
    assert v.warnings == ["gpu2: xGMI error status multiple errors", "gpu6: xGMI error status errors"]
    assert H.evaluate_report(rep(gpu2={"xgmi_error": 0}), 8).state == H.HEALTHY
    # a single-GPU box / --xgmi-links 0: no hive, the status is not judged
    one = fixtures.mi355x_probe_report("n", gpus=1, gpu0={"xgmi_error": 1, "xgmi": "XXXXXXXX"})
    assert H.evaluate_report(one, 1, H.HealthExpectations(xgmi_links=0)).state == H.HEALTHY


def test_firmware_versions_print_as_amd_smi_does():
    # amd-smi firmware on the MI355X box (gpurun_out/fw_list.txt): the same images, formatted
    got = {k: H.fw_version_str(k, v) for k, v in fixtures.MI355X_FW.items()}
    assert got == {"mec": "44", "rlc": "43", "sdma": "14", "psp_sos": "00.45.00.2F", "ta_ras": "1B.45.00.0A",
                   "ta_xgmi": "20.00.00.14", "pm": "04.86.15.106", "pldm_bundle": "01.25.17.07"}


def test_firmware_mismatch_across_gpus():
    fw7 = dict(fixtures.MI355X_FW, psp_sos=4521984)
    v = H.evaluate_report(rep(gpu7={"fw": fw7}), 8)
    assert v.state == H.DEGRADED and v.gpus_ok == 8
    assert v.warnings == ["firmware differs across GPUs: psp_sos: gpu0-6 00.45.00.2F, gpu7 00.45.00.00"]
    # two images differ, groups are ordered by size, non-contiguous GPUs are listed
    fw = dict(fixtures.MI355X_FW, mec=45, rlc=40)
    v = H.evaluate_report(rep(gpu1={"fw": fw}, gpu4={"fw": fw}), 8)
    assert v.warnings == ["firmware differs across GPUs: mec: gpu0,2-3,5-7 44, gpu1,4 45; "
                          "rlc: gpu0,2-3,5-7 43, gpu1,4 40"]
    # the message is what the condition carries: stable between probes (no counters, no timestamps)
    c1 = H.condition_for(v, now=1.0)["message"]
    c2 = H.condition_for(H.evaluate_report(rep(gpu1={"fw": fw}, gpu4={"fw": fw}), 8), now=2.0)["message"]
    assert c1 == c2 and c1.startswith("8/8 MI355X GPUs ok; firmware differs")
    # a GPU whose firmware could not be read is not a mismatch
    assert H.firmware_mismatch([{"index": 0, "fw": {"mec": 1}}, {"index": 1}]) == []


def _extras(reports):
    return [NodeExtras(True, {}, {}, False, json.dumps(r) if r is not None else None) for r in reports]


def test_fleet_versions_counts_drivers_and_firmware():
    a = rep()
    b = rep(driver={"name": "amdgpu", "version": "6.18.60"})
    c = rep(gpu3={"fw": dict(fixtures.MI355X_FW, mec=46)})
    f = fleet_versions(_extras([a, b, c, None, {"schema": H.SCHEMA, "error": "AMDSMI_STATUS_NO_PERM"}]))
    assert f["nodes_reporting"] == 3
    assert f["driver"] == {"6.18.54": 2, "6.18.60": 1}
    assert f["firmware"]["mec"] == {"44": 3, "46": 1}  # node c runs both
    assert f["firmware"]["psp_sos"] == {"00.45.00.2F": 3} and f["firmware"]["pm"] == {"04.86.15.106": 3}
    assert f["mixed"] == ["driver", "mec"]
    assert fleet_versions(_extras([None])) is None


def test_extended_json_carries_the_fleet_summary(mock_cluster, tmp_path):
    nodes = [fixtures.realistic_node(f"n{i}", index=i, annotations=fixtures.health_annotation(
        fixtures.mi355x_probe_report(f"n{i}", driver={"name": "amdgpu", "version": "6.18.54" if i else "6.18.50"})))
        for i in range(3)]
    srv = mock_cluster(nodes)
    res = run_check(ClusterConnection(srv.url), CheckOptions(json_extended=True))
    fleet = res.extended_fields()["mi355x"]["fleet"]
    assert fleet["driver"] == {"6.18.50": 1, "6.18.54": 2} and fleet["mixed"] == ["driver"]
    assert res.exit_code == 0  # a version drift is reported, it does not gate Ready


def test_cli_extended_fleet(run_cli, mock_cluster, tmp_path):
    nodes = [fixtures.realistic_node("a", annotations=fixtures.health_annotation(rep()))]
    kc = write_kubeconfig(str(tmp_path / "kc"), mock_cluster(nodes).url)
    p = run_cli(["--kubeconfig", kc, "--json-extended"])
    assert p.returncode == 0, p.stderr
    fleet = json.loads(p.stdout)["mi355x"]["fleet"]
    assert fleet["nodes_reporting"] == 1 and fleet["mixed"] == [] and fleet["firmware"]["ta_xgmi"] == {"20.00.00.14": 1}


def test_agent_metrics_expose_firmware_driver_and_ras_blocks():
    from prometheus_client.parser import text_string_to_metric_families

    from k8s_gpu_node_checker_amd.agent.agent import _metrics
    r = fixtures.mi355x_probe_report("n", gpus=2, driver={"name": "amdgpu", "version": '6.1 "v"\\1'},
                                     gpu1={"xgmi_error": 2, "ecc_blocks": {"umc": {"ce": 7, "ue": 1, "de": 0}}})
    fams = {f.name: f for f in text_string_to_metric_families(_metrics(r))}  # parses: the exposition is valid
    drv = fams["mi355x_node_driver_info"].samples[0]
    assert drv.labels["version"] == '6.1 "v"\\1' and drv.value == 1
    fw = {(s.labels["gpu"], s.labels["image"]): s.labels["version"] for s in fams["mi355x_gpu_firmware_info"].samples}
    assert fw[("1", "psp_sos")] == "00.45.00.2F" and fw[("0", "pm")] == "04.86.15.106"
    ecc = {(s.labels["block"], s.labels["kind"]): s.value for s in fams["mi355x_gpu_ecc_block_errors"].samples}
    assert ecc == {("umc", "ce"): 7, ("umc", "ue"): 1, ("umc", "de"): 0}
    assert [s.value for s in fams["mi355x_gpu_xgmi_error_status"].samples] == [2]
    r["gpus"][0]["cper"] = {"fatal": 0, "uncorrected": 1, "corrected": 9}
    fams = {f.name: f for f in text_string_to_metric_families(_metrics(r))}
    assert {s.labels["severity"]: s.value for s in fams["mi355x_gpu_cper_records"].samples} == {
        "fatal": 0, "uncorrected": 1, "corrected": 9}


def test_agent_metrics_group_each_family_once_on_a_multi_gpu_node():
    from prometheus_client.parser import text_string_to_metric_families

    from k8s_gpu_node_checker_amd.agent.agent import _metrics
    r = fixtures.mi355x_probe_report("n", gpus=8)
    r["gpus"][3]["diag"] = {"gemm": {"pass": True, "tflops": 1200.0}}
    names = [f.name for f in text_string_to_metric_families(_metrics(r))]
    assert len(names) == len(set(names)), sorted(n for n in names if names.count(n) > 1)
    fams = {f.name: f for f in text_string_to_metric_families(_metrics(r))}
    assert len(fams["mi355x_gpu_power_watts"].samples) == 8
    assert fams["mi355x_gpu_pcie_replays"].type == "counter"


def _bdf(i):
    return f"0000:{0x05 + 0x10 * i:02x}:00.0"


def test_full_board_topology_is_healthy():
    v = H.evaluate_report(rep(), 8)
    assert v.state == H.HEALTHY, v.to_dict()
    assert H.xgmi_topology(rep()["gpus"], 7) == []


def test_split_hive_is_unhealthy():
    other = {"xgmi_hive": "00000000000000aa"}
    v = H.evaluate_report(rep(gpu6=other, gpu7=other), 8)
    assert v.state == H.UNHEALTHY
    assert v.reasons == [f"GPUs span 2 xGMI hives: gpu0-5 {fixtures.MI355X_HIVE}, gpu6-7 00000000000000aa"]


def test_a_link_to_the_wrong_peer_is_unhealthy():
    peers3 = [_bdf(j) for j in range(8) if j not in (3, 6)] + [_bdf(5)]  # two links to gpu5, none to gpu6
    peers6 = [_bdf(j) for j in range(8) if j not in (6, 3)] + ["0000:ff:00.0"]  # its gpu3 link lands elsewhere
    v = H.evaluate_report(rep(gpu3={"xgmi_peers": peers3}, gpu6={"xgmi_peers": peers6}), 8)
    assert v.state == H.UNHEALTHY and v.gpus_ok == 8  # a node-level finding: no single GPU is at fault
    assert v.reasons == [f"gpu3: xGMI links reach 6 of the node's 7 other GPUs (no link to {_bdf(6)})",
                         f"gpu6: xGMI links reach 6 of the node's 7 other GPUs (no link to {_bdf(3)}), "
                         "1 to devices outside the node"]


def test_topology_needs_the_whole_unpartitioned_board():
    # one GPU missing: the count rule fires, the wiring is not judged from a partial view
    seven = fixtures.mi355x_probe_report("n", gpus=7)
    v = H.evaluate_report(seven, 8)
    assert v.reasons == ["7 of 8 GPUs visible to amd-smi"]
    # a single-GPU VM sees peers it cannot resolve (profiles: its 7 links reach other VMs' GPUs)
    one = fixtures.mi355x_probe_report("n", gpus=1, gpu0={"xgmi_peers": [_bdf(j) for j in range(1, 8)]})
    assert H.xgmi_topology(one["gpus"], 7) == []
    # CPX partitions report per-partition devices: not judged
    cpx = rep(**{f"gpu{i}": {"compute_partition": "CPX", "cus": 32, "xgmi_peers": []} for i in range(8)})
    assert H.xgmi_topology(cpx["gpus"], 7) == []
    # a VM whose guest PCI addresses differ from the host's: no link names a GPU it sees -> not judged
    host = {f"gpu{i}": {"xgmi_peers": [f"0001:{0x80 + j:02x}:00.0" for j in range(8) if j != i]} for i in range(8)}
    assert H.xgmi_topology(rep(**host)["gpus"], 7) == []
    # --xgmi-links 0 turns every fabric rule off
    assert H.xgmi_topology(rep(gpu3={"xgmi_peers": []})["gpus"], 0) == []


def test_link_trained_down_degrades():
    v = H.evaluate_report(rep(gpu4={"xgmi_speed_gbps": 25}), 8)
    assert v.state == H.DEGRADED and v.warnings == ["gpu4: xGMI links trained at x16 25 Gb/s (MI355X: x16 38 Gb/s)"]
    v = H.evaluate_report(rep(gpu4={"xgmi_width": 8}), 8)
    assert v.warnings == ["gpu4: xGMI links trained at x8 38 Gb/s (MI355X: x16 38 Gb/s)"]


def test_agent_metrics_xgmi_traffic_counters():
    from prometheus_client.parser import text_string_to_metric_families

    from k8s_gpu_node_checker_amd.agent.agent import _metrics, report_digest
    r = fixtures.mi355x_probe_report("n", gpus=2)
    r["gpus"][0]["xgmi_kb"] = [[1000, 2000]]
    fams = {f.name: f for f in text_string_to_metric_families(_metrics(r))}
    got = {(s.labels["peer"], s.labels["dir"]): s.value for s in fams["mi355x_gpu_xgmi_kilobytes"].samples}
    assert got == {(_bdf(1), "read"): 1000, (_bdf(1), "write"): 2000}
    # traffic moves every probe: it must not make the agent rewrite the annotation
    r2 = json.loads(json.dumps(r))
    r2["gpus"][0]["xgmi_kb"] = [[5000, 9000]]
    assert report_digest(r) == report_digest(r2)


def test_cper_fatal_record_recent_is_unhealthy_old_is_history():
    now = 1_800_000_000.0  # 2027-01-15T08:00:00Z
    recent = {"fatal": 1, "uncorrected": 0, "corrected": 4, "last_fatal": "2027-01-15T07:10:00Z",
              "last_corrected": "2027-01-15T07:00:00Z"}
    v = H.evaluate_report(rep(ts=now, gpu2={"cper": recent}), 8, now=now)
    assert v.state == H.UNHEALTHY and v.reasons == ["gpu2: fatal RAS error record (CPER) at 2027-01-15T07:10:00Z"]
    old = dict(recent, last_fatal="2027-01-10T07:10:00Z")
    v = H.evaluate_report(rep(ts=now, gpu2={"cper": old}), 8, now=now)
    assert v.state == H.DEGRADED
    assert v.warnings == ["gpu2: 1 fatal RAS error record(s) since driver load, last 2027-01-10T07:10:00Z"]
    # the window is a threshold like any other
    v = H.evaluate_report(rep(ts=now, gpu2={"cper": old}), 8, H.HealthExpectations(cper_window_s=7 * 86400), now=now)
    assert v.state == H.UNHEALTHY


def test_cper_uncorrected_recent_degrades_corrected_only_is_healthy():
    now = 1_800_000_000.0
    unc = {"fatal": 0, "uncorrected": 2, "corrected": 0, "last_uncorrected": "2027-01-15T06:00:00Z"}
    v = H.evaluate_report(rep(ts=now, gpu0={"cper": unc}), 8, now=now)
    assert v.state == H.DEGRADED and v.warnings == [
        "gpu0: uncorrected non-fatal RAS error record (CPER) at 2027-01-15T06:00:00Z"]
    ok = {"fatal": 0, "uncorrected": 0, "corrected": 12, "last_corrected": "2027-01-15T06:00:00Z"}
    assert H.evaluate_report(rep(ts=now, gpu0={"cper": ok}), 8, now=now).state == H.HEALTHY
    # a probe that could not read the records (non-root) is not judged on them
    assert H.evaluate_report(rep(ts=now, gpu0={"cper_error": "AMDSMI_STATUS_NO_PERM"}), 8, now=now).state == H.HEALTHY


def test_annotation_leaves_raw_counters_to_metrics():
    from k8s_gpu_node_checker_amd.agent.agent import Agent
    from k8s_gpu_node_checker_amd.models.node import HEALTH_ANNOTATION
    r = fixtures.mi355x_probe_report("n", gpus=2)
    r["gpus"][0].update(xgmi_kb=[[1, 2]], procs=[{"pid": 7, "vram_mb": 9}], probe_us=800)
    ann = json.loads(Agent("n").annotation(r)[HEALTH_ANNOTATION])
    assert not {"xgmi_kb", "throttle_acc", "procs", "probe_us"} & set(ann["gpus"][0])
    assert ann["gpus"][0]["fw"] == fixtures.MI355X_FW and ann["gpus"][0]["xgmi_peers"] == r["gpus"][0]["xgmi_peers"]
    assert "xgmi_kb" in r["gpus"][0]  # the live report (/probe) keeps them
    assert H.evaluate_report(ann, 2, H.HealthExpectations(xgmi_links=0)).state == H.HEALTHY


def test_partition_modes_differing_across_gpus_degrade():
    v = H.evaluate_report(rep(gpu7={"compute_partition": "CPX", "cus": 32}), 8)
    assert v.state == H.DEGRADED
    assert v.warnings == ["partition modes differ across GPUs: compute: gpu0-6 SPX, gpu7 CPX"]
    v = H.evaluate_report(rep(gpu2={"memory_partition": "NPS2", "vram_mb": 147448}), 8)
    assert v.warnings == ["partition modes differ across GPUs: memory: gpu0-1,3-7 NPS1, gpu2 NPS2"]
    # a board partitioned as a whole is one mode everywhere: nothing to report
    cpx = rep(**{f"gpu{i}": {"compute_partition": "CPX", "cus": 32} for i in range(8)})
    assert H.partition_mismatch(cpx["gpus"]) == []


def test_link_trained_down_with_only_one_field_reported():
    g = dict(rep()["gpus"][0])
    g.pop("xgmi_width")
    g["xgmi_speed_gbps"] = 19
    _, warns = H.evaluate_gpu(g, H.HealthExpectations())
    assert warns == ["gpu0: xGMI links trained at 19 Gb/s (MI355X: x16 38 Gb/s)"]


def test_driver_release_from_what_amd_smi_reports():
    assert H.driver_release("6.10.5") == "6.10.5"
    assert H.driver_release("Linuxversion6.18.54-ant.1(nixbld@localhost)(gcc(GCC)15.3.0)#1") == "6.18.54-ant.1"
    assert H.driver_release("") == "" and H.driver_release(None) == "" and H.driver_release("dev") == "dev"


def test_gzip_annotation_roundtrip_and_corruption():
    r = rep()
    for enc in ("json", "gzip"):
        raw = H.encode_annotation(r, enc)
        assert H.parse_annotation(raw) == json.loads(json.dumps(r))
    gz = H.encode_annotation(r, "gzip")
    assert gz.startswith("gz:") and len(gz) * 4 < len(H.encode_annotation(r, "json"))
    assert H.encode_annotation(r, "gzip") == gz  # deterministic: no gzip timestamp
    bad = H.parse_annotation("gz:!!notbase64")
    assert bad["error"] == "annotation is not gzip+base64 JSON"
    assert H.evaluate_report(bad, 8).state == H.UNKNOWN


def test_agent_gzip_annotation_read_by_the_checker(mock_cluster, tmp_path):
    from k8s_gpu_node_checker_amd.agent.agent import Agent
    from k8s_gpu_node_checker_amd.kube.client import KubeClient
    from k8s_gpu_node_checker_amd.models.node import HEALTH_ANNOTATION
    fx = tmp_path / "probe.json"
    fx.write_text(json.dumps(fixtures.mi355x_probe_report("n", gpus=7)))  # 7 of the node's 8 GPUs
    srv = mock_cluster([fixtures.realistic_node("n", gpu_count=8)])
    ag = Agent("n", source="fixture", fixture=str(fx), annotation_encoding="gzip", events=False)
    with KubeClient(ClusterConnection(srv.url)) as kc:
        ag.publish(kc, ag.probe_once())
        assert kc.get_node("n")["metadata"]["annotations"][HEALTH_ANNOTATION].startswith("gz:")
    for opts in (CheckOptions(json_extended=True), CheckOptions(json=True, health_reeval=True)):
        res = run_check(ClusterConnection(srv.url), opts)
        assert res.exit_code == 3 and res.verdicts[0].reasons[0] == "7 of 8 GPUs visible to amd-smi"
    fleet = run_check(ClusterConnection(srv.url), CheckOptions(json_extended=True)).extended_fields()["mi355x"]["fleet"]
    assert fleet["nodes_reporting"] == 1 and fleet["driver"] == {"6.18.54": 1}


def test_retired_pages_use_the_drivers_threshold_when_known():
    def v(**g0):
        rep = fixtures.mi355x_probe_report("n", gpus=1, gpu0=g0)
        return H.evaluate_report(rep, 1, H.HealthExpectations(xgmi_links=0), now=rep["ts"])
    # threshold known (root): the driver's line decides, the fixed 64-page limit does not apply
    assert v(bad_pages=100, bad_page_threshold=2048).state == H.DEGRADED
    assert v(bad_pages=100, bad_page_threshold=2048).warnings == ["gpu0: 100 retired pages"]
    assert v(bad_pages=1900, bad_page_threshold=2048).warnings == ["gpu0: 1900 retired pages, 2048 is the "
                                                                   "driver's threshold"]
    r = v(bad_pages=2048, bad_page_threshold=2048)
    assert r.state == H.UNHEALTHY and r.reasons == ["gpu0: 2048 retired pages reached the driver's threshold 2048"]
    # unknown threshold (non-root probe): the fixed limit
    assert v(bad_pages=65).reasons == ["gpu0: 65 retired pages > 64"]
    assert v(bad_pages=3, bad_pages_unreservable=1).state == H.UNHEALTHY
    assert v(bad_pages=3, bad_pages_pending=3).state == H.DEGRADED
    assert v(ras_eeprom="ok").state == H.HEALTHY
    assert v(ras_eeprom="corrupted").state == H.UNHEALTHY


def test_correctable_ecc_rate_over_the_agents_last_hour():
    from k8s_gpu_node_checker_amd.agent.agent import Agent
    ag = Agent("n", source="fixture")

    def probe(t, ce, bdf="0000:05:00.0"):
        rep = {"gpus": [{"index": 0, "bdf": bdf, "ecc_correctable": ce}]}
        ag._ce_rates(rep, now=t)
        return rep["gpus"][0].get("ecc_ce_per_h")
    assert probe(0, 0) is None
    assert probe(300, 10) is None  # the samples span less than 10 minutes
    assert probe(600, 20) == 120.0
    assert probe(4000, 20) == round(10 * 3600 / 3700, 1)  # baseline: the newest sample >= 1 h old (t=300)
    assert probe(4100, 5) is None  # the counter went down (driver reload): history restarts
    rep = fixtures.mi355x_probe_report("n", gpus=1, gpu0={"ecc_correctable": 140, "ecc_ce_per_h": 120.0,
                                                          "ecc_blocks": {"umc": {"ce": 140, "ue": 0, "de": 0}}})
    v = H.evaluate_report(rep, 1, H.HealthExpectations(xgmi_links=0), now=rep["ts"])
    assert v.state == H.DEGRADED and v.warnings == ["gpu0: correctable ECC errors rising at 120/h (umc 140)"]
    rep["gpus"][0]["ecc_ce_per_h"] = 12.0
    assert H.evaluate_report(rep, 1, H.HealthExpectations(xgmi_links=0), now=rep["ts"]).state == H.HEALTHY
