"""Agent diagnostics schedule on CPU: idle-only active diagnostics (``--diag-when``), per-GPU intervals,
the node-level fabric test waiting for an all-idle node.  A fake ``ops.diag`` stands in for the HIP
library; the probe report is built here."""
import time

import pytest

from k8s_gpu_node_checker_amd.agent import agent as A
from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag, fabric
from k8s_gpu_node_checker_amd.testing import fixtures


def gpu(i, procs=None, act=0, vram_used=300):
    g = dict(fixtures.mi355x_probe_report("n", gpus=i + 1)["gpus"][i])  # a healthy MI355X
    g.update({"index": i, "bdf": f"0000:0{i}:00.0", "vram_used_mb": vram_used, "gfx_activity": act})
    g.pop("processes", None)
    if procs is not None:
        g["procs"] = procs
        g["processes"] = len(procs)
    return g


class World:
    def __init__(self, monkeypatch, n=2):
        self.gpus = [gpu(i, procs=[]) for i in range(n)]
        self.runs = []
        self.fabric_runs = 0
        self.clock = 1000.0
        monkeypatch.setattr(A.time, "time", lambda: self.clock)
        monkeypatch.setattr(amdsmi_probe, "probe", lambda node, src, fx: {
            "schema": "mi355x-health/v1", "node": node, "ts": self.clock, "probe": "fake",
            "gpus": [dict(g) for g in self.gpus]})
        monkeypatch.setattr(diag, "device_count", lambda: n)
        monkeypatch.setattr(diag, "device_info", lambda d: {"bdf": f"0000:0{d}:00.0"})

        def run(level, d, memory_partition=None, **kw):
            self.runs.append(d)
            return {"gemm": {"pass": True, "tflops": 1200.0 + len(self.runs)}}
        monkeypatch.setattr(diag, "run", run)

        def p2p(devs, **kw):
            self.fabric_runs += 1
            return {"pass": True, "median_gbps": 50.0, "min_gbps": 48.0, "detail": "", "wall_s": 0.1}
        monkeypatch.setattr(diag, "p2p_matrix", p2p)
        monkeypatch.setattr(fabric, "collective_suite", lambda devs, **kw: {"pass": True, "best_busbw_gbps": 300.0,
                                                                      "best_busbw_by_op": {}, "detail": "",
                                                                      "wall_s": 0.2, "rccl": "2.27.7"})


def test_gpu_busy_rules():
    own = frozenset((42,))
    assert A.gpu_busy(gpu(0, procs=[])) is None
    assert A.gpu_busy(gpu(0, procs=[{"pid": 42, "vram_mb": 200000}]), own) is None  # the agent itself
    assert A.gpu_busy(gpu(0, procs=[{"pid": 7, "vram_mb": 300}])) is None  # a monitoring tool's context
    assert A.gpu_busy(gpu(0, procs=[{"pid": 7, "vram_mb": 180000}])) == "in use: pid 7 holds 180000 MB"
    assert A.gpu_busy(gpu(0, procs=[], act=55)) == "in use: graphics engine 55% busy"
    assert A.gpu_busy(gpu(0, procs=[], act=9)) is None
    # no per-process list: the device's VRAM in use decides
    assert A.gpu_busy(gpu(0, vram_used=250000)) == "in use: 250000 MB of VRAM allocated"
    assert A.gpu_busy(gpu(0, vram_used=250000), busy_vram_mb=300000) is None
    assert A.gpu_busy({}) is None  # nothing known: idle (the probe failed to say otherwise)


def test_busy_gpu_is_skipped_and_retried_at_next_probe(monkeypatch):
    w = World(monkeypatch)
    w.gpus[1]["procs"] = [{"pid": 999, "vram_mb": 150000}]
    ag = A.Agent("n", source="fake", diag_level=1, diag_interval=3600)
    rep = ag.probe_once()
    assert w.runs == [0]
    g0, g1 = rep["gpus"]
    assert g0["diag"]["gemm"]["pass"] and "diag_skipped" not in g0
    assert "diag" not in g1 and g1["diag_skipped"] == "in use: pid 999 holds 150000 MB"
    # still busy a minute later: GPU 0 is not due, GPU 1 is skipped again
    w.clock += 60
    rep = ag.probe_once()
    assert w.runs == [0] and rep["gpus"][1]["diag_skipped"] and rep["gpus"][0]["diag"]
    # the workload ends: GPU 1 runs at the next probe, not an interval later
    w.gpus[1]["procs"] = []
    w.clock += 60
    rep = ag.probe_once()
    assert w.runs == [0, 1] and "diag_skipped" not in rep["gpus"][1] and rep["gpus"][1]["diag"]


def test_busy_gpu_keeps_its_previous_result(monkeypatch):
    w = World(monkeypatch)
    ag = A.Agent("n", source="fake", diag_level=1, diag_interval=3600)
    first = ag.probe_once()["gpus"][1]["diag"]
    w.gpus[1]["gfx_activity"] = 97
    w.clock += 3600
    rep = ag.probe_once()
    assert w.runs == [0, 1, 0]
    assert rep["gpus"][1]["diag"] == first and rep["gpus"][1]["diag_skipped"] == "in use: graphics engine 97% busy"
    assert rep["gpus"][1]["diag_at"] == 1000.0 and rep["gpus"][0]["diag_at"] == 4600.0  # the kept result's age shows


def test_diag_when_always_ignores_workloads(monkeypatch):
    w = World(monkeypatch)
    w.gpus[0]["procs"] = [{"pid": 5, "vram_mb": 200000}]
    ag = A.Agent("n", source="fake", diag_level=1, diag_when="always")
    rep = ag.probe_once()
    assert sorted(w.runs) == [0, 1] and all("diag_skipped" not in g for g in rep["gpus"])
    with pytest.raises(ValueError):
        A.Agent("n", diag_when="sometimes")


def test_node_level_fabric_waits_for_an_idle_node(monkeypatch):
    w = World(monkeypatch)
    w.gpus[0]["gfx_activity"] = 80
    ag = A.Agent("n", source="fake", diag_level=2, diag_interval=3600)
    rep = ag.probe_once()
    assert w.fabric_runs == 0 and "fabric" not in rep
    w.gpus[0]["gfx_activity"] = 0
    w.clock += 60
    rep = ag.probe_once()
    assert w.fabric_runs == 1 and rep["fabric"]["p2p"]["pass"] and rep["fabric"]["rccl"]["pass"]
    w.clock += 60
    ag.probe_once()
    assert w.fabric_runs == 1  # not due again before the interval


def test_skip_reasons_do_not_rewrite_the_annotation():
    a = {"gpus": [{"index": 0, "diag_skipped": "in use: pid 1 holds 9000 MB", "procs": [{"pid": 1, "vram_mb": 9000}],
                   "gfx_activity": 40}]}
    b = {"gpus": [{"index": 0, "diag_skipped": "in use: pid 2 holds 9100 MB", "procs": [{"pid": 2, "vram_mb": 9100}],
                   "gfx_activity": 70}]}
    assert A.report_digest(a) == A.report_digest(b)


def test_agent_cli_flags():
    args = A.build_parser().parse_args(["--diag-when", "always", "--busy-vram-mb", "4096", "--busy-gfx-activity", "5"])
    assert (args.diag_when, args.busy_vram_mb, args.busy_gfx_activity) == ("always", 4096, 5)
    assert A.build_parser().parse_args([]).diag_when == "idle"


def test_metrics_show_activity_and_skips():
    rep = {"ts": 1, "gpus": [{"index": 0, "bdf": "b0", "gfx_activity": 40, "diag_skipped": "in use: x"},
                             {"index": 1, "bdf": "b1", "gfx_activity": 0, "diag": {"gemm": {"pass": True}}}]}
    m = A._metrics(rep)
    assert 'mi355x_gpu_gfx_activity_percent{gpu="0",bdf="b0"} 40' in m
    assert 'mi355x_gpu_diag_skipped{gpu="0",bdf="b0"} 1' in m and 'mi355x_gpu_diag_skipped{gpu="1",bdf="b1"} 0' in m


def test_hung_diagnostic_is_reported_not_waited_for(monkeypatch):
    import threading
    from k8s_gpu_node_checker_amd.models.health import HEALTHY, UNHEALTHY
    w = World(monkeypatch)
    release = threading.Event()
    started = []

    def run(level, d, memory_partition=None, **kw):
        started.append(d)
        if d == 1:
            release.wait(30)  # GPU 1's queue hangs
        return {"gemm": {"pass": True}}
    monkeypatch.setattr(diag, "run", run)
    ag = A.Agent("n", source="fake", diag_level=1, diag_interval=3600, diag_timeout=0.2)
    rep = ag.probe_once()
    g0, g1 = rep["gpus"]
    assert g0["diag"]["gemm"]["pass"]
    assert g1["diag"]["watchdog"]["pass"] is False and "GPU hang" in g1["diag"]["watchdog"]["detail"]
    assert rep["state"] == UNHEALTHY
    # an interval later: GPU 0 runs again, GPU 1 gets no second diagnostic while the first one lives
    w.clock += 3600
    t = time.monotonic()
    rep = ag.probe_once()
    assert started == [0, 1, 0] and time.monotonic() - t < 5
    assert rep["gpus"][1]["diag"]["watchdog"]["pass"] is False
    # the hang clears: its real result replaces the watchdog failure
    release.set()
    ag._diag_threads[1].job.thread.join(5)
    rep = ag.probe_once()
    assert rep["gpus"][1]["diag"] == {"gemm": {"pass": True}} and rep["state"] == HEALTHY


def test_restarted_agent_clears_a_watchdog_verdict(monkeypatch, mock_cluster):
    """The liveness probe restarts an agent whose diagnostic hung (its thread cannot be cancelled: /healthz
    fails once it has outlived 2 x --diag-timeout, test_healthz_fails_once_a_diagnostic_outlives_twice_its_watchdog).
    The new instance carries no cached watchdog failure: its first publish rewrites the condition, the
    annotation and the taint the old instance left on the node."""
    import threading
    from k8s_gpu_node_checker_amd.kube.client import KubeClient
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    from k8s_gpu_node_checker_amd.models import health as H
    from k8s_gpu_node_checker_amd.models.node import HEALTH_ANNOTATION
    World(monkeypatch)
    srv = mock_cluster([fixtures.realistic_node("n", gpu_count=2)])
    release = threading.Event()

    def hang(level, d, memory_partition=None, **kw):
        if d == 1:
            release.wait(30)
        return {"gemm": {"pass": True}}
    monkeypatch.setattr(diag, "run", hang)
    with KubeClient(ClusterConnection(srv.url)) as kc:
        old = A.Agent("n", source="fake", diag_level=1, diag_timeout=0.2, taint_unhealthy=True)
        old.publish(kc, old.probe_once())
        node = kc.get_node("n")
        cond = [c for c in node["status"]["conditions"] if c["type"] == H.HEALTH_CONDITION][0]
        assert cond["status"] == "False" and "watchdog" in cond["message"]
        assert any(t["key"] == H.UNHEALTHY_TAINT["key"] for t in node["spec"].get("taints") or [])
        release.set()  # the old process is gone; its hung thread with it

        monkeypatch.setattr(diag, "run", lambda level, d, memory_partition=None, **kw: {"gemm": {"pass": True}})
        new = A.Agent("n", source="fake", diag_level=1, taint_unhealthy=True)
        wrote = new.publish(kc, new.probe_once())
        assert wrote["annotation"] and wrote["condition"] and wrote["taint"]
        node = kc.get_node("n")
    cond = [c for c in node["status"]["conditions"] if c["type"] == H.HEALTH_CONDITION][0]
    assert cond["status"] == "True" and cond["message"] == "2/2 MI355X GPUs healthy"
    assert "watchdog" not in node["metadata"]["annotations"][HEALTH_ANNOTATION]
    assert not any(t["key"] == H.UNHEALTHY_TAINT["key"] for t in node["spec"].get("taints") or [])


def test_diagnostic_that_raises_is_a_failed_test(monkeypatch):
    World(monkeypatch)

    def boom(level, d, **kw):
        raise RuntimeError("hipErrorIllegalAddress")
    monkeypatch.setattr(diag, "run", boom)
    rep = A.Agent("n", source="fake", diag_level=1).probe_once()
    assert rep["gpus"][0]["diag"]["run"] == {"pass": False, "detail": "RuntimeError: hipErrorIllegalAddress"}


def test_healthz_turns_503_when_probes_stop(monkeypatch):
    import urllib.error
    import urllib.request
    w = World(monkeypatch)
    ag = A.Agent("n", source="fake")
    srv = A.serve(ag, "127.0.0.1", 0, stale_after=0.3)
    url = f"http://127.0.0.1:{srv.server_address[1]}/healthz"
    try:
        assert urllib.request.urlopen(url, timeout=5).read() == b"ok"  # starting up: grace period
        ag.probe_once()
        assert urllib.request.urlopen(url, timeout=5).status == 200
        time.sleep(0.5)  # the probe loop is stuck
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(url, timeout=5)
        assert e.value.code == 503
        e.value.close()
        ag.probe_once()
        assert urllib.request.urlopen(url, timeout=5).status == 200
    finally:
        srv.shutdown()
        srv.server_close()
    assert w.gpus


def test_hip_runtime_losing_its_devices_restarts_the_agent_not_the_verdict(monkeypatch):
    """After a driver reload under a running agent every HIP call fails: that is the process's runtime, not
    the GPU.  The agent records no failed diagnostic (the verdict stays healthy), starts no more of them,
    and /healthz answers 503 so the liveness probe restarts it."""
    import urllib.error
    import urllib.request
    w = World(monkeypatch)
    lost = "mi355x diag failed (-1): hipSetDevice(device): no ROCm-capable device is detected"
    monkeypatch.setattr(diag, "run", lambda level, d, memory_partition=None, **kw: (
        w.runs.append(d), {"gemm": {"pass": False, "detail": lost}, "hbm": {"pass": False, "detail": lost}})[1])
    ag = A.Agent("n", source="fake", diag_level=1, diag_interval=0.0)
    srv = A.serve(ag, "127.0.0.1", 0, stale_after=60)
    try:
        rep = ag.probe_once()
        assert rep["state"] == "healthy" and "diag" not in rep["gpus"][0]
        assert rep["gpus"][0]["diag_skipped"].startswith("HIP runtime lost its devices (mi355x diag failed")
        assert ag.hip_lost == lost and len(w.runs) == 2
        ag.probe_once()
        assert len(w.runs) == 2  # nothing new starts in this process
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(f"http://127.0.0.1:{srv.server_address[1]}/healthz", timeout=5)
        assert e.value.code == 503 and b"HIP runtime lost its devices" in e.value.read()
    finally:
        srv.shutdown()
        srv.server_close()
    # a GPU fault (illegal address) is still the GPU's failure
    assert A.runtime_lost({"gemm": {"pass": False, "detail": "hipMemcpy: an illegal memory access"}}) is None
    assert A.runtime_lost({"gemm": {"pass": False, "detail": lost}, "hbm": {"pass": True}}) is None


def test_a_hung_fabric_test_is_a_failure_not_a_frozen_agent(monkeypatch):
    import threading
    w = World(monkeypatch, n=2)
    release = threading.Event()

    def hang(devs, **kw):
        w.fabric_runs += 1
        release.wait(10)
        return {"pass": True, "best_busbw_gbps": 300.0, "best_busbw_by_op": {}, "detail": "", "wall_s": 9.0}
    monkeypatch.setattr(fabric, "collective_suite", hang)
    ag = A.Agent("n", source="fake", diag_level=2, diag_interval=0.0, diag_timeout=0.3)
    t0 = time.monotonic()
    rep = ag.probe_once()
    assert time.monotonic() - t0 < 3  # the probe came back
    assert rep["fabric"]["watchdog"]["pass"] is False and "fabric hang" in rep["fabric"]["watchdog"]["detail"]
    assert rep["state"] == "unhealthy"
    runs = w.fabric_runs  # the pair matrix and the hung collectives
    rep = ag.probe_once()  # still stuck: no second suite starts
    assert w.fabric_runs == runs and "watchdog" in rep["fabric"]
    release.set()
    time.sleep(0.2)
    rep = ag.probe_once()  # it finished: its real result replaces the watchdog failure
    assert rep["fabric"]["rccl"]["pass"] and rep["fabric"]["p2p"]["pass"]


def test_status_endpoint_is_the_verdict_in_text(monkeypatch):
    import urllib.request
    w = World(monkeypatch)
    w.gpus[1]["ecc_uncorrectable"] = 3
    ag = A.Agent("n", source="fake")
    srv = A.serve(ag, "127.0.0.1", 0)
    url = f"http://127.0.0.1:{srv.server_address[1]}/status"
    try:
        assert urllib.request.urlopen(url, timeout=5).read() == b"no probe yet\n"
        ag.probe_once()
        txt = urllib.request.urlopen(url, timeout=5).read().decode()
    finally:
        srv.shutdown()
        srv.server_close()
    lines = txt.splitlines()
    assert lines[0].startswith("node n: MI355X verdict unhealthy, 1/2 GPUs ok (probe fake")
    assert "  reason: gpu1: 3 uncorrectable ECC errors" in lines
    row1 = next(ln for ln in lines if ln.startswith("  1 "))
    assert "0000:01:00.0" in row1 and row1.endswith("3 uncorrectable ECC errors")


def test_no_hip_device_is_said_per_gpu(monkeypatch):
    World(monkeypatch)
    monkeypatch.setattr(diag, "device_count", lambda: 0)
    rep = A.Agent("n", source="fake", diag_level=1).probe_once()
    assert [g.get("diag_skipped") for g in rep["gpus"]] == \
        ["no HIP device visible to the agent (/dev/kfd and /dev/dri mounted?)"] * 2


def test_a_slow_result_is_measured_again_soon(monkeypatch):
    w = World(monkeypatch, n=1)
    results = [{"gemm": {"pass": True, "degraded": True, "detail": "tflops 1100 = 90% of 1220"}},
               {"gemm": {"pass": True, "degraded": False}}]
    monkeypatch.setattr(diag, "run", lambda level, d, memory_partition=None, **kw: (w.runs.append(d), results[len(w.runs) - 1])[1])
    ag = A.Agent("n", source="fake", diag_level=1, diag_interval=3600.0)
    rep = ag.probe_once()
    assert rep["gpus"][0]["diag"]["gemm"]["degraded"] and rep["state"] == "degraded"
    assert rep["gpus"][0]["diag_at"] == w.clock  # reported as when it ran, whatever the schedule says
    w.clock += 120
    ag.probe_once()
    assert len(w.runs) == 1  # not yet
    w.clock += A.DIAG_RECHECK_S
    rep = ag.probe_once()
    assert len(w.runs) == 2 and rep["state"] == "healthy"  # the one-off cleared in minutes, not an hour
    w.clock += A.DIAG_RECHECK_S * 2
    ag.probe_once()
    assert len(w.runs) == 2  # clean: back to the full interval


def test_healthz_fails_once_a_diagnostic_outlives_twice_its_watchdog(monkeypatch):
    """A per-GPU diagnostic stuck in a HIP call: the watchdog verdict goes out at 1 x --diag-timeout (the
    agent keeps probing and publishing), /healthz stays 200 until the thread has lived 2 x --diag-timeout,
    then answers 503 so the kubelet starts a fresh process.  It recovers to 200 if the call returns."""
    import threading
    import urllib.error
    import urllib.request
    w = World(monkeypatch)
    release = threading.Event()

    def run(level, d, memory_partition=None, **kw):
        if d == 0:
            release.wait(30)
        return {"gemm": {"pass": True}}
    monkeypatch.setattr(diag, "run", run)
    ag = A.Agent("n", source="fake", diag_level=1, diag_interval=3600, diag_timeout=0.4)
    srv = A.serve(ag, "127.0.0.1", 0, stale_after=60)
    url = f"http://127.0.0.1:{srv.server_address[1]}/healthz"
    try:
        t0 = time.monotonic()
        rep = ag.probe_once()  # returns after the 0.4 s watchdog with the verdict
        assert rep["gpus"][0]["diag"]["watchdog"]["pass"] is False and rep["state"] == "unhealthy"
        assert urllib.request.urlopen(url, timeout=5).status == 200  # 1x: published, not yet restarted
        while time.monotonic() - t0 < 0.85:
            time.sleep(0.05)
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(url, timeout=5)
        assert e.value.code == 503
        body = e.value.read().decode()
        assert body.startswith("gpu0 diagnostics running for") and "2 x --diag-timeout" in body
        assert w.gpus
        release.set()
        ag._diag_threads[0].job.thread.join(5)
        assert urllib.request.urlopen(url, timeout=5).status == 200
    finally:
        release.set()
        srv.shutdown()
        srv.server_close()


def test_healthz_fails_for_a_hung_fabric_suite(monkeypatch):
    import threading
    World(monkeypatch)
    release = threading.Event()

    def hang(devs, **kw):
        release.wait(30)
        return {"pass": True}
    monkeypatch.setattr(diag, "p2p_matrix", hang)  # the pair matrix hangs (and ignores its deadline)
    ag = A.Agent("n", source="fake", diag_level=2, diag_interval=3600, diag_timeout=0.2)
    try:
        rep = ag.probe_once()
        assert "watchdog" in rep["fabric"]
        assert ag.hung_diagnostic() is None
        time.sleep(0.25)
        assert ag.hung_diagnostic().startswith("node-level xGMI/RCCL tests running for")
    finally:
        release.set()


def test_per_gpu_diagnostics_wait_while_a_fabric_suite_is_hung(monkeypatch):
    """a timed-out collective still holds every GPU; the next interval's per-GPU tests must not
    start behind it."""
    import threading
    w = World(monkeypatch)
    release = threading.Event()

    def hang(devs, **kw):
        release.wait(30)
        return {"pass": True, "best_busbw_gbps": 300.0, "best_busbw_by_op": {}, "detail": "", "wall_s": 9.0}
    monkeypatch.setattr(fabric, "collective_suite", hang)
    ag = A.Agent("n", source="fake", diag_level=2, diag_interval=3600, diag_timeout=0.2)
    try:
        ag.probe_once()
        assert w.runs == [0, 1] or sorted(w.runs) == [0, 1]
        w.clock += 3600
        rep = ag.probe_once()
        assert sorted(w.runs) == [0, 1]  # nothing new started
        assert all(g["diag_skipped"].startswith("node-level xGMI/RCCL tests still running") for g in rep["gpus"])
        assert all(g["diag"] for g in rep["gpus"])  # the last results are kept
    finally:
        release.set()
    ag._fabric_thread.job.thread.join(5)
    w.clock += 1
    ag.probe_once()
    assert sorted(w.runs) == [0, 0, 1, 1]


def test_a_persistent_failure_is_rechecked_once_then_back_to_the_interval(monkeypatch):
    """a GPU that keeps failing the same way is not stressed again every 5 minutes."""
    w = World(monkeypatch, n=1)
    bad = {"memtest": {"pass": False, "detail": "12 bad words"}}
    monkeypatch.setattr(diag, "run", lambda level, d, memory_partition=None, **kw: (w.runs.append(d), dict(bad))[1])
    ag = A.Agent("n", source="fake", diag_level=1, diag_interval=3600.0)
    ag.probe_once()
    w.clock += A.DIAG_RECHECK_S
    ag.probe_once()
    assert len(w.runs) == 2  # the one recheck confirmed it
    w.clock += A.DIAG_RECHECK_S
    ag.probe_once()
    assert len(w.runs) == 2  # the same failure again: back to the full interval
    w.clock += 3600 - A.DIAG_RECHECK_S
    ag.probe_once()
    assert len(w.runs) == 3
    # a different result (another test fails) earns one recheck of its own
    bad = {"hbm": {"pass": False, "detail": "copy 3 TB/s"}}
    w.clock += 3600
    ag.probe_once()
    w.clock += A.DIAG_RECHECK_S
    ag.probe_once()
    assert len(w.runs) == 5


def test_allocations_matching_no_local_pci_address_skip_every_gpu(monkeypatch):
    """a device plugin that names partitions by another scheme -- the agent cannot tell which
    device a pod has, so it diagnoses none (fail safe) and says why."""
    w = World(monkeypatch)
    ag = A.Agent("n", source="fake", diag_level=1, pod_resources_socket="/nonexistent.sock")
    monkeypatch.setattr(ag, "_allocated", lambda: {"amdgpu_xcp_3": "ml/train-0"})
    rep = ag.probe_once()
    assert w.runs == []
    assert all(g["diag_skipped"].startswith("kubelet reports 1 allocated GPU device(s) (amdgpu_xcp_3) matching no "
                                            "local PCI address") for g in rep["gpus"])
    # matching addresses: only the allocated GPU is skipped
    monkeypatch.setattr(ag, "_allocated", lambda: {"0000:01:00.0": "ml/train-0"})
    w.clock += 3600
    rep = ag.probe_once()
    assert w.runs == [0] and rep["gpus"][1]["diag_skipped"] == "allocated to pod ml/train-0"


def test_bdf_fallback_is_normalised(monkeypatch):
    """HIP's domain-less, upper-case address still matches amd-smi's and the kubelet's."""
    w = World(monkeypatch)
    monkeypatch.setattr(diag, "device_info", lambda d: {"bdf": f"0{d}:00.0".upper()})
    for g in w.gpus:
        g["bdf"] = g["bdf"].upper()
    ag = A.Agent("n", source="fake", diag_level=1, pod_resources_socket="/x")
    monkeypatch.setattr(ag, "_allocated", lambda: {"0000:01:00.0": "ml/p"})
    rep = ag.probe_once()
    assert w.runs == [0] and rep["gpus"][1]["diag_skipped"] == "allocated to pod ml/p"


def test_configured_device_hip_does_not_have_is_a_configuration_error(monkeypatch):
    """a bad device index is said as such -- not run (it would fail with 'invalid device ordinal'),
    not mistaken for a lost HIP runtime (no /healthz restart loop)."""
    w = World(monkeypatch)
    ag = A.Agent("n", source="fake", diag_level=1, devices=[0, 5])
    rep = ag.probe_once()
    assert w.runs == [0] and ag.hip_lost is None
    assert ag._diag_skipped[5] == "device 5 is not a HIP device of the agent (2 visible): check --devices"


def test_one_gpu_failing_with_runtime_strings_is_that_gpus_failure(monkeypatch):
    """'invalid device ordinal' on one GPU while the other runs fine is not a lost runtime."""
    w = World(monkeypatch)
    lost = "mi355x diag failed (-1): hipSetDevice(device): invalid device ordinal"

    def run(level, d, memory_partition=None, **kw):
        w.runs.append(d)
        return {"gemm": {"pass": False, "detail": lost}} if d == 1 else {"gemm": {"pass": True}}
    monkeypatch.setattr(diag, "run", run)
    ag = A.Agent("n", source="fake", diag_level=1)
    rep = ag.probe_once()
    assert ag.hip_lost is None and rep["gpus"][1]["diag"]["gemm"]["pass"] is False and rep["state"] == "unhealthy"
    # the device count changed under the process: that is the runtime
    monkeypatch.setattr(diag, "device_count", lambda: 1)
    w.clock += A.DIAG_RECHECK_S
    rep = ag.probe_once()
    assert ag.hip_lost == "HIP device count changed from 2 to 1"
    assert all(g["diag_skipped"].startswith("HIP runtime lost its devices (HIP device count changed")
               for g in rep["gpus"][:1])
    # and when every device that ran failed that way together, also the runtime (no count change needed)
    ag2 = A.Agent("n", source="fake", diag_level=1)
    monkeypatch.setattr(diag, "device_count", lambda: 2)
    monkeypatch.setattr(diag, "run", lambda level, d, memory_partition=None, **kw: {"gemm": {"pass": False, "detail": lost}})
    ag2.probe_once()
    assert ag2.hip_lost == lost


def test_publish_refuses_a_foreign_node(monkeypatch, mock_cluster):
    """the agent writes only the node it was started for, whatever report or call reaches it."""
    from k8s_gpu_node_checker_amd.kube.client import KubeClient
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    World(monkeypatch)
    srv = mock_cluster([fixtures.realistic_node("n", gpu_count=2), fixtures.realistic_node("other", gpu_count=2)])
    with KubeClient(ClusterConnection(srv.url)) as kc:
        ag = A.Agent("n", source="fake")
        rep = ag.probe_once()
        assert ag.publish(kc, rep)["condition"]
        foreign = dict(rep, node="other")
        with pytest.raises(A.ForeignNodeError, match="report is for node 'other'"):
            ag.publish(kc, foreign)
        guard = A._OwnNodeClient(kc, "n")
        with pytest.raises(A.ForeignNodeError, match="refusing patch_node_condition on node 'other'"):
            guard.patch_node_condition("other", {"type": "AMDGPUHealthy", "status": "True"})
        with pytest.raises(A.ForeignNodeError, match="refusing an Event about Node 'other'"):
            guard.create_event("default", {"involvedObject": {"kind": "Node", "name": "other"}})
        other = kc.get_node("other")
    assert not any(c["type"] == "AMDGPUHealthy" for c in other["status"]["conditions"])


def test_token_node_claim_is_read_and_a_mismatch_stops_the_agent(monkeypatch, tmp_path):
    import base64
    import json as _json

    def jwt(claims):
        b = lambda d: base64.urlsafe_b64encode(_json.dumps(d).encode()).rstrip(b"=").decode()  # noqa: E731
        return f"{b({'alg': 'RS256'})}.{b(claims)}.sig"
    tok = jwt({"sub": "system:serviceaccount:gpu-health:mi355x-node-agent",
               "kubernetes.io": {"namespace": "gpu-health", "node": {"name": "gpu-7", "uid": "u"}}})
    assert A.token_node_name(tok) == "gpu-7"
    assert A.token_node_name(jwt({"sub": "x"})) is None and A.token_node_name("opaque") is None
    assert A.token_node_name(None) is None
    kc = tmp_path / "kc"
    (tmp_path / "token").write_text(tok)
    kc.write_text(f"""clusters:
- cluster: {{server: "http://127.0.0.1:1"}}
  name: c
contexts:
- context: {{cluster: c, user: u}}
  name: x
current-context: x
users:
- name: u
  user: {{tokenFile: {tmp_path / 'token'}}}
""")
    assert A.main(["--node", "gpu-3", "--kubeconfig", str(kc), "--once", "--source", "fixture",
                   "--fixture", "/nonexistent"]) == 2


def test_single_gpu_failing_with_runtime_strings_is_not_a_restart_loop(monkeypatch):
    """A one-GPU node whose GPU fails every test with a runtime-looking error (device count unchanged) is an
    unhealthy GPU, not a lost runtime: restarting would only re-run the same diagnostics forever."""
    w = World(monkeypatch, n=1)
    bad = "mi355x diag failed (-1): hipSetDevice(device): initialization error"
    monkeypatch.setattr(diag, "run", lambda level, d, memory_partition=None, **kw: (
        w.runs.append(d), {"gemm": {"pass": False, "detail": bad}, "hbm": {"pass": False, "detail": bad}})[1])
    ag = A.Agent("n", source="fake", diag_level=1)
    rep = ag.probe_once()
    assert ag.hip_lost is None and ag.hung_diagnostic() is None
    assert rep["state"] == "unhealthy" and rep["gpus"][0]["diag"]["gemm"]["pass"] is False
    monkeypatch.setattr(diag, "device_count", lambda: 0)  # ... but a count that drops is the runtime
    w.clock += A.DIAG_RECHECK_S
    ag.probe_once()
    assert ag.hip_lost == "HIP device count changed from 1 to 0"


def test_runtime_loss_is_judged_on_devices_that_ran_fine_before(monkeypatch):
    """after a driver reload under a running agent the idle GPUs fail with 'invalid device ordinal'
    while the GPU a pod holds is skipped.  Those GPUs ran fine earlier in this process: the runtime is lost, so
    /healthz restarts the agent -- the idle GPUs are not published as broken hardware for ever."""
    w = World(monkeypatch, n=4)
    lost = "mi355x diag failed (-1): hipSetDevice(device): invalid device ordinal"
    ag = A.Agent("n", source="fake", diag_level=1, diag_interval=0.0)
    assert ag.probe_once()["state"] == "healthy" and ag.hip_lost is None
    monkeypatch.setattr(diag, "run", lambda level, d, memory_partition=None, **kw: (
        w.runs.append(d), {"gemm": {"pass": False, "detail": lost}})[1])
    w.gpus[2] = gpu(2, procs=[{"pid": 7, "vram_mb": 200000}])  # a training job holds gpu2
    w.runs.clear()
    rep = ag.probe_once()
    assert sorted(w.runs) == [0, 1, 3]
    assert ag.hip_lost == lost
    assert all(g["diag_skipped"].startswith("HIP runtime lost its devices") for g in rep["gpus"])


def test_broken_gpus_rechecked_alone_are_not_a_lost_runtime(monkeypatch):
    """two genuinely broken GPUs of eight fail with 'invalid device ordinal'; the recheck runs
    just those two, both fail again -- still their failure, not a lost runtime (no /healthz restart loop)."""
    w = World(monkeypatch, n=8)
    lost = "mi355x diag failed (-1): hipSetDevice(device): invalid device ordinal"

    def run(level, d, memory_partition=None, **kw):
        w.runs.append(d)
        return {"gemm": {"pass": False, "detail": lost}} if d in (3, 6) else {"gemm": {"pass": True}}
    monkeypatch.setattr(diag, "run", run)
    ag = A.Agent("n", source="fake", diag_level=1)
    rep = ag.probe_once()
    assert ag.hip_lost is None and rep["state"] == "unhealthy"
    w.runs.clear()
    w.clock += A.DIAG_RECHECK_S
    rep = ag.probe_once()
    assert sorted(w.runs) == [3, 6]  # the recheck: only the two not-clean GPUs
    assert ag.hip_lost is None and ag.hung_diagnostic() is None and rep["state"] == "unhealthy"
    # the same two as the only idle GPUs of a busy node, on a fresh agent: also their own failure
    for d in range(8):
        if d not in (3, 6):
            w.gpus[d] = gpu(d, procs=[{"pid": 7, "vram_mb": 200000}])
    ag2 = A.Agent("n", source="fake", diag_level=1)
    ag2.probe_once()
    assert ag2.hip_lost is None


def test_one_busy_one_failing_gpu_is_not_a_lost_runtime(monkeypatch):
    """Only one device ran (the other is busy) and it failed with a runtime string: one GPU's failure."""
    w = World(monkeypatch, n=2)
    lost = "mi355x diag failed (-1): hipSetDevice(device): invalid device ordinal"
    monkeypatch.setattr(diag, "run", lambda level, d, memory_partition=None, **kw: (
        w.runs.append(d), {"gemm": {"pass": False, "detail": lost}})[1])
    w.gpus[1] = gpu(1, procs=[{"pid": 7, "vram_mb": 200000}])
    ag = A.Agent("n", source="fake", diag_level=1)
    rep = ag.probe_once()
    assert w.runs == [0] and ag.hip_lost is None and rep["state"] == "unhealthy"

