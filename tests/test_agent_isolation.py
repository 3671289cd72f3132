"""Process isolation of the agent's HIP diagnostics (agent/isolation.py): each cycle's suites
run in disposable children of a forkserver started before the agent touches amd-smi or HIP.  The children run the
real ``ops/diag`` code against the fake C ABIs (``testing/fake_native.install``), so a hung or aborting GPU is
scripted on CPU; the agent process itself never loads a diagnostics library."""
import os
import time
import urllib.request

import pytest

from k8s_gpu_node_checker_amd.agent import agent as A
from k8s_gpu_node_checker_amd.agent import isolation
from k8s_gpu_node_checker_amd.models import health as H
from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag
from k8s_gpu_node_checker_amd.testing import fixtures

FAKE = "k8s_gpu_node_checker_amd.testing.fake_native"


@pytest.fixture
def node(monkeypatch):
    """An n-GPU MI355X node: the amd-smi report in this process, the diagnostics only in children (a call to the
    diag library here fails the test)."""
    def make(n=2, **overrides):
        monkeypatch.setattr(amdsmi_probe, "probe", lambda nd, src, fx: fixtures.mi355x_probe_report(
            nd, gpus=n, **overrides))

        def no_hip_here():
            raise AssertionError("the agent process called the HIP diagnostics library")
        monkeypatch.setattr(diag, "lib", no_hip_here)
    return make


def agent(n=2, level=1, timeout=30.0, **fake):
    return A.Agent("n", source="fake", diag_level=level, diag_interval=0.0, diag_timeout=timeout, expect_gpus=n,
                   diag_when="always", isolation="process", diag_setup=(FAKE, "install", dict(n=n, **fake)))


def gone(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return True
    try:  # a zombie not yet reaped by its parent counts as gone
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] == "Z"
    except OSError:
        return True


def test_diagnostics_run_in_children_and_the_agent_never_loads_hip(node):
    node(2)
    ag = agent(2)
    rep = ag.probe_once()
    assert rep["state"] == H.HEALTHY
    for g in rep["gpus"]:
        assert g["diag"]["gemm"]["pass"] and g["diag"]["hbm"]["pass"]
        proc = g["diag_proc"]
        assert proc["pid"] != os.getpid() and proc["peak_rss_mib"] > 0 and gone(proc["pid"])
    kinds = [c["what"] for c in ag.workers.started]
    assert kinds == ["hip-enumerate", "diag-gpu0", "diag-gpu1"]
    assert ag._bdf == {0: "0000:05:00.0", 1: "0000:15:00.0"}  # PCI addresses from the enumeration child
    # the child's metadata is not part of the annotation nor of the change digest
    assert "diag_proc" not in ag.annotation(rep)[A.HEALTH_ANNOTATION]
    m = A._metrics(rep)
    assert 'mi355x_agent_diag_child_peak_rss_bytes{gpu="0"' in m
    # the next cycle starts fresh children (new pids): nothing of the last one is kept
    rep2 = ag.probe_once()
    assert {g["diag_proc"]["pid"] for g in rep2["gpus"]}.isdisjoint({g["diag_proc"]["pid"] for g in rep["gpus"]})


def test_a_hung_gpu_child_is_killed_at_the_watchdog_and_published_failed(node, mock_cluster):
    """The done-when of VERDICT r5 #2: the agent publishes a failed verdict within --diag-timeout, /healthz stays
    200, the hung child is gone, and the next cycle diagnoses the GPU again in a new child."""
    from k8s_gpu_node_checker_amd.kube.client import KubeClient
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    node(2)
    srv = mock_cluster([fixtures.realistic_node("n", gpu_count=2)])
    ag = agent(2, timeout=2.0, hang_devices=(1,))
    http = A.serve(ag, "127.0.0.1", 0, stale_after=60)
    url = f"http://127.0.0.1:{http.server_address[1]}/healthz"
    try:
        t0 = time.monotonic()
        rep = ag.probe_once()
        wall = time.monotonic() - t0
        with KubeClient(ClusterConnection(srv.url)) as kc:
            ag.publish(kc, rep)
            cond = [c for c in kc.get_node("n")["status"]["conditions"] if c["type"] == H.HEALTH_CONDITION][0]
        assert wall < 2.0 + isolation.KILL_GRACE_S + 3, wall
        g0, g1 = rep["gpus"]
        assert g0["diag"]["gemm"]["pass"]
        wd = g1["diag"]["watchdog"]
        assert wd["pass"] is False and "within 2 s (GPU hang?): diagnostic process" in wd["detail"]
        assert wd["detail"].endswith("killed")
        assert rep["state"] == H.UNHEALTHY and cond["status"] == "False" and "watchdog" in cond["message"]
        hung = [c["pid"] for c in ag.workers.started if c["what"] == "diag-gpu1"]
        assert len(hung) == 1 and gone(hung[0])
        assert ag._diag_threads == {} and ag.hung_diagnostic() is None and ag.hip_lost is None
        assert urllib.request.urlopen(url, timeout=5).status == 200
        # the next cycle: GPU 1 gets a new child (and is reported hung again), GPU 0 keeps passing
        rep = ag.probe_once()
        assert len([c for c in ag.workers.started if c["what"] == "diag-gpu1"]) == 2
        assert "watchdog" in rep["gpus"][1]["diag"] and rep["gpus"][0]["diag"]["gemm"]["pass"]
        assert urllib.request.urlopen(url, timeout=5).status == 200
    finally:
        http.shutdown()
        http.server_close()


def test_a_gpu_fault_that_aborts_the_runtime_costs_its_child_not_the_agent(node):
    node(2)
    ag = agent(2, abort_devices=(0,))
    rep = ag.probe_once()
    run = rep["gpus"][0]["diag"]["run"]
    assert run["pass"] is False and "ended before reporting (signal SIGABRT)" in run["detail"]
    assert rep["gpus"][1]["diag"]["gemm"]["pass"] and rep["state"] == H.UNHEALTHY
    assert ag.hung_diagnostic() is None and ag.hip_lost is None


def test_no_hip_device_in_the_enumeration_child(node):
    node(2)
    ag = agent(0)
    rep = ag.probe_once()
    assert [g.get("diag_skipped") for g in rep["gpus"]] == \
        ["no HIP device visible to the agent (/dev/kfd and /dev/dri mounted?)"] * 2
    assert [c["what"] for c in ag.workers.started] == ["hip-enumerate"]


def test_level2_fabric_suite_runs_in_its_own_child(node):
    node(2)
    ag = agent(2, level=2)
    rep = ag.probe_once()
    assert rep["fabric"]["p2p"]["pass"] and rep["fabric"]["rccl"]["pass"] and rep["state"] == H.HEALTHY
    assert [c["what"] for c in ag.workers.started] == ["hip-enumerate", "diag-gpu0", "diag-gpu1", "diag-fabric"]
    assert "fabric" in ag.diag_procs and ag.diag_procs["fabric"]["pid"] != os.getpid()


def test_a_hung_fabric_child_is_killed_and_the_suite_runs_again(node):
    """An RCCL wait that ignores its deadline (stuck in the driver): the fabric child is SIGKILLed at the watchdog;
    what it left queued ended with it, so the suite is not barred from running again (thread isolation must bar it,
    fabric_abandoned)."""
    node(2)
    ag = agent(2, level=2, timeout=2.0, fabric={"hang_op": 0, "ignore_deadline": True})
    t0 = time.monotonic()
    rep = ag.probe_once()
    assert time.monotonic() - t0 < 2 * 2.0 + isolation.KILL_GRACE_S + 3
    wd = rep["fabric"]["watchdog"]
    assert wd["pass"] is False and "fabric hang?): diagnostic process" in wd["detail"] and rep["state"] == H.UNHEALTHY
    assert ag.fabric_abandoned is None and ag._fabric_thread is None
    rep = ag.probe_once()
    assert len([c for c in ag.workers.started if c["what"] == "diag-fabric"]) == 2


def test_host_link_turns_are_shared_across_children(node):
    """The suites of one cycle take turns at the PCIe host link through a multiprocessing lock: with a child that
    hangs inside its host-link test, another child reports that test skipped, naming the holder, within its own
    deadline."""
    lock, cell = isolation.Workers("process").host_lock()
    diag.use_host_lock(lock, cell)
    try:
        assert diag._acquire_shared(3, None) is None
        assert cell[0] == 3.0
        why = diag._acquire_shared(5, time.monotonic() + 0.2)
        assert why.startswith("host link held by gpu3 for ")
        diag._release_shared()
        assert cell[0] == -1.0 and diag._acquire_shared(5, time.monotonic() + 0.2) is None
        diag._release_shared()
    finally:
        import threading
        diag.use_host_lock(threading.Lock(), None)


def test_isolation_flag_and_thread_mode_default():
    assert A.build_parser().parse_args([]).diag_isolation == "process"
    assert A.build_parser().parse_args(["--diag-isolation", "thread"]).diag_isolation == "thread"
    assert A.Agent("n", diag_level=1).isolation == "thread"  # the library default (benchmark, in-process tests)
    assert A.Agent("n", diag_level=0, isolation="process").isolation == "thread"  # no diagnostics: no forkserver
    with pytest.raises(ValueError):
        A.Agent("n", isolation="container")
    assert isolation.describe_exit(-9) == "signal SIGKILL" and isolation.describe_exit(3) == "exit code 3"


def test_narrowing_and_a_misdirected_child():
    """Each device child sees only its GPU (HIP_VISIBLE_DEVICES), picked from a list the agent itself was narrowed
    to; a child that reports another PCI address than the enumeration gave its ordinal is not that GPU's result."""
    env = {}
    assert isolation.narrow_to(3, env) == "3" and env == {"HIP_VISIBLE_DEVICES": "3"}
    env = {"HIP_VISIBLE_DEVICES": "4,6,7"}
    assert isolation.narrow_to(1, env) == "6" and env["HIP_VISIBLE_DEVICES"] == "6"
    env = {"CUDA_VISIBLE_DEVICES": "GPU-aa,GPU-bb"}
    assert isolation.narrow_to(1, env) == "GPU-bb" and env == {"HIP_VISIBLE_DEVICES": "GPU-bb"}
    env = {"HIP_VISIBLE_DEVICES": "2"}
    assert isolation.narrow_to(1, env) is None and env == {"HIP_VISIBLE_DEVICES": "2"}
    assert A.misdirected("0000:05:00.0", {"bdf": "0000:05:00.0"}) is None
    assert A.misdirected("", {"bdf": "0000:05:00.0"}) is None and A.misdirected("0000:05:00.0", None) is None
    assert A.misdirected("0000:05:00.0", {"bdf": "15:00.0"}) == (
        "diagnostic process ran on 0000:15:00.0, not 0000:05:00.0: HIP device visibility mismatch")



def test_agent_cli_default_isolation_on_a_box_without_a_gpu(tmp_path, capsys):
    """The DaemonSet's entry point with its default (process isolation) where HIP sees no GPU: the enumeration
    child says so, every GPU carries the reason, and the agent itself exits normally."""
    import json
    fx = tmp_path / "fx.json"
    fx.write_text(json.dumps(fixtures.mi355x_probe_report("n", gpus=2)))
    rc = A.main(["--node", "n", "--once", "--source", "fixture", "--fixture", str(fx), "--publish", "stdout",
                 "--diag-level", "1", "--diag-timeout", "60"])
    rep = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1])
    assert rc == 0
    reasons = [g.get("diag_skipped") or "" for g in rep["gpus"]]
    assert all(r.startswith(("no HIP device visible", "HIP device enumeration failed")) for r in reasons), reasons


def test_a_child_that_cannot_start_is_that_gpus_failure(node, monkeypatch):
    node(2)
    ag = agent(2)

    class Broken:
        def __init__(self, *a, **kw):
            pass

        def start(self):
            raise OSError(12, "Cannot allocate memory")
    monkeypatch.setattr(ag.workers.ctx, "Process", Broken)
    rep = ag.probe_once()  # the enumeration could not start either: said per GPU, the agent goes on
    assert all(g["diag_skipped"].startswith("HIP device enumeration failed: could not start the diagnostic process")
               for g in rep["gpus"])
    job = ag.workers.device(1, 0, {}, __import__("threading").Event())
    assert not job.is_alive() and job.box["res"]["run"]["detail"].startswith("could not start the diagnostic process")


def _record_env():
    """Child setup: the fake C ABI, and a suite that reports the environment the child's HIP runtime would start with."""
    from k8s_gpu_node_checker_amd.testing import fake_native
    fake_native.install(n=1)
    diag.run = lambda level, device, **kw: {"env": {"pass": True, "sdma": os.environ.get("HSA_ENABLE_SDMA"),
                                                    "visible": os.environ.get("HIP_VISIBLE_DEVICES")}}


def test_a_child_whose_suite_times_no_dma_copy_starts_hip_without_sdma(monkeypatch):
    """Level 1 times no DMA-engine copy: its child starts HIP with HSA_ENABLE_SDMA=0 (the SDMA queues' ~180 MiB of
    host memory never allocated); level 2's host-link test times SDMA, so its child keeps the engines."""
    import threading
    monkeypatch.delenv("HSA_ENABLE_SDMA", raising=False)
    assert not diag.uses_dma(1) and diag.uses_dma(2) and not diag.uses_dma(0)
    w = isolation.Workers("process", setup=(__name__, "_record_env", {}), method="fork")
    for level, want in ((1, "0"), (2, None)):
        done = threading.Event()
        job = w.device(level, 0, {}, done)
        assert done.wait(30)
        env = job.box["res"]["env"]
        assert env["sdma"] == want and env["visible"] == "0", (level, env)
    assert os.environ.get("HSA_ENABLE_SDMA") is None  # the agent's own environment is untouched


def _sigkill_self():
    """Child setup: the child is SIGKILLed from outside the agent (as the kernel's OOM killer would) before reporting."""
    import signal
    os.kill(os.getpid(), signal.SIGKILL)


def test_a_child_killed_from_outside_the_agent_says_so():
    """A SIGKILL the agent did not send (the pod's memory limit) is told apart from the watchdog's."""
    import threading
    w = isolation.Workers("process", setup=(__name__, "_sigkill_self", {}), method="fork")
    done = threading.Event()
    job = w.device(1, 0, {}, done)
    assert done.wait(30)
    detail = job.box["res"]["run"]["detail"]
    assert "signal SIGKILL" in detail and "not killed by the agent" in detail and "memory limit" in detail
    assert not job.killed


def test_an_oom_killed_child_is_not_the_gpus_failure(node, monkeypatch):
    """A device child the pod's memory limit kills (a SIGKILL the agent did not send) leaves that GPU's last result
    standing, says why in ``diag_skipped``, and the GPU is diagnosed again next cycle; the same for the node-level
    child, in ``fabric_skipped``."""
    node(2)
    ag = agent(2, level=2)
    rep = ag.probe_once()
    assert rep["state"] == H.HEALTHY and all(g["diag"]["gemm"]["pass"] for g in rep["gpus"]) and rep["fabric"]
    first = {g["index"]: g["diag_proc"]["pid"] for g in rep["gpus"]}
    real_spawn = ag.workers._spawn

    def oom(victims):
        def spawn(what, target, args, done, died):
            if what in victims:
                args = ((__name__, "_sigkill_self", {}),) + tuple(args[1:])
            return real_spawn(what, target, args, done, died)
        monkeypatch.setattr(ag.workers, "_spawn", spawn)
    oom({"diag-gpu1"})
    rep = ag.probe_once()
    g0, g1 = rep["gpus"]
    assert rep["state"] == H.HEALTHY, rep.get("reasons")  # not the GPU's finding
    assert g0["diag_proc"]["pid"] != first[0] and g0["diag"]["gemm"]["pass"]
    assert "not killed by the agent" in g1["diag_skipped"] and g1["diag"]["gemm"]["pass"]  # last result stands
    assert ag._diag_at[1] == float("-inf")  # due again next cycle
    oom({"diag-fabric"})  # every GPU fine this time, so the node-level child runs -- and is killed
    rep = ag.probe_once()
    assert rep["state"] == H.HEALTHY and "diag_skipped" not in rep["gpus"][1]
    assert "not killed by the agent" in rep["fabric_skipped"] and rep["fabric"]  # the last fabric result stands
    monkeypatch.setattr(ag.workers, "_spawn", real_spawn)
    rep = ag.probe_once()
    assert "fabric_skipped" not in rep and rep["fabric"] and rep["state"] == H.HEALTHY
