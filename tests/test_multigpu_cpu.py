"""Multi-GPU readiness on CPU (VERDICT r1 "next round" #5): whole 8-GPU agent cycles through the fake C
ABIs of libmi355x_diag.so / libmi355x_fabric.so (testing/fake_native.py) -- per-GPU diagnostic threads,
the node-level xGMI pair matrix and the in-process RCCL suite, and their verdicts -- plus a 4-rank gloo
``torchrun bench.py --gpus 4``.  The real libraries run on an MI355X in tests/test_gpu.py."""
import json
import os
import subprocess
import sys
import time

import pytest

from k8s_gpu_node_checker_amd.agent import agent as A
from k8s_gpu_node_checker_amd.models import health as H
from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag, fabric
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.fake_native import FakeDiagLib, FakeFabricLib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def node8(monkeypatch):
    """An 8 x MI355X node: amd-smi report (all idle), fake diag + fabric libraries."""
    state = {"overrides": {}}

    def install(**kw):
        lib = FakeDiagLib(n=8, **kw)
        fab = FakeFabricLib()
        monkeypatch.setattr(diag, "lib", lambda: lib)
        monkeypatch.setattr(fabric, "_lib", fab)
        monkeypatch.setattr(amdsmi_probe, "probe", lambda node, src, fx: fixtures.mi355x_probe_report(
            node, gpus=8, **state["overrides"]))
        return lib, fab
    install.state = state
    return install


def test_eight_gpu_level2_cycle_is_healthy_and_parallel(node8):
    lib, fab = node8(delay_s=0.15)
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8, diag_timeout=60)
    t0 = time.monotonic()
    rep = ag.probe_once()
    wall = time.monotonic() - t0
    # one host thread per GPU, named after it; the 16 GEMM calls (2 per GPU, 0.15 s each) overlap
    assert {d: lib.threads[d] for d in range(8)} == {d: {f"diag-gpu{d}"} for d in range(8)}
    assert wall < 8 * 2 * 0.15 * 0.6, wall
    for g in rep["gpus"]:
        assert set(g["diag"]) == {"gemm", "gemm_fp8", "hbm", "hbm_xcd", "memtest", "mfma", "lds", "l2", "host_link"}
        assert all(r["pass"] and not r.get("degraded") for r in g["diag"].values()), g["diag"]
    p2p, rccl = rep["fabric"]["p2p"], rep["fabric"]["rccl"]
    assert p2p["pass"] and p2p["median_gbps"] == 48.0
    assert sum(1 for c in lib.calls if c.startswith("p2p")) == 56  # every ordered pair
    assert rccl["pass"] and rccl["rccl"] == "2.27.7" and fab.opened == [list(range(8))] and fab.closed == 1
    assert rep["state"] == H.HEALTHY and rep["expected_gpus"] == 8
    v = ag.evaluate(rep)
    assert (v.gpus_ok, v.gpus_seen) == (8, 8)
    c = H.condition_for(v)
    assert c["status"] == "True" and c["message"] == "8/8 MI355X GPUs healthy"


def test_downed_xgmi_link_makes_the_node_unhealthy(node8):
    # gpu5's link 5 is down (amd-smi) and its traffic to gpu3 crawls over the detour (p2p matrix)
    node8.state["overrides"] = {"gpu5": {"xgmi": "XUUUUDUU"}}
    lib, fab = node8(slow_pairs={(5, 3): 12.0, (3, 5): 13.0})
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8)
    rep = ag.probe_once()
    v = ag.evaluate(rep)
    assert rep["state"] == H.UNHEALTHY and v.state == H.UNHEALTHY and (v.gpus_ok, v.gpus_seen) == (7, 8)
    assert "gpu5: 1 xGMI link(s) down (XUUUUDUU)" in v.reasons
    p2p = [r for r in v.reasons if r.startswith("xGMI p2p failed")]
    assert p2p and "5->3 12.0 GB/s" in p2p[0] and "3->5 13.0 GB/s" in p2p[0]
    cond = H.condition_for(v)
    assert cond["status"] == "False" and cond["reason"] == "MI355XUnhealthy"


def test_rccl_failure_and_a_slow_gpu_on_an_eight_gpu_node(node8):
    lib, fab = node8(gpu_rate={6: 0.55})
    fab.fail_open = True
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8)
    rep = ag.probe_once()
    v = ag.evaluate(rep)
    assert v.state == H.UNHEALTHY and (v.gpus_ok, v.gpus_seen) == (7, 8)
    assert any(r.startswith("gpu6: diag gemm failed") for r in v.reasons)
    assert any(r.startswith("xGMI rccl failed (RCCL init: ncclCommInitAll") for r in v.reasons)
    assert all(g["diag"]["gemm"]["pass"] for g in rep["gpus"] if g["index"] != 6)


def test_eight_gpu_node_with_a_missing_gpu_and_an_allocated_one(node8, monkeypatch):
    """amd-smi sees 7 of the node's 8 GPUs; the fabric test waits while any GPU is busy."""
    lib, fab = node8()
    monkeypatch.setattr(amdsmi_probe, "probe", lambda node, src, fx: dict(
        fixtures.mi355x_probe_report(node, gpus=8), gpus=fixtures.mi355x_probe_report(node, gpus=8)["gpus"][:7]))
    lib.n = 7
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8)
    rep = ag.probe_once()
    v = ag.evaluate(rep)
    assert v.state == H.UNHEALTHY and v.reasons == ["7 of 8 GPUs visible to amd-smi"]
    assert rep["fabric"]["p2p"]["pass"]  # the 7 it has still form a full matrix (42 pairs)
    assert sum(1 for c in lib.calls if c.startswith("p2p")) == 42


def test_bench_torchrun_four_ranks_gloo():
    from test_bench_distributed import env, free_port, last_json
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py"), "--gpus", "4",
           "--steps", "20", "--warmup", "2"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env(), cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    d = last_json(p.stdout)
    assert d["n_gpus"] == 4 and d["config"]["global_batch"] == 4 and d["config"]["parallelism"] == "dp4"
    assert d["check_ok"] and d["health"] == {"healthy": 4} and d["scaling"] == "weak"
    assert d["value"] == pytest.approx(4 * 1e3 / d["ms_per_step"], rel=0.01)
    fab = d["fabric"]
    assert fab["pass"] and fab["world"] == 4 and fab["backend"] == "gloo"
    assert {r["op"] for r in fab["rows"]} == {"all_reduce", "reduce_scatter", "all_gather", "all_to_all"}
    assert all(r["correct"] for r in fab["rows"])
    json.dumps(d)


# --- 8-GPU / 64-partition safety (VERDICT r2 "next round" #2) ----------------------------------------------

def test_shared_host_link_is_serialized_so_halved_concurrent_rates_do_not_fail(node8):
    """Two GPUs behind one switch uplink read the host at half rate each when measured together.  The agent
    measures the host link one GPU at a time (ops/diag.SHARED_TESTS), so an 8-GPU level-2 cycle stays
    healthy; without the lock the same node fails host_link on every GPU."""
    lib, fab = node8(delay_s=0.05)
    lib.link_shared, lib.link_delay_s = True, 0.05
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8, diag_timeout=60)
    rep = ag.probe_once()
    assert lib.peak["host_link"] == 1 and sum(c == "host_link" for c in lib.calls) == 8
    assert all(g["diag"]["host_link"]["pass"] and not g["diag"]["host_link"].get("degraded") for g in rep["gpus"])
    assert rep["state"] == H.HEALTHY
    assert lib.peak.get("gemm", 0) > 1  # the per-GPU compute tests still overlap


def test_unserialized_host_link_would_fail_every_gpu(node8, monkeypatch):
    """The control for the test above: with the shared-test lock disabled the halved rates fail."""
    lib, fab = node8()
    lib.link_shared, lib.link_delay_s = True, 0.2
    monkeypatch.setattr(diag, "SHARED_TESTS", frozenset())
    res = {}

    def one(d):
        res[d] = diag.host_link(d)
    import threading
    ts = [threading.Thread(target=one, args=(d,)) for d in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert lib.peak["host_link"] > 1
    assert any(not r["pass"] for r in res.values())


def test_cpx_node_runs_at_most_diag_parallel_threads_and_finishes_in_time(monkeypatch):
    """64 CPX partitions (8 GPUs x 8): at most --diag-parallel diagnostic threads at once, every partition
    diagnosed in one probe cycle, within the watchdog."""
    import threading
    n = 64
    lib = FakeDiagLib(n=n, cus=32, mem_gib=36, delay_s=0.05)
    monkeypatch.setattr(diag, "lib", lambda: lib)
    rep64 = fixtures.mi355x_probe_report("cpx", gpus=8)
    gpus = []
    for i in range(n):
        g = dict(rep64["gpus"][i // 8], index=i, bdf=f"0000:{0x05 + 0x10 * i:02x}:00.0", compute_partition="CPX",
                 memory_partition="NPS1", cus=32)
        gpus.append(g)
    monkeypatch.setattr(amdsmi_probe, "probe", lambda node, src, fx: dict(rep64, gpus=[dict(g) for g in gpus]))
    live, peak = [0], [0]
    lock = threading.Lock()
    real_run = diag.run

    def run(level, d, **kw):
        with lock:
            live[0] += 1
            peak[0] = max(peak[0], live[0])
        try:
            return real_run(level, d, **kw)
        finally:
            with lock:
                live[0] -= 1
    monkeypatch.setattr(diag, "run", run)
    ag = A.Agent("cpx", source="fake", diag_level=1, diag_timeout=30, diag_parallel=8, expect_gpus=64)
    t0 = time.monotonic()
    rep = ag.probe_once()
    wall = time.monotonic() - t0
    assert peak[0] == 8, peak
    assert all(g.get("diag") and "diag_skipped" not in g for g in rep["gpus"]), \
        [g.get("diag_skipped") for g in rep["gpus"] if g.get("diag_skipped")]
    assert len(set(c for c in lib.threads)) == 64
    assert wall < 30 and rep["state"] in (H.HEALTHY, H.DEGRADED), (wall, rep["state"])
    with pytest.raises(ValueError):
        A.Agent("x", diag_parallel=0)
    assert A.build_parser().parse_args(["--diag-parallel", "4"]).diag_parallel == 4
    assert A.build_parser().parse_args([]).diag_parallel == A.DIAG_PARALLEL


def test_hung_slots_leave_the_rest_waiting_not_running(monkeypatch):
    """With every --diag-parallel slot held by a hung diagnostic the remaining GPUs wait (said per GPU);
    nothing piles more threads onto a wedged device set."""
    import threading
    lib = FakeDiagLib(n=4)
    monkeypatch.setattr(diag, "lib", lambda: lib)
    monkeypatch.setattr(amdsmi_probe, "probe", lambda node, src, fx: fixtures.mi355x_probe_report(node, gpus=4))
    release = threading.Event()
    started = []

    def run(level, d, **kw):
        started.append(d)
        release.wait(20)
        return {"gemm": {"pass": True}}
    monkeypatch.setattr(diag, "run", run)
    ag = A.Agent("n4", source="fake", diag_level=1, diag_timeout=0.2, diag_parallel=2, diag_interval=0.0)
    rep = ag.probe_once()
    assert sorted(started) == [0, 1]
    g = rep["gpus"]
    assert g[0]["diag"]["watchdog"]["pass"] is False and g[1]["diag"]["watchdog"]["pass"] is False
    assert g[2]["diag_skipped"].startswith("waiting for a diagnostic slot: 2 of 2 held by hung")
    rep = ag.probe_once()
    assert sorted(started) == [0, 1] and rep["gpus"][3]["diag_skipped"].startswith("waiting for a diagnostic slot")
    release.set()
    for r in list(ag._diag_threads.values()):
        r.job.thread.join(5)
    rep = ag.probe_once()
    assert sorted(started) == [0, 1, 2, 3]


def test_capped_power_scales_the_compute_references(node8):
    """A GPU whose power cap an operator lowered to 60 % of the default computes at ~60 %: judged against
    its cap it passes (the cap itself is the health model's warning), uncapped it would fail."""
    node8.state["overrides"] = {"gpu3": {"power_cap_w": 840, "power_cap_default_w": 1400}}
    lib, fab = node8(compute_rate={3: 0.62})
    ag = A.Agent("n8", source="fake", diag_level=1, expect_gpus=8)
    rep = ag.probe_once()
    g3 = rep["gpus"][3]
    assert g3["diag"]["gemm"]["pass"] and g3["diag"]["gemm"]["scale"]["compute"] == pytest.approx(0.6)
    v = ag.evaluate(rep)
    assert v.state == H.DEGRADED and any("power cap 840 W of 1400 W" in w for w in v.warnings)
    assert g3["diag"]["hbm"]["pass"] and g3["diag"]["gemm"]["scale"]["memory"] == pytest.approx(1.0, abs=1e-3)
    # the same GPU without the cap on record fails its compute tests
    node8.state["overrides"] = {}
    rep = A.Agent("n8", source="fake", diag_level=1, expect_gpus=8).probe_once()
    assert rep["gpus"][3]["diag"]["gemm"]["pass"] is False and rep["state"] == H.UNHEALTHY
    assert A.power_fraction({"power_cap_w": 1400, "power_cap_default_w": 1400}) == 1.0
    assert A.power_fraction({"power_cap_w": 0, "power_cap_default_w": 1400}) is None
    assert A.power_fraction({}) is None


def test_a_uniformly_slow_hive_fails_the_absolute_floor(node8):
    """every xGMI pair at 20 GB/s is "normal" against its own median, so the relative rule alone
    passes it; the absolute anchor (half a 76 GB/s x16 link at 38 Gb/s, from amd-smi's training) fails it."""
    lib, fab = node8(p2p_gbps=20.0)
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8)
    rep = ag.probe_once()
    p2p = rep["fabric"]["p2p"]
    assert p2p["pass"] is False and p2p["median_gbps"] == 20.0
    assert p2p["link_gbps"] == 76.0 and p2p["floor_gbps"] == 38.0
    assert "0->1 20.0 GB/s under 38 GB/s (50% of a 76 GB/s link)" in p2p["detail"]
    assert rep["state"] == H.UNHEALTHY and any(r.startswith("xGMI p2p failed") for r in ag.evaluate(rep).reasons)
    # a healthy hive at 48 GB/s a pair passes both rules, and both passes ran: 56 pairs, 8 fans of 7
    lib2, _ = node8()
    rep = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8).probe_once()
    p2p = rep["fabric"]["p2p"]
    assert p2p["pass"] and p2p["fan"]["sources"] == 8 and p2p["fan"]["median_gbps"] == 48.0
    assert sum(1 for c in lib2.calls if c.startswith("fan")) == 8 and p2p["fan"]["total_gbps"]["0"] == 7 * 48.0


def test_the_floor_follows_the_trained_link_of_the_median_gpu(node8):
    """Links trained x16 at 25 Gb/s on every GPU (amd-smi): the floor is half of 50 GB/s, so 30 GB/s pairs pass;
    one GPU whose links trained down does not lower the hive's floor."""
    node8.state["overrides"] = {f"gpu{i}": {"xgmi_speed_gbps": 25} for i in range(8)}
    node8(p2p_gbps=30.0)
    rep = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8).probe_once()
    assert rep["fabric"]["p2p"]["floor_gbps"] == 25.0 and rep["fabric"]["p2p"]["pass"]
    node8.state["overrides"] = {"gpu4": {"xgmi_width": 4}}
    node8(p2p_gbps=48.0)
    rep = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8).probe_once()
    assert rep["fabric"]["p2p"]["floor_gbps"] == 38.0


def test_one_link_slow_only_under_load_fails_the_fan_pass(node8):
    """gpu2's link to gpu6 copies at full rate alone (the pair pass) but at 9 GB/s while every link of
    gpu2 is busy (the fan): the fan names it; bad data under load fails too."""
    lib, fab = node8(fan_slow={(2, 6): 9.0})
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8)
    rep = ag.probe_once()
    p2p = rep["fabric"]["p2p"]
    assert p2p["min_gbps"] == 48.0  # the pair pass saw nothing
    assert p2p["pass"] is False and "fan 2->6 9.0 GB/s with every link of 2 busy" in p2p["detail"]
    assert p2p["fan"]["min_gbps"] == 9.0 and rep["state"] == H.UNHEALTHY
    node8(fan_errors={(5, 1): 3})
    rep = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8).probe_once()
    assert "fan 5->1 3 bad words" in rep["fabric"]["p2p"]["detail"]


def test_fan_pass_arguments_and_a_hung_fan(node8):
    from k8s_gpu_node_checker_amd.ops import diag as D
    lib, _ = node8(hung_pairs=((4, 0),))
    # the pair pass hangs first at 4->0 with a deadline; without the pair pass in the way, the fan hangs at it
    f = D.p2p_fan(4, [0, 1, 2], mib=1, iters=1, timeout_s=0.05)
    assert f["hung"] and "p2p fan 4->0" in f["detail"]
    with pytest.raises(RuntimeError, match="every peer must be a device other than the source"):
        D.p2p_fan(1, [1, 2])
    assert D.link_gbs(16, 38) == 76.0 and D.link_gbs(None, None) == 76.0 and D.link_gbs(8, 32) == 32.0


def test_hung_collective_is_aborted_and_reported_as_a_failed_rccl_row(node8):
    """A collective that never completes: the fabric suite's own deadline (0.9 x the watchdog) aborts the
    communicators (ncclCommAbort in fabric.hip) and the report names the hung collective."""
    lib, fab = node8()
    fab.hang_op = 0  # all_reduce never completes
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8, diag_timeout=1.0)
    t0 = time.monotonic()
    rep = ag.probe_once()
    assert time.monotonic() - t0 < 3
    rccl = rep["fabric"]["rccl"]
    assert rccl["pass"] is False and rccl["aborted"] is True and fab.aborts == 1 and fab.closed == 1
    assert "all_reduce" in rccl["detail"] and "ncclCommAbort" in rccl["detail"]
    assert 0 < fab.timeouts_ms[0] <= 900.0
    assert "watchdog" not in rep["fabric"] and rep["state"] == H.UNHEALTHY
    assert any(r.startswith("xGMI rccl failed (all_reduce") for r in ag.evaluate(rep).reasons)
    assert ag._fabric_thread is None  # the suite returned: nothing left holding the GPUs
    assert ag.fabric_abandoned.startswith("RCCL collectives aborted: all_reduce")


def test_hung_xgmi_pair_is_given_up_at_its_share_of_the_deadline(node8):
    """A pair whose copies never complete (diag_p2p_copy_t polls its completion event): the matrix gives up at
    P2P_SHARE of the watchdog, names the pair, and the RCCL suite still runs in what is left."""
    lib, fab = node8(hung_pairs=((3, 5),))
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8, diag_timeout=1.0)
    t0 = time.monotonic()
    rep = ag.probe_once()
    assert time.monotonic() - t0 < 3
    p2p = rep["fabric"]["p2p"]
    assert p2p["pass"] is False and p2p["stopped"].startswith("3->5 hung: p2p 3->5: copies did not complete")
    assert max(lib.p2p_timeouts_ms) <= A.P2P_SHARE * 1000.0
    assert rep["fabric"]["rccl"]["pass"] and fab.closed == 1 and "watchdog" not in rep["fabric"]
    assert any(r.startswith("xGMI p2p failed (3->5 hung") for r in ag.evaluate(rep).reasons)
    assert ag._fabric_thread is None
    # what the hung pair left (queued copies, their buffers) stays with the process: the node-level suite is
    # not run again here -- the failed result stays, marked, until a restart re-tests
    assert ag.fabric_abandoned.startswith("xGMI pair test abandoned: 3->5 hung")
    assert p2p["retest"].startswith("not re-run in this process")
    pairs = sum(1 for c in lib.calls if c.startswith("p2p"))
    ag._fabric_at -= 2 * ag.diag_interval
    for d in list(ag._diag_at):
        ag._diag_at[d] -= 2 * ag.diag_interval
    rep2 = ag.probe_once()
    assert sum(1 for c in lib.calls if c.startswith("p2p")) == pairs and fab.opened == [list(range(8))]
    assert rep2["fabric"]["p2p"]["pass"] is False and rep2["state"] == H.UNHEALTHY


def test_node_cycle_module_over_eight_fake_gpus(node8):
    """agent/node_cycle.py (what bench.py runs on a multi-GPU job): every device diagnosed at once, the
    pair matrix and the RCCL suite, one summary."""
    from k8s_gpu_node_checker_amd.agent import node_cycle
    lib, fab = node8(delay_s=0.05)
    res = node_cycle.run(list(range(8)), level=1, timeout_s=30, parallel=8)
    assert res["peak_threads"] == 8 and res["verdict"] == H.HEALTHY
    assert all(d["pass"] for d in res["per_device"].values()) and len(res["per_device"]) == 8
    assert res["fabric"]["p2p"]["pass"] and res["fabric"]["rccl"]["pass"]
    assert diag.run.__name__ == "run"  # the counting wrapper is removed again
    res4 = node_cycle.run(list(range(8)), level=1, timeout_s=30, parallel=4, fabric=False)
    assert res4["peak_threads"] == 4 and "fabric" not in res4


def test_async_rccl_error_aborts_and_latches_like_a_deadline(node8):
    """a communicator's async error aborts every communicator (fabric.hip wait_comms / sync_all) and
    leaks their buffers like a missed deadline; the suite reports ``aborted`` and the agent does not re-run it
    every --diag-interval (it used to come back as a plain failure and be re-run, leaking each time)."""
    lib, fab = node8()
    fab.async_error_op = 1  # reduce_scatter
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8, diag_timeout=5.0)
    rep = ag.probe_once()
    rccl = rep["fabric"]["rccl"]
    assert rccl["pass"] is False and rccl["aborted"] is True and "communicators aborted" in rccl["detail"]
    assert ag.fabric_abandoned.startswith("RCCL collectives aborted: reduce_scatter")
    ag._fabric_at -= 2 * ag.diag_interval
    for d in list(ag._diag_at):
        ag._diag_at[d] -= 2 * ag.diag_interval
    rep2 = ag.probe_once()
    assert fab.opened == [list(range(8))]  # not opened again
    assert rep2["fabric"]["rccl"]["retest"].startswith("not re-run in this process")


def test_a_gpu_stuck_in_its_host_link_turn_does_not_hang_the_others(node8):
    """the host-link lock was taken with a blocking acquire, so one GPU hung inside its host-link test
    held every other GPU's diagnostics past their watchdog (all reported hung).  Now a device waits only until its
    own deadline and reports the test skipped, naming the holder; its other tests still run."""
    lib, fab = node8()
    assert diag._acquire_shared(5, None) is None  # gpu5 is stuck inside its turn
    try:
        t0 = time.monotonic()
        res = diag.run(2, 1, deadline=time.monotonic() + 0.3)
        assert time.monotonic() - t0 < 2.0
        assert res["host_link"]["skipped"].startswith("host link held by gpu5 for ")
        assert res["host_link"]["pass"] is True and res["gemm"]["pass"]
        v = H.evaluate_report(dict(fixtures.mi355x_probe_report("n", gpus=1), gpus=[
            dict(fixtures.mi355x_probe_report("n", gpus=1)["gpus"][0], diag=res)]), 1)
        assert v.state == H.HEALTHY  # gpu1 is not blamed for gpu5's hang
        text = diag.render_text({"devices": {1: {"info": {}, "tests": res}}, "pass": True})
        assert "host_link  SKIPPED   host link held by gpu5" in text
    finally:
        diag._release_shared()
    assert diag.run(2, 1)["host_link"].get("skipped") is None  # the lock is free again


def test_eight_gpu_baselines_re_form_on_a_driver_upgrade_and_the_floor_holds(node8, monkeypatch):
    """Round-5 rules on a whole 8-GPU node (fake ABI): every GPU forms its self-baseline, a driver upgrade that
    makes the whole node 12 % slower re-forms all eight without a drift warning, and all eight at half rate --
    alike, so peers would excuse each other -- fail under the absolute floor."""
    from k8s_gpu_node_checker_amd.models import baseline as B
    lib, _fab = node8(rate=1.10)
    ag = A.Agent("n8", source="fake", diag_level=1, expect_gpus=8, diag_timeout=60, diag_interval=0.0)
    for _ in range(B.BASELINE_RUNS):
        assert ag.probe_once()["state"] == H.HEALTHY
    assert len(ag.baselines.data) == 8
    epochs = {ag.baselines.epoch(k) for k in ag.baselines.data}
    assert len(epochs) == 1 and next(iter(epochs)).startswith("driver 6.18.54;")
    node8.state["overrides"] = {"driver": {"name": "amdgpu", "version": "6.19.2"}}
    lib.rate = 0.97
    for _ in range(B.BASELINE_RUNS):
        rep = ag.probe_once()
        assert rep["state"] == H.HEALTHY, ag.evaluate(rep).warnings
    assert all(ag.baselines.epoch(k).startswith("driver 6.19.2;") for k in ag.baselines.data)
    lib.rate = 0.5
    rep = ag.probe_once()
    v = ag.evaluate(rep)
    assert v.state == H.UNHEALTHY and (v.gpus_ok, v.gpus_seen) == (0, 8)


def test_eight_node_fleet_with_a_withdrawn_device_plugin(mock_cluster, tmp_path):
    """The membership rule over eight 8-GPU agents' reports: one node's device plugin withdrew every GPU; the
    --mi355x check keeps it as Not Ready with the reason, the other seven Ready."""
    from k8s_gpu_node_checker_amd.checker import CheckOptions, run_check
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    nodes = fixtures.cluster(8, "amd", with_health=True)
    nodes[5]["status"]["allocatable"]["amd.com/gpu"] = "0"
    srv = mock_cluster(nodes)
    res = run_check(ClusterConnection(srv.url), CheckOptions(gpu_source="allocatable", health_policy="require",
                                                             require_schedulable=True))
    assert res.exit_code == 0 and len(res.gpu_nodes) == 8 and len(res.ready_gpu_nodes) == 7
    v = res.verdicts[5]
    assert v.state == H.UNHEALTHY and v.reasons[0] == "device plugin allocates 0 of 8 amd.com/gpu"


def test_eight_gpu_level2_cycle_with_process_isolation(monkeypatch):
    """the DaemonSet's configuration on a whole 8-GPU node, on CPU -- every GPU's suite in its own
    child narrowed to that GPU, at most --diag-parallel at once, then the xGMI matrix (pairs and fans) and the RCCL
    suite in one node-level child; one GPU hangs and is SIGKILLed at the watchdog, another's link is slow only under
    the fan.  The agent process never loads the diagnostics library."""
    from k8s_gpu_node_checker_amd.agent import isolation
    monkeypatch.setattr(amdsmi_probe, "probe", lambda node, src, fx: fixtures.mi355x_probe_report(node, gpus=8))

    def no_hip_here():
        raise AssertionError("the agent process called the HIP diagnostics library")
    monkeypatch.setattr(diag, "lib", no_hip_here)
    fake = {"n": 8, "hang_devices": (5,), "fan_slow": {(3, 6): 9.0}}
    ag = A.Agent("n8", source="fake", diag_level=2, expect_gpus=8, diag_timeout=4.0, diag_parallel=4, diag_interval=0.0,
                 diag_when="always", isolation="process",
                 diag_setup=("k8s_gpu_node_checker_amd.testing.fake_native", "install", fake))
    t0 = time.monotonic()
    rep = ag.probe_once()
    assert time.monotonic() - t0 < 2 * 4.0 + isolation.KILL_GRACE_S + 5
    started = [c["what"] for c in ag.workers.started]
    assert started[0] == "hip-enumerate" and sorted(started[1:9]) == sorted(f"diag-gpu{d}" for d in range(8))
    for d, g in enumerate(rep["gpus"]):
        if d == 5:
            assert g["diag"]["watchdog"]["pass"] is False and "killed" in g["diag"]["watchdog"]["detail"]
            continue
        assert all(r["pass"] for r in g["diag"].values()), (d, g["diag"])
        assert g["diag_proc"]["bdf"] == g["bdf"]  # each child measured its own GPU (narrowed, then checked)
    # the node-level suite waits for an all-clean cycle of per-GPU jobs: not this one (gpu5 hung)
    assert "diag-fabric" not in started
    v = ag.evaluate(rep)
    assert v.state == H.UNHEALTHY and (v.gpus_ok, v.gpus_seen) == (7, 8)
    # a later cycle without the hang runs the fabric child, whose fan pass names the slow link
    ag.workers.setup = ("k8s_gpu_node_checker_amd.testing.fake_native", "install", dict(fake, hang_devices=()))
    rep = ag.probe_once()
    assert [c["what"] for c in ag.workers.started].count("diag-fabric") == 1
    p2p = rep["fabric"]["p2p"]
    assert p2p["pass"] is False and "fan 3->6 9.0 GB/s with every link of 3 busy" in p2p["detail"]
    assert p2p["fan"]["sources"] == 8 and rep["fabric"]["rccl"]["pass"]
