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
