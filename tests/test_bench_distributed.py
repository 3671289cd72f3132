"""bench.py contract (single process and torchrun world_size=2 on gloo) and the RCCL/xGMI
collective diagnostic's logic on gloo (the GPU run uses backend nccl = RCCL)."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def env():
    e = dict(os.environ)
    e["CUDA_VISIBLE_DEVICES"] = ""  # CPU path even if torch sees a device
    e["HIP_VISIBLE_DEVICES"] = ""
    return e


def last_json(out):
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_single_process_contract():
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "30", "--warmup", "3"],
                       capture_output=True, text=True, timeout=300, env=env(), cwd=REPO)
    assert p.returncode == 0, p.stderr
    d = last_json(p.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 30 and d["warmup"] == 3 and d["scaling"] == "weak"
    assert d["higher_is_better"] is True and d["check_ok"] is True
    assert d["value"] == pytest.approx(1 * 30 / (d["ms_per_step"] * 30 / 1e3), rel=0.01)
    assert d["vs_baseline"] == pytest.approx(d["value"] / (1 / 2.17e-3), rel=0.01)
    assert d["config"]["global_batch"] == 1 and d["backend"] == "native"
    # the BASELINE metric's node-count curve, each row timed like the headline
    curve = d["curve"]
    assert [r["nodes"] for r in curve] == [1, 2, 4, 8, 16, 1000]
    assert all(r["check_ok"] and r["exit_code"] == 0 for r in curve)
    head = curve[0]
    assert head["ms_per_step"] == d["ms_per_step"] and head["annotations"] in ("live", "fixture")
    assert all(r["annotations"] == "recorded" for r in curve[1:])
    for r in curve:
        assert r["vs_baseline"] == pytest.approx(r["baseline_ms"] / r["ms_per_step"], rel=0.01)
        assert r["nodes_per_s"] == pytest.approx(r["nodes"] / (r["ms_per_step"] / 1e3), rel=0.01)
        bd = r["step_ms"]
        # checker_ms is the step minus the socket and the mock's time, per step (medians of sums)
        assert 0 < r["checker_ms"] < bd["step"] and r["transport_ms"] > 0
        assert r["checker_ms"] == bd["checker"] and r["transport_ms"] == bd["transport"]
    assert d["checker_ms"] == head["checker_ms"] and "different machine" in d["baseline_basis"]
    # the checking thread and the mock apiservers on one L3 domain, or the reason they are not
    pin = d["pinning"]
    assert ("skipped" in pin) or (pin["server_cpu"] not in pin["client_cpus"] and pin["client_cpus"])
    # pinned runs also time the headline's check with neither side pinned
    assert d["unpinned"] is None if "skipped" in pin else d["unpinned"]["ms_per_step"] > 0


def test_cpu_pair_and_cpu_lists():
    import bench
    assert bench._cpu_list("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11} and bench._cpu_list("5") == {5}
    pair = bench.cpu_pair()
    if pair is not None:  # this machine's topology: all CPUs allowed, the server apart from the client's
        allowed = os.sched_getaffinity(0)
        assert pair["server_cpu"] in allowed and set(pair["client_cpus"]) <= allowed
        assert pair["server_cpu"] not in pair["client_cpus"] and pair["l3_cpus"] >= 2


def test_bench_torchrun_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py"), "--gpus", "2",
           "--steps", "20", "--warmup", "2"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env(), cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    d = last_json(p.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["check_ok"] and d["health"] == {"healthy": 2}
    assert [r["nodes"] for r in d["curve"]] == [1, 2, 4, 8, 16, 1000] and all(r["check_ok"] for r in d["curve"])
    assert next(r for r in d["curve"] if r["nodes"] == 2)["annotations"] == "fixture"  # the ranks' own: headline
    fab = d["fabric"]  # untimed all-reduce check over the job's process group (gloo here, RCCL on GPUs)
    assert fab["pass"] and fab["world"] == 2 and fab["backend"] == "gloo"
    assert all(r["correct"] for r in fab["rows"]) and len({r["op"] for r in fab["rows"]}) == 4


def test_bench_sweep_mode_and_slack():
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "10", "--warmup", "2", "--mode",
                        "sweep", "--slack", "--nodes", "4"], capture_output=True, text=True, timeout=300, env=env(),
                       cwd=REPO)
    assert p.returncode == 0, p.stderr
    d = last_json(p.stdout)
    assert d["config"]["mode"] == "sweep" and d["config"]["slack"] and d["check_ok"]
    assert d["config"]["global_batch"] == 4


def test_collectives_gloo_two_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "k8s_gpu_node_checker_amd.parallel.collectives",
           "--sizes", "4K,1M", "--iters", "3", "--warmup", "1", "--backend", "gloo"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env(), cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    d = last_json(p.stdout)
    assert d["backend"] == "gloo" and d["world"] == 2 and d["pass"]
    assert all(r["correct"] for r in d["rows"]) and d["rows"][1]["busbw_gbps"] > 0
    assert {r["op"] for r in d["rows"]} == {"all_reduce", "reduce_scatter", "all_gather", "all_to_all"}
    assert set(d["best_busbw_by_op"]) == {"all_reduce", "reduce_scatter", "all_gather", "all_to_all"}


def test_collective_verdict_logic():
    from k8s_gpu_node_checker_amd.parallel.collectives import parse_size, verdict
    assert parse_size("256M") == 256 << 20 and parse_size("1.5K") == 1536
    rows = [{"bytes": 1 << 30, "busbw_gbps": 50.0, "correct": True}]
    assert not verdict(rows, 8)["pass"] and verdict(rows, 8, min_busbw=40)["pass"]
    assert not verdict([dict(rows[0], correct=False)], 8, 1)["pass"]
    bad = verdict(rows + [{"op": "all_to_all", "bytes": 1 << 20, "busbw_gbps": 9.0, "correct": False}], 8, 40)
    assert not bad["pass"] and bad["detail"] == "result mismatch: all_to_all"


def _torchrun(n, *extra, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py"), "--gpus", str(n),
           "--steps", "20", "--warmup", "2", "--coldstart-runs", "2", *extra]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env(), cwd=REPO)


def test_bench_kills_a_node_cycle_that_outlives_the_extras_budget(tmp_path):
    """A node cycle that would run for minutes is killed when the extras budget runs out; the timed loop
    still runs and the line prints with check_ok, every phase's wall time and the kill recorded."""
    sleeper = tmp_path / "sleepy_node_cycle.py"
    sleeper.write_text("import time\ntime.sleep(600)\n")
    t = time.monotonic()
    p = _torchrun(2, "--extras-budget", "12", "--node-cycle-always", "--node-cycle-cmd", f"{sys.executable} {sleeper}")
    wall = time.monotonic() - t
    assert p.returncode == 0, p.stderr[-3000:]
    d = last_json(p.stdout)
    assert d["check_ok"] and d["n_gpus"] == 2 and d["steps"] == 20
    nc = d["node_cycle"]
    assert nc["pass"] is False and nc["killed"] == "budget" and nc["child_wall_s"] < 12
    assert set(d["phases_s"]) >= {"control_plane", "coldstart", "init", "agent_cycle", "publish", "fabric",
                                  "node_cycle", "warmup", "timed"}
    assert d["phases_s"]["node_cycle"] < 12 and d["extras_budget_s"]["budget"] == 12.0
    assert wall < 120, wall


def test_bench_with_no_budget_skips_every_extra_and_still_measures():
    p = _torchrun(2, "--extras-budget", "0", "--node-cycle-always")
    assert p.returncode == 0, p.stderr[-3000:]
    d = last_json(p.stdout)
    assert d["check_ok"] and d["ms_per_step"] > 0
    assert d["coldstart"] == {"skipped": "budget"}
    assert d["fabric"] == {"skipped": "budget"} and d["node_cycle"] == {"skipped": "budget"}
    assert set(d["extras_budget_s"]["skipped"]) == {"coldstart", "fabric", "node_cycle"}
    assert "timed" in d["phases_s"] and "node_cycle" not in d["phases_s"]
