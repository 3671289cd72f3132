"""Fleet-relative diagnostic verdicts (models/fleet.py): the checker judges each MI355X node's diagnostic rates
against the other nodes of the same LIST.

Agent reports come from whole agent cycles on the fake C ABI of libmi355x_diag.so (testing/fake_native.py), one
agent per node; the checker reads them from node annotations served by the mock apiserver.  Reference: the
verdict is a stable binary read off each node (/root/reference/check-gpu-node.py:172-178) -- a fleet whose
platform is slower than the boxes the references were measured on must not page as degraded.
"""
import json

import pytest

from k8s_gpu_node_checker_amd.agent import agent as A
from k8s_gpu_node_checker_amd.checker import CheckOptions, apply_health, scan_cluster
from k8s_gpu_node_checker_amd.models import fleet as F
from k8s_gpu_node_checker_amd.models import health as H
from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag, fabric
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.fake_native import FakeDiagLib, FakeFabricLib
from k8s_gpu_node_checker_amd.testing.mock_apiserver import write_kubeconfig
from k8s_gpu_node_checker_amd.utils.timing import NullTracer


@pytest.fixture
def reports(monkeypatch):
    """``reports({name: rate or {gpu: rate}}, gpus=8, **agent kw)`` -> {name: the agent's report}."""
    def make(rates, gpus=8, **kw):
        out = {}
        monkeypatch.setattr(fabric, "_lib", FakeFabricLib())
        monkeypatch.setattr(amdsmi_probe, "probe", lambda nd, src, fx: fixtures.mi355x_probe_report(nd, gpus=gpus))
        for name, rate in rates.items():
            lib = (FakeDiagLib(n=gpus, gpu_rate=rate) if isinstance(rate, dict) else FakeDiagLib(n=gpus, rate=rate))
            monkeypatch.setattr(diag, "lib", lambda lib=lib: lib)
            out[name] = A.Agent(name, source="fake", diag_level=1, expect_gpus=gpus, diag_timeout=60,
                                diag_baseline=False, **kw).probe_once()
        return out
    return make


def _judge(reps, gpus=8):
    names = list(reps)
    summary, views = F.judge_fleet(names, [reps[n] for n in names])
    return summary, {n: H.evaluate_report(reps[n], gpus, fleet=v) for n, v in zip(names, views)}


def test_a_fleet_slow_alike_is_the_platforms_normal(reports):
    """Four 8-GPU nodes, every GPU at 0.88 of the references: each agent alone calls its node degraded (one
    node-wide finding); across the fleet that is the platform, and every node is healthy."""
    reps = reports({f"n{i}": 0.88 for i in range(4)})
    assert all(H.evaluate_report(r, 8).state == H.DEGRADED for r in reps.values())
    summary, verdicts = _judge(reps)
    assert all(v.state == H.HEALTHY and not v.warnings for v in verdicts.values()), \
        {n: v.warnings for n, v in verdicts.items()}
    row = summary["gemm@[4096, 4096, 4096]/tflops"]
    assert row["nodes"] == 4 and row["platform_shortfall"] and row["median_fraction"] == pytest.approx(0.88, abs=1e-3)
    assert row["outliers"] == []


def test_one_node_behind_the_fleet_is_degraded_by_name(reports):
    """A fast fleet (1.10 of the references) and one node whose GPUs all run at 0.88: above the absolute floor,
    so its own agent calls it at most degraded; 80 % of the other nodes' median names it."""
    reps = reports({"n0": 1.10, "n1": 1.10, "n2": 1.10, "slow": 0.88})
    summary, verdicts = _judge(reps)
    assert all(verdicts[n].state == H.HEALTHY for n in ("n0", "n1", "n2"))
    v = verdicts["slow"]
    assert v.state == H.DEGRADED and not v.reasons  # all of its GPUs alike, above the floor: the node's condition
    fleet_w = [w for w in v.warnings if w.startswith("fleet: ")]
    assert any(w.startswith("fleet: diag gemm tflops at 80% of the other 3 nodes' median (88% vs 110%") for w in fleet_w)
    assert {"node": "slow", "ratio": 0.8} in summary["gemm@[4096, 4096, 4096]/tflops"]["outliers"]


def test_a_node_at_the_reference_behind_a_fast_fleet_is_listed_not_degraded(reports):
    """A fleet at 1.15 of the references and one node at 0.96: 83 % of the others, but at the MI355X reference
    itself (healthy devices differ this much, profiles/diag_box_spread_r05_mi355x.jsonl) -- no degraded finding,
    no outlier (the MI355XNodeBehindFleet alert counts outliers); the summary lists it as behind at the reference."""
    reps = reports({"n0": 1.15, "n1": 1.15, "n2": 1.15, "ok": 0.96})
    summary, verdicts = _judge(reps)
    assert verdicts["ok"].state == H.HEALTHY and not [w for w in verdicts["ok"].warnings if w.startswith("fleet: ")]
    row = summary["gemm@[4096, 4096, 4096]/tflops"]
    assert row["outliers"] == [] and [o["node"] for o in row["behind_at_reference"]] == ["ok"]


def test_a_node_behind_the_fleet_under_the_floor_fails(reports):
    """GPUs alike under the absolute failure line fail; the fleet names the node as well."""
    reps = reports({"n0": 1.0, "n1": 1.0, "n2": 1.0, "slow": 0.80})
    summary, verdicts = _judge(reps)
    v = verdicts["slow"]
    assert v.state == H.UNHEALTHY and {r.split(":")[0] for r in v.reasons} == {f"gpu{d}" for d in range(8)}
    assert {"node": "slow", "ratio": 0.8} in summary["gemm@[4096, 4096, 4096]/tflops"]["outliers"]


def test_lone_gpu_nodes_slow_alike_pass_but_the_floor_stays(reports):
    """1-GPU nodes judge their GPU against the references (no peers on the node): a fleet of them at 0.88 is
    the platform; at 0.80 they are under the absolute floor and still fail -- the fleet excuses slowness only."""
    reps = reports({f"n{i}": 0.88 for i in range(3)}, gpus=1)
    assert all(any(w.startswith("gpu0: diag gemm slow") for w in H.evaluate_report(r, 1).warnings)
               for r in reps.values())
    _, verdicts = _judge(reps, 1)
    assert all(v.state == H.HEALTHY for v in verdicts.values()), {n: v.warnings for n, v in verdicts.items()}
    reps = reports({f"n{i}": 0.80 for i in range(3)}, gpus=1)
    _, verdicts = _judge(reps, 1)
    assert all(v.state == H.UNHEALTHY and v.reasons[0].startswith("gpu0: diag gemm failed") for v in verdicts.values())


def test_a_gpu_failing_its_peers_is_not_excused_by_the_fleet(reports):
    reps = reports({"n0": 0.88, "n1": 0.88, "n2": 0.88, "bad": {d: (0.70 if d == 3 else 0.88) for d in range(8)}})
    _, verdicts = _judge(reps)
    assert verdicts["bad"].state == H.UNHEALTHY and all(r.startswith("gpu3: ") for r in verdicts["bad"].reasons)
    assert all(verdicts[n].state == H.HEALTHY for n in ("n0", "n1", "n2"))


def test_fewer_than_three_nodes_change_nothing(reports):
    reps = reports({"n0": 0.88, "n1": 0.88})
    summary, verdicts = _judge(reps)
    assert summary == {} and all(v.state == H.DEGRADED for v in verdicts.values())


def test_the_fleet_judgement_leaves_the_reports_as_they_were(reports):
    """The watcher keeps parsed reports across checks: judging must not change them."""
    reps = reports({f"n{i}": 0.88 for i in range(3)} | {"slow": 0.7})
    snap = json.dumps(reps, sort_keys=True)
    a = _judge(reps)
    assert json.dumps(reps, sort_keys=True) == snap
    b = _judge(reps)
    def verdicts(x):
        return {n: (v.state, v.reasons, v.warnings) for n, v in x[1].items()}
    assert a[0] == b[0] and verdicts(a) == verdicts(b)


def test_stale_reports_are_left_out_of_the_fleet(reports):
    reps = reports({f"n{i}": 0.88 for i in range(4)})
    for n in ("n0", "n1"):
        reps[n]["ts"] -= 10 * 86400
    names = list(reps)
    exp = H.HealthExpectations()
    current = [r if H.report_gate(r, exp) is None else None for r in reps.values()]
    summary, views = F.judge_fleet(names, current)
    assert summary == {} and views == [None] * 4


# --- through the checker --------------------------------------------------------------------------------------

def _cluster(mock_cluster, tmp_path, reps, gpus=8):
    nodes = [fixtures.realistic_node(name, gpu_count=gpus, index=i, annotations=fixtures.health_annotation(rep),
                                     extra_conditions=[fixtures.health_condition(rep, gpus)])
             for i, (name, rep) in enumerate(reps.items())]
    srv = mock_cluster(nodes)
    return srv, write_kubeconfig(str(tmp_path / "kc"), srv.url)


def test_checker_paths(reports, mock_cluster, tmp_path):
    """The default check trusts each agent's condition (degraded); with the reports read (--health-reeval or
    --json-extended) the fleet judgement applies; the summary rides in --json-extended."""
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    reps = reports({f"n{i}": 0.88 for i in range(3)} | {"slow": 0.70})
    srv, _kc = _cluster(mock_cluster, tmp_path, reps)
    cluster = ClusterConnection(srv.url)

    def states(**kw):
        opts = CheckOptions(**kw)
        scan = scan_cluster(cluster, opts, NullTracer())
        out: dict = {}
        vs = apply_health(scan, opts, NullTracer(), [], cluster, out)
        return {n["name"]: v.state for n, v in zip(scan.gpu_nodes, vs)}, out
    plain, out = states()
    # the 0.70 node is under the absolute floor on every GPU: its agent already calls it unhealthy
    assert plain == {"n0": H.DEGRADED, "n1": H.DEGRADED, "n2": H.DEGRADED, "slow": H.UNHEALTHY} and out == {}
    for kw in ({"health_reeval": True}, {"json_extended": True}):
        st, out = states(**kw)
        assert st == {"n0": H.HEALTHY, "n1": H.HEALTHY, "n2": H.HEALTHY, "slow": H.UNHEALTHY}, (kw, st)
        assert out["summary"]["gemm@[4096, 4096, 4096]/tflops"]["outliers"][0]["node"] == "slow"


def test_cli_fleet_and_explain_show_the_fleet(run_cli, reports, mock_cluster, tmp_path):
    reps = reports({f"n{i}": 0.88 for i in range(3)} | {"slow": 0.70})
    _srv, kc = _cluster(mock_cluster, tmp_path, reps)
    p = run_cli(["--kubeconfig", kc, "--fleet"])
    assert p.returncode == 0, p.stdout + p.stderr
    assert "MI355X verdicts: 3 healthy, 1 unhealthy" in p.stdout
    assert "  slow: unhealthy (not Ready)  " in p.stdout
    line = next(ln for ln in p.stdout.splitlines() if ln.startswith("  gemm@[4096, 4096, 4096]/tflops: "))
    assert "4 nodes, median 88% (70%-88%)" in line and "platform shortfall" in line and "slow x0.80" in line
    p = run_cli(["--kubeconfig", kc, "--explain", "n1"])
    assert p.returncode == 0 and "MI355X verdict: healthy" in p.stdout
    assert "  fleet: diag gemm tflops: the fleet's median node is at 88% of the MI355X reference (4 nodes alike)" \
        in p.stdout
    assert "  fleet: lowest against the fleet's median node: " in p.stdout
    p = run_cli(["--kubeconfig", kc, "--explain", "slow"])
    low = next(ln for ln in p.stdout.splitlines() if "lowest against the fleet's median node" in ln)
    assert "x0.80" in low, low
    d = json.loads(run_cli(["--kubeconfig", kc, "--explain", "slow", "--json"]).stdout)
    assert d["fleet_diag"]["node_ratio"]["gemm@[4096, 4096, 4096]/tflops"] == pytest.approx(0.795, abs=0.01)
    d = json.loads(run_cli(["--kubeconfig", kc, "--json", "--json-extended"]).stdout)
    assert d["mi355x"]["diag_fleet"]["gemm@[4096, 4096, 4096]/tflops"]["nodes"] == 4


def test_fleet_gauges_in_the_metrics(reports, mock_cluster, tmp_path):
    from k8s_gpu_node_checker_amd.checker import run_check
    from k8s_gpu_node_checker_amd.kube.config import ClusterConnection
    from k8s_gpu_node_checker_amd.utils import prom
    reps = reports({f"n{i}": 0.88 for i in range(3)} | {"slow": 0.70})
    srv, _kc = _cluster(mock_cluster, tmp_path, reps)
    res = run_check(ClusterConnection(srv.url), CheckOptions(health_reeval=True))
    text = "\n".join(prom.render(res))
    assert 'k8s_gpu_checker_diag_fleet_median_fraction{test="gemm@[4096, 4096, 4096]/tflops"} 0.88' in text
    assert 'k8s_gpu_checker_diag_fleet_outlier_nodes{test="gemm@[4096, 4096, 4096]/tflops"} 1' in text
    assert 'k8s_gpu_checker_mi355x_health{node="n0",state="healthy"} 1' in text


# --- property tests --------------------------------------------------------------------------------------------

from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from k8s_gpu_node_checker_amd.models import peers as P  # noqa: E402


def _node_report(name, fracs):
    """A report whose GPUs ran only the level-1 GEMM at the given fractions of a 1,228 TFLOP/s reference, judged
    by the agent's peer rules."""
    pool = {d: {"gemm": dict(diag._rated({"shape": [4096, 4096, 4096]}, {"tflops": 1228.0 * f}, {"tflops": 1228.0},
                                         "TFLOP/s"))} for d, f in enumerate(fracs)}
    findings = P.judge_node(pool)
    rep = fixtures.mi355x_probe_report(name, gpus=len(fracs))
    for d, g in enumerate(rep["gpus"]):
        g["diag"] = pool[d]
    if findings:
        rep["diag_node"] = {"findings": findings}
    return rep


_frac = st.floats(min_value=0.3, max_value=1.3, allow_nan=False)


@settings(max_examples=150, deadline=None)
@given(st.lists(st.lists(_frac, min_size=1, max_size=4), min_size=1, max_size=7))
def test_fleet_properties(nodes):
    reps = {f"n{i}": _node_report(f"n{i}", fr) for i, fr in enumerate(nodes)}
    names = list(reps)
    summary, views = F.judge_fleet(names, [reps[n] for n in names])
    assert len(views) == len(names)
    if len(names) < F.FLEET_MIN_NODES:
        assert summary == {} and views == [None] * len(names)
    for n, view in zip(names, views):
        alone = H.evaluate_report(reps[n], 0)
        v = H.evaluate_report(reps[n], 0, fleet=view)
        # the fleet never adds a failure and never removes one
        assert v.reasons == alone.reasons
        if view is None:
            assert (v.state, v.warnings) == (alone.state, alone.warnings)
            continue
        # it only excuses when the fleet's median is itself short
        if view["explained"]:
            row = summary["gemm@[4096, 4096, 4096]/tflops"]
            assert row["platform_shortfall"] and row["median_fraction"] <= P.DEGRADED_FRACTION  # rounded
        for f in view["findings"]:
            assert f["ratio"] <= F.FLEET_FAIL_RATIO  # rounded to 3 places
        # every warning the fleet added is a fleet finding
        added = [w for w in v.warnings if w not in alone.warnings]
        assert all(w.startswith("fleet: ") for w in added)


def test_watcher_with_reeval_serves_fleet_gauges_that_follow_events(reports, mock_cluster, tmp_path):
    """deploy/watcher.yaml plus --health-reeval: the fleet gauges on /metrics, and a node that falls behind the
    fleet after a watch event shows up as an outlier."""
    import os
    import socket
    import subprocess
    import sys
    import time

    from k8s_gpu_node_checker_amd.utils.http import request
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    reps = reports({f"n{i}": 1.0 for i in range(4)})
    srv, kc = _cluster(mock_cluster, tmp_path, reps)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("SLACK_WEBHOOK_URL", "KUBECONFIG")}
    p = subprocess.Popen([sys.executable, os.path.join(repo, "check-gpu-node.py"), "--kubeconfig", kc, "--json",
                          "--mi355x", "--health-reeval", "--watch-events", "--watch-duration", "30",
                          "--watch-debounce", "0.1", "--metrics-listen", f"127.0.0.1:{port}"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, cwd=str(tmp_path))
    gauge = 'k8s_gpu_checker_diag_fleet_outlier_nodes{test="gemm@[4096, 4096, 4096]/tflops"}'

    def outliers():
        try:
            text = request(f"http://127.0.0.1:{port}/metrics").text
        except Exception:  # not listening yet
            return None
        line = next((ln for ln in text.splitlines() if ln.startswith(gauge)), None)
        return float(line.split()[-1]) if line else None
    try:
        t0 = time.monotonic()
        while time.monotonic() - t0 < 20 and outliers() is None:
            time.sleep(0.1)
        assert outliers() == 0
        slow = reports({"n3": 0.70})["n3"]
        nodes = [fixtures.realistic_node(name, gpu_count=8, index=i,
                                         annotations=fixtures.health_annotation(slow if name == "n3" else rep),
                                         extra_conditions=[fixtures.health_condition(slow if name == "n3" else rep, 8)])
                 for i, (name, rep) in enumerate(reps.items())]
        srv.state.set_nodes(nodes)
        t0 = time.monotonic()
        while time.monotonic() - t0 < 20 and outliers() != 1:
            time.sleep(0.1)
        assert outliers() == 1
    finally:
        p.terminate()
        p.communicate(timeout=20)


_json = st.recursive(st.none() | st.booleans() | st.integers(-5, 5) | st.floats(allow_nan=True) | st.text(max_size=3),
                     lambda kids: st.lists(kids, max_size=3) | st.dictionaries(st.text(max_size=4), kids, max_size=3),
                     max_leaves=12)
_result = st.fixed_dictionaries({}, optional={
    "rates": st.dictionaries(st.sampled_from(["tflops", "read_tbs", "x"]), _json | st.floats(0.1, 2.0), max_size=2),
    "expect": st.dictionaries(st.sampled_from(["tflops", "read_tbs", "x"]), _json | st.just(1.0), max_size=2),
    "shape": _json, "pass": _json, "degraded": _json, "lag": _json, "drift": _json, "detail": _json})


@settings(max_examples=200, deadline=None)
@given(st.lists(st.lists(st.dictionaries(st.sampled_from(["gemm", "hbm", "mfma"]), _result | _json, max_size=3)
                         | _json, max_size=3), min_size=3, max_size=5),
       st.lists(_json, max_size=2))
def test_hostile_reports_do_not_break_the_fleet(gpu_diags, node_findings):
    """Reports are untrusted JSON: whatever their diagnostics hold, the fleet judgement neither raises nor turns a
    verdict into anything but a verdict."""
    reps = []
    for i, diags in enumerate(gpu_diags):
        r = fixtures.mi355x_probe_report(f"n{i}", gpus=max(1, len(diags)) if isinstance(diags, list) else 1)
        for g, d in zip(r["gpus"], diags if isinstance(diags, list) else [diags]):
            g["diag"] = d
        r["diag_node"] = {"findings": node_findings}
        reps.append(r)
    summary, views = F.judge_fleet([f"n{i}" for i in range(len(reps))], reps)
    for r, v in zip(reps, views):
        assert H.evaluate_report(r, 0, fleet=v).state in (H.HEALTHY, H.DEGRADED, H.UNHEALTHY, H.UNKNOWN)


def test_a_node_whose_fabric_runs_behind_the_fleet(reports):
    """Level-2 fabric results are node-level raw rates (GB/s): compared across nodes for outliers only -- a node
    whose RCCL all-reduce busbw is 60 % of the others' is degraded; a fabric the whole fleet shares is no
    shortfall (there is no reference to be short of)."""
    def rep(name, busbw, p2p):
        r = fixtures.mi355x_probe_report(name, gpus=8)
        r["fabric"] = {"rccl": {"pass": True, "world": 8, "best_busbw_gbps": busbw, "detail": ""},
                       "p2p": {"pass": True, "pairs": [[0, 1]] * 56, "median_gbps": p2p, "detail": ""}}
        return r
    reps = {"n0": rep("n0", 310.0, 48.0), "n1": rep("n1", 300.0, 47.0), "n2": rep("n2", 305.0, 49.0),
            "weak": rep("weak", 183.0, 47.5)}
    summary, verdicts = _judge(reps)
    assert all(verdicts[n].state == H.HEALTHY for n in ("n0", "n1", "n2"))
    w = verdicts["weak"]
    assert w.state == H.DEGRADED and w.warnings == [
        "fleet: rccl busbw_gbps at 60% of the other 3 nodes' median (183.0 vs 305.0): this node's xGMI fabric"]
    row = summary["rccl@world=8/busbw_gbps"]
    assert row["unit"] == "GB/s" and not row["platform_shortfall"] and row["outliers"] == [{"node": "weak", "ratio": 0.6}]
    assert summary["xgmi_p2p@pairs=56/median_gbps"]["outliers"] == []


@settings(max_examples=200, deadline=None)
@given(st.dictionaries(st.integers(0, 50), st.floats(0.01, 2.0) | st.sampled_from([0.5, 1.0]), min_size=2,
                       max_size=40))
def test_leave_one_out_medians_match_the_definition(vals):
    import statistics
    loo = F._loo_medians(vals)
    for i in vals:
        assert loo[i] == pytest.approx(statistics.median([x for j, x in vals.items() if j != i]), abs=1e-12)


def test_node_fractions_are_cached_per_node_object(reports, monkeypatch):
    """The watcher re-judges the fleet on every event: a node object computes its fractions once."""
    from k8s_gpu_node_checker_amd.models.node import NodeExtras
    rep = reports({"n0": 0.9})["n0"]
    ex = NodeExtras(True, {"amd.com/gpu": 8}, {"amd.com/gpu": 8}, False,
                    next(iter(fixtures.health_annotation(rep).values())))
    calls = []
    real = F.node_fractions
    monkeypatch.setattr(F, "node_fractions", lambda r: calls.append(1) or real(r))
    first = ex.fleet_fractions()
    assert ex.fleet_fractions() is first and len(calls) == 1
    assert first == real(ex.report()) and first[("gemm", "[4096, 4096, 4096]", "tflops")] == pytest.approx(0.9)


def test_other_gpu_models_are_compared_with_their_own_kind(reports):
    """An MI350X node (another device id) is not an outlier of an MI355X fleet: each model is its own fleet."""
    reps = reports({"n0": 1.0, "n1": 1.0, "n2": 1.0, "m0": 0.80, "m1": 0.80, "m2": 0.80})
    for n in ("m0", "m1", "m2"):
        for g in reps[n]["gpus"]:
            g["device_id"] = "0x75a0"
    summary, verdicts = _judge(reps)
    assert summary["gemm@[4096, 4096, 4096]/tflops"]["outliers"] == []
    assert summary["gemm@[4096, 4096, 4096] on 0x75a0/tflops"]["nodes"] == 3
    assert not any(w.startswith("fleet: ") for v in verdicts.values() for w in v.warnings)
    assert F._shape({"shape": [1, 2, 3]}) == "[1, 2, 3]" and F._shape({}, None) == ""
