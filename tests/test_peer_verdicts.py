"""Peer-relative and self-baselined diagnostic verdicts (models/peers.py, models/baseline.py) through whole agent
cycles on the fake C ABI of libmi355x_diag.so (testing/fake_native.py).

The reference's verdict is a stable binary read off the node (/root/reference/check-gpu-node.py:172-178); here
a node's GPUs are judged against each other, so a platform slower than the box the absolute references were
measured on is one node-level warning, while one GPU slower than its peers still fails, by name.
"""
import json

import pytest

from k8s_gpu_node_checker_amd.agent import agent as A
from k8s_gpu_node_checker_amd.models import baseline as B
from k8s_gpu_node_checker_amd.models import health as H
from k8s_gpu_node_checker_amd.models import peers as P
from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag, fabric
from k8s_gpu_node_checker_amd.testing import fixtures
from k8s_gpu_node_checker_amd.testing.fake_native import FakeDiagLib, FakeFabricLib

RATE_TESTS = ("gemm", "gemm_fp8", "hbm", "hbm_xcd", "mfma", "l2")


@pytest.fixture
def node(monkeypatch):
    """``node(n, **FakeDiagLib kwargs)`` -> the fake library of an n x MI355X node (all idle)."""
    def install(n=8, **kw):
        lib = FakeDiagLib(n=n, **kw)
        monkeypatch.setattr(diag, "lib", lambda: lib)
        monkeypatch.setattr(fabric, "_lib", FakeFabricLib())
        monkeypatch.setattr(amdsmi_probe, "probe", lambda nd, src, fx: fixtures.mi355x_probe_report(nd, gpus=n))
        return lib
    return install


def _agent(n, level=1, **kw):
    return A.Agent("n", source="fake", diag_level=level, expect_gpus=n, diag_timeout=60, **kw)


def test_eight_gpus_alike_at_088_are_one_node_level_warning(node):
    node(8, rate=0.88)
    rep = _agent(8).probe_once()
    v = H.evaluate_report(rep, 8)
    assert rep["state"] == v.state == H.DEGRADED and v.reasons == []
    assert (v.gpus_ok, v.gpus_seen) == (8, 8)
    # no GPU is singled out: every per-GPU rate test passed, not degraded, judged against its peers
    for g in rep["gpus"]:
        for t in RATE_TESTS:
            r = g["diag"][t]
            assert r["pass"] and not r.get("degraded") and r["peers"]["gpus"] == 8, (g["index"], t, r)
    node_warn = [w for w in v.warnings if w.startswith("node-wide: ")]
    assert node_warn and not [w for w in v.warnings if not w.startswith("node-wide: ")], v.warnings
    assert any("diag gemm tflops at 88% of the MI355X reference on all 8 GPUs alike" in w for w in node_warn)
    assert {f["test"] for f in rep["diag_node"]["findings"]} >= {"gemm", "gemm_fp8", "hbm", "mfma", "l2"}


@pytest.mark.parametrize("rate", [0.70, 0.5, 0.3])
def test_a_node_wide_shortfall_under_the_floor_fails_every_gpu(node, rate):
    """GPUs alike do not excuse each other below the absolute failure line -- a node whose 8
    GPUs all run at half rate is unhealthy, not one node-level note."""
    node(8, rate=rate)
    rep = _agent(8).probe_once()
    v = H.evaluate_report(rep, 8)
    assert v.state == H.UNHEALTHY and (v.gpus_ok, v.gpus_seen) == (0, 8)
    assert {r.split(":")[0] for r in v.reasons} == {f"gpu{d}" for d in range(8)}
    assert any(r.startswith("gpu0: diag gemm failed (tflops") for r in v.reasons), v.reasons
    assert all(f["below_floor"] for f in rep["diag_node"]["findings"])
    assert H.condition_for(v)["status"] == "False"


def test_a_node_wide_shortfall_between_the_lines_stays_a_warning(node):
    node(8, rate=0.86)
    v = H.evaluate_report(_agent(8).probe_once(), 8)
    assert v.state == H.DEGRADED and not v.reasons
    assert H.condition_for(v)["status"] == "True"  # degraded still counts as Ready


def test_one_gpu_at_080_of_its_peers_is_unhealthy_by_name(node):
    node(8, gpu_rate={3: 0.80})
    rep = _agent(8).probe_once()
    v = H.evaluate_report(rep, 8)
    assert v.state == H.UNHEALTHY and (v.gpus_ok, v.gpus_seen) == (7, 8)
    assert v.reasons and all(r.startswith("gpu3: diag ") for r in v.reasons), v.reasons
    gemm = next(r for r in v.reasons if r.startswith("gpu3: diag gemm failed"))
    assert "80% of the node's other GPUs' median" in gemm
    assert "diag_node" not in rep  # the other seven are at the reference
    assert all(g["diag"]["gemm"]["pass"] for g in rep["gpus"] if g["index"] != 3)


def test_a_gpu_at_the_reference_next_to_fast_peers_is_degraded_not_failed(node):
    """Seven GPUs at 1.15 of the references and gpu2 at 0.96: gpu2 is at 83 % of its peers but at the MI355X
    reference itself -- healthy devices differ this much (profiles/diag_box_spread_r05_mi355x.jsonl) -- so it is
    degraded with the ratio in the detail, never unhealthy."""
    node(8, rate=1.15, gpu_rate={2: 0.96})
    rep = _agent(8).probe_once()
    v = H.evaluate_report(rep, 8)
    assert v.state == H.DEGRADED and not v.reasons and (v.gpus_ok, v.gpus_seen) == (8, 8)
    g2 = next(g for g in rep["gpus"] if g["index"] == 2)["diag"]["gemm"]
    assert g2["pass"] and g2["degraded"] and "itself at 96% of the MI355X reference" in g2["detail"], g2
    assert g2["peers"]["ratio"]["tflops"] == pytest.approx(0.96 / 1.15, abs=0.01)


def test_one_gpu_behind_peers_on_a_slow_platform_still_fails(node):
    """Peers at 0.90 of the references, gpu5 at 0.72: gpu5 fails (80 % of its peers) while the other seven
    share one node-level warning -- the slow platform excuses the node, not the outlier."""
    node(8, rate=0.90, gpu_rate={5: 0.72})
    rep = _agent(8).probe_once()
    v = H.evaluate_report(rep, 8)
    assert v.state == H.UNHEALTHY and all(r.startswith("gpu5: ") for r in v.reasons)
    assert any(w.startswith("node-wide: diag gemm tflops at 90%") for w in v.warnings)


def test_a_majority_of_slow_gpus_falls_back_to_the_references(node):
    """Five of eight at half rate: no clear outlier (the slow GPUs are each other's peers) and the GPUs
    disagree, so each is judged absolutely -- the five fail, the three at the reference pass."""
    node(8, gpu_rate={d: 0.5 for d in range(5)})
    rep = _agent(8).probe_once()
    v = H.evaluate_report(rep, 8)
    assert v.state == H.UNHEALTHY and (v.gpus_ok, v.gpus_seen) == (3, 8)
    assert {r.split(":")[0] for r in v.reasons} == {f"gpu{d}" for d in range(5)}
    assert "diag_node" not in rep


def test_a_lone_gpu_is_judged_as_before(node):
    node(1, rate=0.88)
    rep = _agent(1).probe_once()
    v = H.evaluate_report(rep, 1)
    assert v.state == H.DEGRADED and "diag_node" not in rep
    assert any(w.startswith("gpu0: diag gemm slow (tflops") for w in v.warnings)
    assert "peers" not in rep["gpus"][0]["diag"]["gemm"]
    node(1, rate=0.80)
    v = H.evaluate_report(_agent(1).probe_once(), 1)
    assert v.state == H.UNHEALTHY and any(r.startswith("gpu0: diag gemm failed (tflops") for r in v.reasons)


def test_two_gpus_the_slower_is_the_outlier(node):
    node(2, gpu_rate={1: 0.80})
    rep = _agent(2).probe_once()
    v = H.evaluate_report(rep, 2)
    assert v.state == H.UNHEALTHY and all(r.startswith("gpu1: ") for r in v.reasons)


def test_numerics_failures_are_not_excused_by_peers(node):
    node(8, rate=0.88, gemm_bad_tiles={(2, "gemm"): {4: 1}})
    rep = _agent(8).probe_once()
    v = H.evaluate_report(rep, 8)
    assert v.state == H.UNHEALTHY
    assert [r.split(" (")[0] for r in v.reasons] == ["gpu2: diag gemm failed"]
    assert "checksums" in v.reasons[0]


def test_judgement_is_idempotent_and_recovers_when_peers_leave():
    """judge_node re-derives every verdict from the raw fields: judging twice changes nothing, and a result
    left without peers goes back to the absolute references."""
    def res(frac):
        return diag._rated({}, {"tflops": 1228.0 * frac}, {"tflops": 1228.0}, "TFLOP/s")
    pool = {d: {"gemm": res(0.88)} for d in range(4)}
    f1 = P.judge_node(pool)
    snap = json.dumps(pool, sort_keys=True)
    f2 = P.judge_node(pool)
    assert f1 == f2 and json.dumps(pool, sort_keys=True) == snap
    assert all(r["gemm"]["pass"] and not r["gemm"]["degraded"] for r in pool.values())
    lone = {0: pool[0]}
    assert P.judge_node(lone) == []
    assert lone[0]["gemm"]["degraded"] and "peers" not in lone[0]["gemm"]


def test_peer_ratios_compare_partitions_by_their_own_references():
    """A CPX partition (1/8 of the CUs, 1/8 the reference) next to a full GPU of the same node: compared as
    fractions of their own scaled references, both at 100 %."""
    full = diag._rated({}, {"tflops": 1228.0}, {"tflops": 1228.0}, "TFLOP/s")
    part = diag._rated({}, {"tflops": 153.5}, {"tflops": 153.5}, "TFLOP/s")
    P.judge_node({0: {"gemm": full}, 1: {"gemm": part}})
    assert full["pass"] and part["pass"] and part["peers"]["ratio"]["tflops"] == 1.0


def test_mi355x_diag_cli_judges_devices_together(node, capsys):
    node(4, rate=0.88)
    assert diag.main(["--level", "1"]) == 0
    out = json.loads(capsys.readouterr().out)
    assert out["pass"] and out["node"]["findings"]
    assert all(t["pass"] and not t.get("degraded") for d in out["devices"].values() for t in d["tests"].values())
    node(4, gpu_rate={2: 0.8})
    assert diag.main(["--level", "1", "--format", "text"]) == 1
    text = capsys.readouterr().out
    assert "of the node's other GPUs' median" in text and "result: FAIL" in text
    assert "(x0.80 vs the other 3 GPUs)" in text and "(x1.00 vs the other 3 GPUs)" in text


# --- self-baselines ----------------------------------------------------------------------------------------

def test_baseline_forms_from_clean_runs_then_flags_drift(node, tmp_path):
    """A fast node (1.10 of the references) forms each GPU's baseline over its first 5 clean cycles; when
    every GPU then drops to 0.96 -- above the references, alike across the node, so neither the absolute nor
    the peer judgement objects -- each GPU is degraded for drifting to 87 % of its own baseline."""
    lib = node(4, rate=1.10)
    path = tmp_path / "baseline.json"
    ag = _agent(4, diag_interval=0.0, baseline_file=str(path))
    for _ in range(B.BASELINE_RUNS):
        rep = ag.probe_once()
        assert rep["state"] == H.HEALTHY
    doc = json.loads(path.read_text())
    assert doc["schema"] == B.SCHEMA and len(doc["gpus"]) == 4
    entry = next(iter(doc["gpus"].values()))
    assert entry["tests"]["gemm@[4096,4096,4096]"]["baseline"]["tflops"] == pytest.approx(1.10, rel=1e-3)
    assert entry["epoch"].startswith("driver 6.18.54; vbios 00175784; fw ")
    lib.rate = 0.96
    rep = ag.probe_once()
    v = H.evaluate_report(rep, 4)
    assert v.state == H.DEGRADED and not v.reasons and "diag_node" not in rep
    drift = [w for w in v.warnings if "of this GPU's own baseline" in w]
    assert {w.split(":")[0] for w in drift} == {f"gpu{d}" for d in range(4)}
    assert any("gpu0: diag gemm slow (tflops at 87% of this GPU's own baseline (5 clean runs))" in w for w in drift)
    # a restarted agent keeps the baselines (the file), so the drift is still seen
    ag2 = _agent(4, diag_interval=0.0, baseline_file=str(path))
    assert H.evaluate_report(ag2.probe_once(), 4).state == H.DEGRADED
    # back to its own normal: clean again
    lib.rate = 1.10
    assert ag2.probe_once()["state"] == H.HEALTHY


def test_unclean_runs_do_not_enter_the_baseline(node):
    lib = node(2, rate=1.0, gpu_rate={1: 0.5})
    ag = _agent(2, diag_interval=0.0)
    for _ in range(B.BASELINE_RUNS):
        ag.probe_once()
    keys = {d: A.baseline_key(g, "", d) for d, g in enumerate(fixtures.mi355x_probe_report("n", gpus=2)["gpus"])}
    assert ag.baselines.baseline(keys[0], "gemm", {"shape": [4096, 4096, 4096]}) is not None
    assert ag.baselines.baseline(keys[1], "gemm", {"shape": [4096, 4096, 4096]}) is None  # failed every run


def test_baselines_can_be_turned_off(node):
    node(2)
    ag = _agent(2, diag_baseline=False)
    assert ag.probe_once()["state"] == H.HEALTHY and ag.baselines is None
    args = A.build_parser().parse_args(["--node", "n", "--no-diag-baseline", "--diag-baseline-file", "/x"])
    assert args.diag_baseline is False and args.diag_baseline_file == "/x"


def test_unreadable_baseline_file_starts_empty(tmp_path):
    p = tmp_path / "b.json"
    p.write_text("{not json")
    b = B.Baselines(str(p))
    assert b.data == {}
    p.write_text(json.dumps({"schema": "other", "gpus": {"x": {}}}))
    assert B.Baselines(str(p)).data == {}


def test_malformed_baseline_entries_are_rebuilt_not_fatal(tmp_path):
    p = tmp_path / "b.json"
    res = lambda: {"pass": True, "rates": {"tflops": 1000.0}, "expect": {"tflops": 1000.0},  # noqa: E731
                   "shape": [1, 1, 1]}
    from k8s_gpu_node_checker_amd.ops.diag import rate_revision
    rev = rate_revision("gemm")
    p.write_text(json.dumps({"schema": B.SCHEMA, "gpus": {
        "a": {"epoch": None, "tests": {"gemm@[1,1,1]": ["not", "a", "dict"]}},
        "b": {"epoch": None, "tests": {"gemm@[1,1,1]": {"samples": "junk", "rev": rev}}},
        "c": {"epoch": None, "tests": {"gemm@[1,1,1]": {"samples": [1, {"tflops": 1.0}], "rev": rev}}},
        "d": {"epoch": None, "tests": {"gemm@[1,1,1]": {"baseline": {"tflops": 0}, "runs": 5, "rev": rev}}}}}))
    b = B.Baselines(str(p), runs=2)
    for gpu in "abcd":
        assert b.observe(gpu, {"gemm": res()}) == []
    assert b.baseline("c", "gemm", res()) == {"tflops": 1.0}  # the one well-formed sample + this run
    assert b.baseline("a", "gemm", res()) is None and b.baseline("b", "gemm", res()) is None


# --- property tests --------------------------------------------------------------------------------------------

from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

_fracs = st.floats(min_value=0.05, max_value=1.6, allow_nan=False)


@settings(max_examples=300, deadline=None)
@given(st.lists(_fracs, min_size=1, max_size=12), st.booleans())
def test_peer_judgement_properties(fracs, numerics_bad):
    """For any node: judging twice changes nothing; a GPU failing numerics always fails; a lone GPU gets the
    absolute verdict; a node-wide finding is reported only when no GPU of that metric was failed by the floor;
    a GPU at or above its peers' median, or at or above the absolute degraded line, is never failed on rate."""
    def res(f, bad=False):
        return diag._rated({}, {"tflops": 1228.0 * f}, {"tflops": 1228.0}, "TFLOP/s", not bad, "wrong" if bad else "")
    pool = {d: {"gemm": res(f, numerics_bad and d == 0)} for d, f in enumerate(fracs)}
    f1 = P.judge_node(pool)
    snap = json.dumps(pool, sort_keys=True)
    assert P.judge_node(pool) == f1 and json.dumps(pool, sort_keys=True) == snap
    if numerics_bad:
        assert pool[0]["gemm"]["pass"] is False
    if len(fracs) == 1:
        expect = diag.judge_rate(1228.0 * fracs[0], 1228.0)
        r = pool[0]["gemm"]
        assert (r["pass"], r["degraded"]) == ((False, False) if numerics_bad or expect == "fail" else
                                              (True, expect == "degraded"))
        return
    import statistics as S
    for d, f in enumerate(fracs):
        others = S.median([x for j, x in enumerate(fracs) if j != d])
        r = pool[d]["gemm"]
        if f >= others and not (numerics_bad and d == 0):
            assert r["pass"] or f < P.FAIL_FRACTION, (fracs, d, r)
        if f >= P.DEGRADED_FRACTION and not (numerics_bad and d == 0):
            assert r["pass"], (fracs, d, r)  # at the reference: never failed on rate, whatever the peers
    for f in f1:
        assert f["test"] == "gemm" and f["median_fraction"] < P.DEGRADED_FRACTION
        assert f["max_fraction"] <= P.NODE_UNIFORM_SPREAD * f["min_fraction"] + 1e-9


_json = st.recursive(st.none() | st.booleans() | st.integers() | st.text(max_size=8),
                     lambda k: st.lists(k, max_size=4) | st.dictionaries(st.text(max_size=8), k, max_size=4),
                     max_leaves=12)


@settings(max_examples=300, deadline=None)
@given(st.lists(st.dictionaries(st.sampled_from(["endpoints", "metadata", "x"]), _json | st.lists(
    st.dictionaries(st.sampled_from(["addresses", "nodeName", "conditions"]), _json), max_size=4)), max_size=4))
def test_agent_addresses_never_raises_on_untrusted_slices(slices):
    from k8s_gpu_node_checker_amd.parallel import fanout
    out = fanout.agent_addresses(slices)
    assert all(isinstance(k, str) and isinstance(v, str) and k and v for k, v in out.items())


def test_agent_metrics_carry_peer_ratios_and_node_wide_findings(node):
    from prometheus_client.parser import text_string_to_metric_families
    node(8, rate=0.88, gpu_rate={3: 0.70})
    rep = _agent(8).probe_once()
    fams = {f.name: f for f in text_string_to_metric_families(A._metrics(rep))}
    ratios = {(s.labels["gpu"], s.labels["test"], s.labels["metric"]): s.value
              for s in fams["mi355x_gpu_diag_peer_ratio"].samples}
    assert ratios[("3", "gemm", "tflops")] == pytest.approx(0.70 / 0.88, abs=0.01)
    assert ratios[("0", "gemm", "tflops")] == pytest.approx(1.0, abs=0.01)
    short = {(s.labels["test"], s.labels["metric"]): s.value for s in fams["mi355x_node_diag_shortfall_fraction"].samples}
    assert short[("gemm", "tflops")] == pytest.approx(0.88, abs=0.01)


def test_status_table_shows_each_gpus_lowest_ratio_to_its_peers(node):
    from k8s_gpu_node_checker_amd.explain import report_text
    node(4, gpu_rate={2: 0.80})
    ag = _agent(4)
    rep = ag.probe_once()
    text = report_text(rep, ag.evaluate(rep))
    head = next(ln for ln in text.splitlines() if "vs peers" in ln)
    row2 = next(ln for ln in text.splitlines() if ln.strip().startswith("2 "))
    row0 = next(ln for ln in text.splitlines() if ln.strip().startswith("0 "))
    assert "x0.80" in row2 and "fail:" in row2 and "x1.00" in row0
    assert head.index("vs peers") < head.index("findings")


def test_status_table_shows_each_gpus_lowest_ratio_to_its_own_baseline(node):
    from k8s_gpu_node_checker_amd.explain import report_text
    lib = node(2, rate=1.10)
    ag = _agent(2, diag_interval=0.0)
    for _ in range(B.BASELINE_RUNS):
        ag.probe_once()
    lib.rate = 0.96
    rep = ag.probe_once()
    text = report_text(rep, ag.evaluate(rep))
    head = next(ln for ln in text.splitlines() if "vs own" in ln)
    row0 = next(ln for ln in text.splitlines() if ln.strip().startswith("0 "))
    assert head.index("vs peers") < head.index("vs own") < head.index("findings")
    assert "x0.87" in row0 and "own baseline" in row0


# --- baseline epochs and clean runs -------------------------------------------------

def _fw(node_fixture, **over):
    """Swap amd-smi's report for one with other driver / firmware fields."""
    def probe(nd, src, fx, _n=node_fixture):
        rep = fixtures.mi355x_probe_report(nd, gpus=_n)
        rep["driver"].update(over.get("driver", {}))
        for g in rep["gpus"]:
            g["fw"].update(over.get("fw", {}))
        return rep
    return probe


def test_a_driver_change_re_forms_the_baseline_without_drift(node, monkeypatch, tmp_path):
    lib = node(2, rate=1.10)
    path = tmp_path / "b.json"
    ag = _agent(2, diag_interval=0.0, baseline_file=str(path))
    for _ in range(B.BASELINE_RUNS):
        ag.probe_once()
    # the upgrade makes every GPU 12 % slower: under the old baseline that would be drift on every GPU forever
    monkeypatch.setattr(amdsmi_probe, "probe", _fw(2, driver={"version": "6.19.2"}))
    lib.rate = 0.97
    for _ in range(B.BASELINE_RUNS):
        rep = ag.probe_once()
        assert rep["state"] == H.HEALTHY, H.evaluate_report(rep, 2).warnings
        assert not any("own baseline" in w for w in H.evaluate_report(rep, 2).warnings)
    doc = json.loads(path.read_text())
    per = next(iter(doc["gpus"].values()))
    assert per["epoch"].startswith("driver 6.19.2;") and per["previous"]["epoch"].startswith("driver 6.18.54;")
    assert per["previous"]["baselines"]["gemm@[4096,4096,4096]"]["tflops"] == pytest.approx(1.10, rel=1e-3)
    assert per["tests"]["gemm@[4096,4096,4096]"]["baseline"]["tflops"] == pytest.approx(0.97, rel=1e-3)
    # drift is judged against the new software's normal: 0.86 is 89 % of 0.97
    lib.rate = 0.86
    rep = ag.probe_once()
    assert any("gemm slow (tflops at 89% of this GPU's own baseline" in w for w in H.evaluate_report(rep, 2).warnings)
    # a firmware flash is a new epoch too
    monkeypatch.setattr(amdsmi_probe, "probe", _fw(2, driver={"version": "6.19.2"}, fw={"pm": 72748907}))
    rep = ag.probe_once()
    assert not any("own baseline" in w for w in H.evaluate_report(rep, 2).warnings)
    gpu = next(iter(doc["gpus"]))
    assert "pm=04.86.15.107" in B.Baselines(str(path)).epoch(gpu)


def test_a_lone_gpu_at_093_forms_a_baseline_and_sees_a_drop_to_080_as_drift(node):
    lib = node(1, rate=0.93)
    ag = _agent(1, diag_interval=0.0)
    for _ in range(B.BASELINE_RUNS):
        rep = ag.probe_once()
        assert rep["state"] == H.DEGRADED  # absolutely degraded (0.93 < 0.95), yet its runs are clean
    key = A.baseline_key(fixtures.mi355x_probe_report("n", gpus=1)["gpus"][0], "", 0)
    assert ag.baselines.baseline(key, "gemm", {"shape": [4096, 4096, 4096]})["tflops"] == pytest.approx(0.93, rel=1e-3)
    lib.rate = 0.80
    rep = ag.probe_once()
    gemm = rep["gpus"][0]["diag"]["gemm"]
    assert gemm["drift"] == ["tflops at 86% of this GPU's own baseline (5 clean runs)"]
    assert H.evaluate_report(rep, 1).state == H.UNHEALTHY  # and under the absolute floor: failed as well


def test_peer_excused_runs_under_the_floor_never_form_a_baseline():
    """clean is judged on the result's own numbers, whatever pass/degraded flags a peer or
    fleet judgement left on it."""
    b = B.Baselines(runs=2)
    res = lambda f, **kw: dict({"pass": True, "degraded": False, "rates": {"tflops": 1000.0 * f},  # noqa: E731
                                "expect": {"tflops": 1000.0}, "shape": [1, 1, 1]}, **kw)
    for _ in range(3):
        b.observe("g", {"gemm": res(0.6)})
    assert b.baseline("g", "gemm", res(0.6)) is None
    for _ in range(3):
        b.observe("g", {"gemm": res(1.0, numerics="checksum mismatch")})
        b.observe("g", {"gemm": res(1.0, lag=["xcd3 at 80%"])})
    assert b.baseline("g", "gemm", res(1.0)) is None
    b.observe("g", {"gemm": res(0.9, **{"pass": False, "degraded": True})})
    b.observe("g", {"gemm": res(0.9)})
    assert b.baseline("g", "gemm", res(0.9)) == {"tflops": 0.9}


def test_baselines_from_before_revisions_are_dropped_not_adopted(tmp_path):
    """a baseline is a fraction of the references of its day; v1 (no epoch) and v2 (no revision)
    entries were formed under references that may since have moved, so they re-form instead of silently shifting the
    drift line."""
    res = {"rates": {"tflops": 900.0}, "expect": {"tflops": 1000.0}, "shape": [1, 1, 1]}
    p = tmp_path / "b.json"
    p.write_text(json.dumps({"schema": B.SCHEMA_V1, "gpus": {"uuid:x": {
        "gemm@[1,1,1]": {"baseline": {"tflops": 1.0}, "runs": 5, "since": 1.0}}}}))
    assert B.Baselines(str(p)).data == {}
    p.write_text(json.dumps({"schema": B.SCHEMA_V2, "gpus": {"uuid:x": {"epoch": "driver 6.18.54", "tests": {
        "gemm@[1,1,1]": {"baseline": {"tflops": 1.0}, "runs": 5, "since": 1.0}}}}}))
    b = B.Baselines(str(p))
    assert b.data["uuid:x"]["tests"] == {} and b.epoch("uuid:x") == "driver 6.18.54"
    assert b.observe("uuid:x", {"gemm": dict(res)}, epoch="driver 6.18.54") == []  # forming again: no drift
    doc = json.loads(p.read_text())
    assert doc["schema"] == B.SCHEMA and doc["gpus"]["uuid:x"]["tests"]["gemm@[1,1,1]"]["samples"] == [{"tflops": 0.9}]


def test_a_reference_or_kernel_change_re_forms_that_test_only(tmp_path):
    """new REFERENCE_RATES (or a new kernel) for one test move its fractions; that test's
    baseline re-forms, the others keep theirs."""
    b = B.Baselines(runs=2)
    gemm = lambda f: {"rates": {"tflops": 1000.0 * f}, "expect": {"tflops": 1000.0}, "shape": [1, 1, 1]}  # noqa: E731
    hbm = lambda f: {"rates": {"read_tbs": 7.0 * f}, "expect": {"read_tbs": 7.0}, "gib": 2.0}  # noqa: E731
    revs = {"gemm": "r1", "hbm": "h1"}
    for _ in range(2):
        b.observe("g", {"gemm": gemm(1.0), "hbm": hbm(1.0)}, revision=revs.get)
    assert b.baseline("g", "gemm", gemm(1.0)) == {"tflops": 1.0}
    # the gemm references were raised 7.6 %: the same GPU now measures 0.93 of them -- not drift, a new yardstick
    revs["gemm"] = "r2"
    assert b.observe("g", {"gemm": gemm(0.85), "hbm": hbm(0.85)}, revision=revs.get) == [
        "hbm: read_tbs at 85% of this GPU's own baseline (2 clean runs)"]
    assert b.baseline("g", "gemm", gemm(1.0)) is None and b.baseline("g", "hbm", hbm(1.0)) == {"read_tbs": 1.0}
    b.observe("g", {"gemm": gemm(0.93)}, revision=revs.get)
    assert b.baseline("g", "gemm", gemm(1.0)) == {"tflops": 0.89}  # re-formed on the new references
    # the stamp the agent uses moves with REFERENCE_RATES and KERNEL_REVISION
    from k8s_gpu_node_checker_amd.ops import diag
    before = diag.rate_revision("gemm")
    old = dict(diag.REFERENCE_RATES["gemm"])
    try:
        diag.REFERENCE_RATES["gemm"][4096] += 1
        assert diag.rate_revision("gemm") != before and diag.rate_revision("hbm") == diag.rate_revision("hbm")
    finally:
        diag.REFERENCE_RATES["gemm"].clear()
        diag.REFERENCE_RATES["gemm"].update(old)
    assert diag.rate_revision("gemm") == before and set(diag.KERNEL_REVISION) >= {"gemm", "gemm_fp8", "hbm", "mfma"}


def test_a_transient_amd_smi_miss_is_not_a_new_epoch():
    """one probe without the VBIOS (or the driver) must neither wipe the baselines nor, when the
    field comes back, re-form them a second time; a component that does differ still re-forms."""
    b = B.Baselines(runs=1)
    res = lambda f: {"rates": {"tflops": 1000.0 * f}, "expect": {"tflops": 1000.0}, "shape": [1, 1, 1]}  # noqa: E731
    full = "driver 6.18.54; vbios 00175784; fw pm=1,sos=2"
    b.observe("g", {"gemm": res(1.0)}, epoch=full)
    for partial in ("driver 6.18.54; fw pm=1,sos=2", "vbios 00175784; fw pm=1,sos=2", "driver 6.18.54; vbios 00175784",
                    None, full):
        assert b.observe("g", {"gemm": res(0.8)}, epoch=partial) == [
            "gemm: tflops at 80% of this GPU's own baseline (1 clean runs)"], partial
        assert b.epoch("g") == full and "previous" not in b.data["g"]
    # a component first seen later is filled in, nothing re-forms
    b2 = B.Baselines(runs=1)
    b2.observe("g", {"gemm": res(1.0)}, epoch="fw pm=1")
    assert b2.observe("g", {"gemm": res(0.8)}, epoch="driver 6.18.54; fw pm=1")
    assert b2.epoch("g") == "driver 6.18.54; fw pm=1"
    # a real change of a known component re-forms
    b.observe("g", {"gemm": res(0.9)}, epoch="driver 6.19.2; fw pm=1,sos=2")
    assert b.data["g"]["previous"]["epoch"] == full and b.epoch("g") == "driver 6.19.2; fw pm=1,sos=2"
    assert B.epoch_parts(full) == {"driver": "6.18.54", "vbios": "00175784", "fw:pm": "1", "fw:sos": "2"}
    assert B.epoch_str(B.epoch_parts(full)) == full


def test_baselines_can_be_dropped_by_flag_and_by_a_loopback_post(node, tmp_path, monkeypatch):
    import urllib.error
    import urllib.request
    from k8s_gpu_node_checker_amd.agent.server import serve
    lib = node(2, rate=1.0)
    path = tmp_path / "b.json"
    ag = _agent(2, diag_interval=0.0, baseline_file=str(path))
    for _ in range(B.BASELINE_RUNS):
        ag.probe_once()
    keys = sorted(ag.baselines.data)
    assert len(keys) == 2
    srv = serve(ag, "127.0.0.1", 0)
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}/baseline/reset?gpu={keys[0].split(':', 1)[1]}"
        with urllib.request.urlopen(urllib.request.Request(url, method="POST", data=b""), timeout=5) as r:
            assert json.loads(r.read()) == {"dropped": [keys[0]]}
        assert sorted(ag.baselines.data) == keys[1:]
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(urllib.request.Request(url.replace("/baseline/reset", "/nope"), method="POST",
                                                          data=b""), timeout=5)
        assert e.value.code == 404
        # a malformed Content-Length is a 400, not a crashed handler
        import socket
        with socket.create_connection(("127.0.0.1", srv.server_address[1]), timeout=5) as c:
            c.sendall(b"POST /baseline/reset HTTP/1.1\r\nHost: x\r\nContent-Length: nope\r\n\r\n")
            assert c.recv(4096).startswith(b"HTTP/1.1 400 ")
        assert sorted(ag.baselines.data) == keys[1:]
    finally:
        srv.shutdown()
        srv.server_close()
    assert json.loads(path.read_text())["gpus"].keys() == set(keys[1:])
    b = B.Baselines(str(path))
    assert b.drop(["no-such-gpu"]) == [] and b.drop(None) == keys[1:]
    assert json.loads(path.read_text())["gpus"] == {}
    # the start-up flag (--once with the fixture source: no HIP, the file is read, reset and written back)
    path.write_text(json.dumps({"schema": B.SCHEMA, "gpus": {k: {"epoch": None, "tests": {}} for k in keys}}))
    fx = tmp_path / "fx.json"
    fx.write_text(json.dumps(fixtures.mi355x_probe_report("n", gpus=2)))
    assert A.main(["--node", "n", "--once", "--source", "fixture", "--fixture", str(fx), "--publish", "stdout",
                   "--diag-level", "0", "--diag-baseline-file", str(path), "--diag-baseline-reset", keys[1]]) in (0, 3)
    assert set(json.loads(path.read_text())["gpus"]) == {keys[0]}


def test_baseline_reset_is_refused_from_off_the_pod(node):
    """POST /baseline/reset answers only a loopback peer: the checker's fan-out or Prometheus cannot reset it."""
    import socket
    import urllib.error
    import urllib.request
    from k8s_gpu_node_checker_amd.agent.server import serve
    node(1)
    ag = _agent(1, diag_interval=0.0)
    ip = next((a[4][0] for a in socket.getaddrinfo(socket.gethostname(), None, socket.AF_INET)
               if not a[4][0].startswith("127.")), None)
    if ip is None:
        pytest.skip("no non-loopback address")
    srv = serve(ag, "0.0.0.0", 0)
    try:
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(urllib.request.Request(f"http://{ip}:{srv.server_address[1]}/baseline/reset",
                                                          method="POST", data=b""), timeout=5)
        assert e.value.code == 403
    finally:
        srv.shutdown()
        srv.server_close()


def test_a_shared_host_link_failure_is_held_once_before_it_fails_the_gpu(node):
    """The host-link test shares the PCIe path with the host's other GPUs and processes: its first rate-only
    failure is published degraded (and re-measured), the second in a row fails the GPU, failures stand until the
    test passes again, and a pass resets it.  Re-judging a cached result (every cycle) keeps the hold."""
    lib = node(1, link=(20.0, 20.0))  # a third of the Gen5 x16 reference both ways
    ag = _agent(1, level=2, diag_interval=0.0, diag_when="always")
    states = []
    for _ in range(3):
        rep = ag.probe_once()
        hl = rep["gpus"][0]["diag"]["host_link"]
        states.append((rep["state"], hl["pass"], bool(hl.get("degraded"))))
        if len(states) == 1:
            assert A.HELD_NOTE in hl["detail"] and "h2d_gbps" in hl["detail"], hl["detail"]
    assert states == [(H.DEGRADED, True, True), (H.UNHEALTHY, False, False), (H.UNHEALTHY, False, False)], states
    lib.link = None  # back at its reference
    rep = ag.probe_once()
    assert rep["state"] == H.HEALTHY and rep["gpus"][0]["diag"]["host_link"]["pass"]
    lib.link = (20.0, 20.0)  # a new dip: held again first
    rep = ag.probe_once()
    assert rep["state"] == H.DEGRADED and A.HELD_NOTE in rep["gpus"][0]["diag"]["host_link"]["detail"]
    # a held result re-judged later (diagnostics not due) is still published degraded
    ag.diag_interval = 3600.0
    rep = ag.probe_once()
    assert rep["state"] == H.DEGRADED and rep["gpus"][0]["diag"]["host_link"]["pass"]
