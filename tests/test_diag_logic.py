"""ops/diag.py verdict logic on CPU: a fake C ABI stands in for libmi355x_diag.so (the real kernels
run under tests/test_gpu.py on the MI355X)."""
import pytest

from k8s_gpu_node_checker_amd.ops import diag
from k8s_gpu_node_checker_amd.testing.fake_native import FakeDiagLib


FakeLib = FakeDiagLib  # the C ABI with scripted results (testing/fake_native.py)


@pytest.fixture
def fake(monkeypatch):
    def install(**kw):
        lib = FakeLib(**kw)
        monkeypatch.setattr(diag, "lib", lambda: lib)
        return lib
    return install


def test_mfma_burn_pass_and_each_failure_mode(fake):
    fake()
    r = diag.mfma_burn(0)
    assert r["pass"] and set(r["kinds"]) == {"bf16", "fp8", "mxfp8", "mxfp4"} and r["detail"] == ""
    fake(mfma={0: (1900.0, 0), 1: (4350.0, 0), 2: (4300.0, 3), 3: (7600.0, 0)})
    r = diag.mfma_burn(0)
    assert not r["pass"] and r["detail"] == "mxfp8: 3 wrong results"
    fake(mfma={0: (400.0, 0), 1: (4350.0, 0), 2: (4300.0, 0), 3: (7600.0, 0)})
    assert diag.mfma_burn(0)["detail"] == "bf16 400 TFLOP/s = 21% of 1.9e+03"


def test_host_link_threshold(fake):
    fake()
    assert diag.host_link(0)["pass"]
    fake(link=(24.0, 56.0))  # a Gen4 / x8 link: half rate one way
    r = diag.host_link(0)
    assert not r["pass"] and "h2d_gbps 24 GB/s" in r["detail"] and "d2h" not in r["detail"]


def test_c_abi_failure_raises_with_library_message(fake):
    fake(rc=-1, err=b"hipMalloc: out of memory")
    with pytest.raises(RuntimeError, match="out of memory"):
        diag.mfma_burn(0, kinds=("bf16",))


def test_run_turns_a_failing_test_into_a_verdict(fake, monkeypatch):
    fake()

    def broken(*a, **k):
        raise RuntimeError("mi355x diag failed (-1): hipMemcpy: illegal address")
    monkeypatch.setattr(diag, "gemm", broken)
    monkeypatch.setattr(diag, "gemm_fp8", lambda *a, **k: {"pass": True})
    monkeypatch.setattr(diag, "hbm", lambda *a, **k: {"pass": True})
    out = diag.run(1, 0)
    assert out["gemm"]["pass"] is False and "illegal address" in out["gemm"]["detail"]
    assert out["mfma"]["pass"] and out["hbm"]["pass"]


def _verdict(results, memory_partition="NPS1", cus=256):
    """The agent's verdict for one GPU whose diag results are ``results``."""
    from k8s_gpu_node_checker_amd.models import health as H
    from k8s_gpu_node_checker_amd.testing import fixtures
    rep = fixtures.mi355x_probe_report("n", gpus=1)
    rep["gpus"][0].update({"diag": results, "memory_partition": memory_partition, "cus": cus,
                           "compute_partition": "SPX" if cus == 256 else "CPX"})
    return H.evaluate_report(rep, 1, now=rep["ts"])


@pytest.mark.parametrize("level", [1, 2])
def test_full_rate_gpu_is_healthy(fake, level):
    lib = fake(link=(57.2, 56.8))
    out = diag.run(level, 0)
    assert all(r["pass"] and not r["degraded"] for r in out.values() if "fraction" in r), out
    assert "scale" not in out["gemm"] and out["gemm"]["fraction"] == 1.0
    assert "retried" not in out["gemm"] and lib.calls.count("gemm") == 1
    assert _verdict(out).state == "healthy"


def test_gpu_at_55_percent_is_unhealthy(fake):
    fake(rate=0.55, mfma={k: (0.55 * diag.REFERENCE_RATES["mfma"][n], 0) for k, n in enumerate(diag.MFMA_KINDS)})
    out = diag.run(1, 0)
    for t in ("gemm", "gemm_fp8", "hbm", "mfma"):
        assert out[t]["pass"] is False and out[t]["retried"] and 0.54 < out[t]["fraction"] < 0.56, out[t]
    assert "tflops 720 TFLOP/s = 55% of 1.31e+03" in out["gemm"]["detail"]
    v = _verdict(out)
    assert v.state == "unhealthy" and any("diag gemm failed" in r for r in v.reasons)


def test_gpu_at_90_percent_is_degraded_and_measured_three_times(fake):
    lib = fake(rate=0.90)
    out = diag.run(1, 0)
    assert out["gemm"]["pass"] and out["gemm"]["degraded"] and out["gemm"]["retried"]
    assert lib.calls.count("gemm") == 1 + diag.REMEASURE and lib.calls.count("hbm") == 1 + diag.REMEASURE
    v = _verdict(out)
    assert v.state == "degraded" and v.ok and any("diag gemm slow" in w for w in v.warnings), v.warnings


def test_one_slow_sample_is_remeasured_not_reported(fake):
    lib = fake(rates=[0.80, 1.0])  # the first gemm sample is slow, the re-measurement is normal
    out = diag.run(1, 0)
    assert out["gemm"]["pass"] and not out["gemm"]["degraded"] and out["gemm"]["retried"]
    assert out["gemm"]["fraction"] == 1.0 and lib.calls.count("gemm") == 2  # normal again: no third run


def test_two_slow_samples_then_a_normal_one(fake):
    lib = fake(rates=[0.90, 0.91, 1.0])
    out = diag.run(1, 0)
    assert out["gemm"]["pass"] and not out["gemm"]["degraded"] and lib.calls.count("gemm") == 3


def test_numerics_failure_is_not_remeasured(fake):
    lib = fake(gemm_err=5e-2)
    out = diag.run(1, 0)
    assert out["gemm"]["pass"] is False and out["gemm"]["detail"].startswith("rel err 5.00e-02")
    assert lib.calls.count("gemm") == 1


def test_gemm_tiles_failing_their_checksums_fail_the_gpu_and_name_the_xcd(fake):
    """Every GEMM output is covered by tile checksums: tiles that fail them fail the test (not measured again:
    a wrong result does not get better), the detail names the XCDs, and the agent's verdict is unhealthy."""
    lib = fake(gemm_bad_tiles={(0, "gemm_fp8"): {5: 2}})
    out = diag.run(1, 0)
    assert out["gemm"]["pass"] and out["gemm"]["checksum_bad_tiles"] == 0 and out["gemm"]["checksum_err"] < 1e-7
    r = out["gemm_fp8"]
    assert not r["pass"] and r["checksum_bad_tiles"] == 2 and r["checksum_bad_xcds"] == {"5": 2}, r
    assert r["detail"].startswith("2 output tile(s) fail their checksums (XCD 5: 2; first at tile row 0"), r
    assert lib.calls.count("gemm_fp8") == 1
    v = _verdict(out)
    assert v.state == "unhealthy" and any("diag gemm_fp8 failed" in x for x in v.reasons), v.reasons
    # the test hook: one injected output is one bad tile
    fake()
    r = diag.gemm(0, inject_elem=12345)
    assert not r["pass"] and r["checksum_bad_tiles"] == 1 and r["checksum_first_bad_tile"] == [0, 0]


def test_cpx_partition_at_one_eighth_is_healthy(fake):
    # CPX: 32 CUs, NPS1 (all of HBM addressable, an eighth of the bandwidth share); every rate 1/8
    lib = fake(rate=1 / 8, cus=32, link=(57.2 / 8, 56.8 / 8),
               mfma={k: (diag.REFERENCE_RATES["mfma"][n] / 8, 0) for k, n in enumerate(diag.MFMA_KINDS)})
    for level in (1, 2):
        out = diag.run(level, 0, memory_partition="NPS1")
        assert all(r["pass"] and not r.get("degraded") for r in out.values()), out
        assert out["gemm"]["scale"] == {"compute": 0.125, "memory": 0.125}
        assert _verdict(out, cus=32).state == "healthy"
    # and the same partition at 1/16 (half speed) fails
    lib.rate = 1 / 16
    out = diag.run(1, 0, memory_partition="NPS1")
    assert not out["gemm"]["pass"] and not out["hbm"]["pass"]


def test_scale_from_partition_modes():
    s = diag.Scale.of(256, 288 << 30, "NPS1")
    assert (s.compute, s.memory) == (1.0, 1.0)
    s = diag.Scale.of(128, 144 << 30, "NPS2")  # DPX + NPS2: half of everything
    assert (s.compute, s.memory) == (0.5, 0.5)
    s = diag.Scale.of(256, 288 << 30, "NPS2")  # SPX but an NPS2 memory partition: memory share halves
    assert (s.compute, s.memory) == (1.0, 0.5)
    assert diag.Scale.of(None, None, None).to_dict() == {"compute": 1.0, "memory": 1.0}
    assert diag.judge_rate(84.9, 100) == "fail" and diag.judge_rate(85, 100) == "degraded"
    assert diag.judge_rate(95, 100) == "pass"


def test_mfma_burn_maps_waves_to_cus_and_xcds(fake):
    fake()
    r = diag.mfma_burn(0)
    m = r["map"]
    assert m["cus"] == 256 and len(m["xcds"]) == 8 and all(x == {"cus": 32, "rel_time": 1.0} for x in m["xcds"].values())
    assert "bad_cus" not in m and r["pass"] and not r["degraded"]


def test_mfma_wrong_results_are_located_to_their_cu(fake):
    slot = (3 << 7) | (1 << 5) | 5
    fake(mfma_errors={(0, 0): 12, (0, 2): 2}, bad_cu={(0, 0): slot, (0, 2): slot})
    r = diag.mfma_burn(0)
    assert not r["pass"]
    assert r["map"]["bad_cus"] == ["xcd3/se1/cu5 (bf16 12, mxfp8 2)"]
    assert r["detail"] == "bf16: 12 wrong results; mxfp8: 2 wrong results; on xcd3/se1/cu5 (bf16 12, mxfp8 2)"
    assert diag.slot_name((7 << 7) | (3 << 5) | (1 << 4) | 15) == "xcd7/se3/cu15/sh1"


def test_a_lagging_xcd_degrades_the_burn_in(fake):
    fake(slow_xcd={6: 1.3})
    r = diag.mfma_burn(0)
    assert r["pass"] and r["degraded"]
    assert r["map"]["slowest_xcd"] == 6 and r["map"]["slowest_rel"] == 1.3
    assert r["detail"] == "xcd6 waves take 1.30x the median XCD's time"
    assert _verdict({"mfma": r}).state == "degraded"
    fake(slow_xcd={6: 1.1})  # inside the spread of a healthy chip
    r = diag.mfma_burn(0)
    assert r["pass"] and not r["degraded"] and r["map"]["slowest_rel"] == 1.1


def test_cpx_partition_has_one_xcd_and_no_xcd_verdict(fake):
    fake(cus=32, mfma={k: (diag.REFERENCE_RATES["mfma"][n] / 8, 0) for k, n in enumerate(diag.MFMA_KINDS)})
    r = diag.mfma_burn(0, scale=diag.Scale(0.125, 0.125))
    assert r["pass"] and not r["degraded"] and r["map"]["cus"] == 32 and "slowest_xcd" not in r["map"]


def test_a_lagging_xcd_is_measured_again(fake):
    lib = fake(slow_xcd={2: 1.4})
    out = diag.run(1, 0)
    assert lib.calls.count("mfma") == 4 * (1 + diag.REMEASURE)  # 4 kinds per measurement
    assert out["mfma"]["retried"] and out["mfma"]["degraded"]
    lib.slow_xcd = {}
    lib.calls.clear()
    out = diag.run(1, 0)
    assert lib.calls.count("mfma") == 4 and not out["mfma"].get("retried")


def test_lds_test_passes_on_every_cu_and_locates_bad_words(fake):
    fake()
    r = diag.lds_test(0)
    assert r["pass"] and r["errors"] == 0 and r["cus"] == 256 and r["bytes_per_cu"] == 163824
    assert r["workgroups"] == 256 * 4 and "bad_cus" not in r
    slot = (5 << 7) | (2 << 5) | 7
    fake(lds_bad={(0, slot): 3})
    r = diag.lds_test(0)
    assert not r["pass"] and r["bad_cus"] == ["xcd5/se2/cu7 (3 words)"]
    assert r["detail"] == "3 LDS words wrong on xcd5/se2/cu7 (3 words)"
    assert _verdict({"lds": r}).state == "unhealthy"


def test_lds_runs_at_both_levels(fake):
    lib = fake()
    for level in (1, 2):
        lib.calls.clear()
        out = diag.run(level, 0)
        assert out["lds"]["pass"] and lib.calls.count("lds") == 1


def test_l2_bandwidth_rate_xcd_lag_and_located_errors(fake):
    fake()
    r = diag.l2_bandwidth(0)
    assert r["pass"] and not r["degraded"] and r["map"]["cus"] == 256 and len(r["map"]["xcds"]) == 8
    fake(slow_xcd={3: 1.25})
    r = diag.l2_bandwidth(0)
    assert r["pass"] and r["degraded"] and r["detail"] == "xcd3 L2 reads take 1.25x the median XCD's time"
    fake(l2_bad={(0, (1 << 7) | 4): 2})
    r = diag.l2_bandwidth(0)
    assert not r["pass"] and r["detail"] == "2 wrong words on xcd1/se0/cu4 (l2 2)"
    fake(rate=0.5)
    r = diag.l2_bandwidth(0)
    assert not r["pass"] and r["detail"].startswith("read_tbs 15.2 TB/s = 50% of 30.5")
    # a CPX partition (one XCD): its share of the rate, no XCD comparison
    fake(cus=32, rate=1 / 8)
    r = diag.l2_bandwidth(0, scale=diag.Scale(0.125, 0.125))
    assert r["pass"] and not r["degraded"] and "slowest_xcd" not in r["map"]


def test_a_single_lagging_cu_degrades_the_burn_in(fake):
    slot = (6 << 7) | (1 << 5) | 3
    fake(slow_cu={slot: 1.4})
    r = diag.mfma_burn(0)
    m = r["map"]
    assert m["slowest_cu"] == "xcd6/se1/cu3" and m["slowest_cu_rel"] == 1.4 and m["waves_per_cu"] == [48, 48]
    # one CU of 32 barely moves its XCD's mean: only the per-CU comparison sees it
    assert m["slowest_rel"] < diag.XCD_SLOW_RATIO
    assert r["pass"] and r["degraded"] and r["detail"] == "xcd6/se1/cu3 waves take 1.40x its XCD's median CU's time"
    fake(slow_cu={slot: 1.05})
    assert not diag.mfma_burn(0)["degraded"]


def test_cu_lag_is_not_judged_on_an_uneven_deal():
    m = diag.cu_map_summary({"k": [0] * 3 * 1024})
    assert m["cus"] == 0
    flat = [0] * 3 * 1024
    for slot, (w, t) in {0: (8, 8000), 1: (8, 8100), 2: (16, 24000)}.items():  # slot 2 got twice the waves
        flat[3 * slot], flat[3 * slot + 2] = w, t
    where = diag.cu_map_summary({"k": flat})
    assert where["waves_per_cu"] == [8, 16] and where["slowest_cu_rel"] > 1.4
    assert diag._lag_notes(where, "waves") == []


def test_text_summary(fake, capsys):
    fake(slow_xcd={2: 1.3})
    rc = diag.main(["--level", "1", "--format", "text"])
    out = capsys.readouterr().out.splitlines()
    assert out[0].startswith("GPU 0  0000:05:00.0  AMD Instinct MI355X  gfx950  256 CUs  288 GiB")
    rows = {ln.split()[0]: ln for ln in out[1:] if ln.startswith("  ") and ln.split()}
    assert rows["gemm"].split()[1] == "pass" and "TFLOP/s" in rows["gemm"]
    assert rows["mfma"].split()[1] == "DEGRADED" and "XCD spread 1.300" in rows["mfma"]
    assert any("xcd2 waves take 1.30x" in ln for ln in out)
    assert rows["lds"].endswith("256 CUs x 159 KiB, 0 bad words")
    assert out[-1] == "result: PASS" and rc == 0  # degraded still passes


def test_hbm_per_xcd_alone_rates_find_one_slow_xcd(fake):
    lib = fake()
    r = diag.hbm_xcd(0)
    assert r["pass"] and not r["degraded"] and len(r["alone_tbs"]) == 8 and r["slowest_xcd_rel"] == 1.0
    assert r["expect"] == {"read_tbs": 5.8, "slowest_xcd_tbs": 1.28}
    # one XCD's path at 85 % of the others: the aggregate (HBM-bound) would not show it; alone it is 0.85x
    # the median XCD -> degraded, and measured again before it is reported
    lib = fake(hbm_xcd_slow={5: 0.97 * 0.85 / 0.97})
    out = diag.run(1, 0)
    r = out["hbm_xcd"]
    assert r["pass"] and r["degraded"] and r["slowest_xcd"] == 5 and r["retried"]
    assert "xcd5 reads HBM at 1.11 TB/s alone, 0.85x the median XCD" in r["detail"]
    assert lib.calls.count("hbm_xcd") == 1 + diag.REMEASURE
    # an XCD at half rate fails outright (below 85 % of the per-XCD reference)
    fake(hbm_xcd_slow={2: 0.5})
    r = diag.hbm_xcd(0)
    assert not r["pass"] and r["detail"].startswith("slowest_xcd_tbs 0.655 TB/s = 51% of 1.28")
    assert _verdict({"hbm_xcd": r}).state == "unhealthy"
    # wrong words are located to the CU that read them
    fake(hbm_bad={(0, (3 << 7) | (1 << 5) | 2): 4})
    r = diag.hbm_xcd(0)
    assert not r["pass"] and r["detail"] == "4 wrong words on xcd3/se1/cu2 (hbm_xcd 4)"
    # a CPX partition: one XCD, the partition's memory share of the aggregate
    fake(cus=32, rate=1 / 8)
    r = diag.hbm_xcd(0, scale=diag.Scale(0.125, 0.125))
    assert list(r["alone_tbs"]) == ["0"] and r["expect"]["read_tbs"] == 0.725


def test_no_device_is_a_failure_not_a_pass(fake, capsys):
    fake(n=0)
    assert diag.main(["--level", "1"]) == 1
    doc = __import__("json").loads(capsys.readouterr().out)
    assert doc["pass"] is False and "no HIP devices" in doc["error"]


def test_p2p_matrix_deadline_names_a_hung_pair_and_stops(fake):
    """A pair whose copies never complete comes back at the deadline as a failed, named pair (the native side
    polls its completion event) and ends the matrix; every pair gets only what is left of the budget."""
    lib = fake(n=3, hung_pairs=((1, 0),))
    m = diag.p2p_matrix([0, 1, 2], timeout_s=0.3)
    assert not m["pass"] and m["stopped"].startswith("1->0 hung: p2p 1->0: copies did not complete within")
    assert [f"{p['src']}->{p['dst']}" for p in m["pairs"]] == ["0->1", "0->2"]  # order: 0->1 0->2 1->0 ...
    assert "1->0 hung" in m["detail"]
    assert len(lib.p2p_timeouts_ms) == 3 and all(0 < t <= 300.0 for t in lib.p2p_timeouts_ms)
    assert lib.p2p_timeouts_ms[2] <= lib.p2p_timeouts_ms[0]
    assert 0.25 <= m["wall_s"] < 2.0


def test_p2p_matrix_deadline_between_pairs(fake):
    fake(n=3, p2p_wall_s=0.06)
    m = diag.p2p_matrix([0, 1, 2], timeout_s=0.1)
    assert not m["pass"] and m["stopped"].startswith("deadline of 0.1 s passed after 2/6 pairs")
    assert len(m["pairs"]) == 2 and m["min_gbps"] == 48.0


def test_p2p_matrix_without_a_deadline_blocks_and_with_one_passes(fake):
    lib = fake(n=2)
    m = diag.p2p_matrix([0, 1], timeout_s=5.0)
    assert m["pass"] and "stopped" not in m and len(m["pairs"]) == 2
    assert diag.p2p_matrix([0, 1])["pass"] and lib.p2p_timeouts_ms[-1] == 0.0  # no deadline: 0 to the ABI


def test_diag_cli_runs_devices_concurrently_like_the_agent(fake, capsys):
    import json
    import time
    lib = fake(n=4, delay_s=0.15)
    t0 = time.monotonic()
    assert diag.main(["--level", "1", "--parallel", "4"]) == 0
    wall = time.monotonic() - t0
    out = json.loads(capsys.readouterr().out)
    assert sorted(out["devices"], key=int) == ["0", "1", "2", "3"] and out["pass"]
    assert {d: lib.threads[d] for d in range(4)} == {d: {f"diag-gpu{d}"} for d in range(4)}
    assert wall < 4 * 2 * 0.15 * 0.7, wall  # 2 GEMMs of 0.15 s per device, overlapped
    lib2 = fake(n=2)
    assert diag.main(["--level", "1", "--parallel", "1"]) == 0
    assert all(len(t) == 1 for t in lib2.threads.values())


def test_burn_in_reports_spread_and_every_failing_round(fake, capsys):
    import json
    fake(n=2, rates=[1.0, 1.0, 0.98, 0.97] * 50)
    b = diag.burn_in(1, [0, 1], minutes=0.0005)
    assert b["pass"] and b["rounds"] >= 1 and not b["failures"]
    g = b["devices"][0]["gemm.tflops"]
    assert g["min"] <= g["median"] <= g["max"]
    assert "mfma.bf16.tflops" in b["devices"][1]
    # a GPU at half speed fails every round it runs, and the report names the rounds
    fake(n=2, gpu_rate={1: 0.5})
    b = diag.burn_in(1, [0, 1], minutes=0.0005)
    assert not b["pass"] and {f["device"] for f in b["failures"]} == {1} and b["failures"][0]["round"] == 1
    assert b["failed_rounds"] == b["rounds"]
    lines = []
    fake(n=2, gpu_rate={1: 0.5})
    diag.burn_in(1, [0, 1], minutes=0.0005, progress=lines.append)
    assert lines and all(ln.startswith("burn-in round ") and "FAIL gpu1:" in ln for ln in lines)
    assert diag.main(["--level", "1", "--duration", "0.0005"]) == 1
    assert json.loads(capsys.readouterr().out)["failures"]
    # a GPU at 90 %: every round passes, as degraded, and the count says so
    fake(n=2, gpu_rate={1: 0.9})
    b = diag.burn_in(1, [0, 1], minutes=0.0005)
    assert b["pass"] and list(b["degraded_rounds"]) == [1], b
    assert b["degraded_rounds"][1]["gemm"] == b["degraded_rounds"][1]["gemm_fp8"] == b["rounds"], b
    assert diag.main(["--level", "1", "--duration", "0.0005", "--format", "text", "--device", "1"]) == 0
    assert f"GPU 1 degraded (below 95% of the reference after re-measuring) in " in capsys.readouterr().out
    fake(n=1)
    assert diag.main(["--level", "1", "--duration", "0.0005", "--format", "text"]) == 0
    text = capsys.readouterr().out
    assert text.startswith("burn-in: ") and "GPU 0 gemm.tflops" in text and text.rstrip().endswith("result: PASS")


def test_diag_cli_fabric_timeout_reports_a_hung_pair(fake, capsys):
    import json
    fake(n=3, hung_pairs=((2, 1),))
    assert diag.main(["--level", "2", "--no-rccl", "--timeout", "0.4"]) == 1
    out = json.loads(capsys.readouterr().out)
    assert out["fabric"]["p2p"]["stopped"].startswith("2->1 hung") and "rccl" not in out["fabric"]
    assert all(t["pass"] for d in out["devices"].values() for t in d["tests"].values())
    # the burn-in runs the node-level tests once after its rounds, under the same deadline
    assert diag.main(["--level", "2", "--no-rccl", "--timeout", "0.4", "--duration", "0.0005"]) == 1
    b = json.loads(capsys.readouterr().out)
    assert not b["failures"] and b["fabric"]["p2p"]["stopped"].startswith("2->1 hung") and not b["pass"]


def test_run_devices_raises_a_missing_library_in_the_caller(monkeypatch):
    from k8s_gpu_node_checker_amd.ops.native import NativeUnavailable

    def gone(level, d, **kw):
        raise NativeUnavailable("libmi355x_diag.so not built")
    monkeypatch.setattr(diag, "run", gone)
    with pytest.raises(NativeUnavailable):
        diag.run_devices(1, [0, 1, 2], parallel=3)
    calls = []

    def flaky(level, d, **kw):
        calls.append(d)
        if d == 1:
            raise RuntimeError("mi355x diag failed (-1): hipMalloc: out of memory")
        return {"gemm": {"pass": True}}
    monkeypatch.setattr(diag, "run", flaky)
    out = diag.run_devices(1, [0, 1, 2], parallel=3)
    assert out[1]["run"]["pass"] is False and "out of memory" in out[1]["run"]["detail"] and out[0]["gemm"]["pass"]


def test_fabric_tests_report_a_raising_test_as_failed(fake, monkeypatch):
    from k8s_gpu_node_checker_amd.ops import fabric
    fake(n=2)

    def boom(*a, **kw):
        raise OSError("librccl.so.1: cannot open shared object file")
    monkeypatch.setattr(fabric, "collective_suite", boom)
    out = diag.fabric_tests([0, 1], timeout_s=10.0)
    assert out["p2p"]["pass"] and out["rccl"]["pass"] is False and "librccl" in out["rccl"]["detail"]

    def bad_pair(*a, **kw):
        raise RuntimeError("mi355x diag failed (-1): hipMalloc: out of memory")
    monkeypatch.setattr(diag, "p2p_matrix", bad_pair)
    out = diag.fabric_tests([0, 1], rccl=False)
    assert out["p2p"]["pass"] is False and "out of memory" in out["p2p"]["detail"] and "rccl" not in out
