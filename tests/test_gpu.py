"""MI355X-only tests (``pytest -m gpu`` on a gfx950 box via gpurun).

Numerics of the HIP MFMA GEMM are checked against a plain PyTorch fp32
reference of the same op; the probe is checked against what amd-smi reported
on a real MI355X (profiles/amdsmi_mi355x.json).
"""
import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def test_native_libraries_present(dev):
    from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag, fastpath
    assert fastpath.backend() == "native"
    assert amdsmi_probe.native_available()
    assert diag.device_count() >= 1
    info = diag.device_info(0)
    assert info["arch"].startswith("gfx950"), info
    assert info["cus"] == 256, info


def test_native_probe_reports_healthy_mi355x(dev):
    from k8s_gpu_node_checker_amd.models.health import HEALTHY, HealthExpectations, evaluate_report
    from k8s_gpu_node_checker_amd.ops.amdsmi_probe import probe_native
    rep = probe_native("test-node")
    assert not rep.get("error"), rep
    g = rep["gpus"][0]
    assert g["gfx"] == "gfx950"
    from k8s_gpu_node_checker_amd.models.health import is_mi35x
    assert is_mi35x(g), g
    assert g["vram_type"] == 5  # HBM3E
    assert g["vram_mb"] > 280000
    assert g["ecc_uncorrectable"] == 0
    assert g["kfd"] is True
    assert set(g["xgmi"]) <= set("UXDN")
    v = evaluate_report(rep, len(rep["gpus"]), HealthExpectations(xgmi_links=g["xgmi"].count("U")))
    assert v.state == HEALTHY, v.to_dict()
    # amd-smi stays initialised: a second probe is fast
    rep2 = probe_native("test-node")
    assert rep2["probe_ms"] < 200, rep2["probe_ms"]


def test_native_probe_reopens_its_session_cleanly(dev):
    """Re-enumeration (driver reload / repartition) on the real library: the session is shut down and
    initialised again between probes, and the GPUs come back the same."""
    import ctypes
    import time
    from k8s_gpu_node_checker_amd.ops import amdsmi_probe as P
    L = P._native()
    L.mi355x_probe_set_reopen_interval.argtypes = [ctypes.c_double]
    first = P.probe_native("n")
    try:
        L.mi355x_probe_set_reopen_interval(0.01)
        for _ in range(3):
            time.sleep(0.05)
            r = P.probe_native("n")
            assert not r.get("error") and [g["bdf"] for g in r["gpus"]] == [g["bdf"] for g in first["gpus"]]
            assert all(not g.get("error") for g in r["gpus"])
    finally:
        L.mi355x_probe_set_reopen_interval(600.0)


def test_python_probe_agrees_with_native(dev):
    pytest.importorskip("amdsmi")
    from k8s_gpu_node_checker_amd.ops.amdsmi_probe import probe_native, probe_python
    ra, rb = probe_native("n"), probe_python("n")
    a, b = ra["gpus"][0], rb["gpus"][0]
    for k in ("gfx", "vram_type", "vram_mb", "ecc_uncorrectable", "xgmi", "compute_partition",
              "memory_partition", "cus", "power_cap_w", "power_cap_default_w", "fw", "vbios_version",
              "xgmi_error", "ecc_blocks", "xgmi_hive", "xgmi_peers", "xgmi_width", "xgmi_speed_gbps",
              "cper", "cper_error"):
        assert a.get(k) == b.get(k), (k, a.get(k), b.get(k))
    assert ra.get("driver") == rb.get("driver") and ra["driver"]["name"] == "amdgpu", (ra.get("driver"), rb.get("driver"))
    # the firmware a node runs: power management / security processor / compute-queue images
    assert a["fw"] and {"mec", "psp_sos"} <= set(a["fw"]), a["fw"]
    # the fabric: one peer per Up link, trained x16 at 38 Gb/s, a hive id
    assert len(a["xgmi_peers"]) == a["xgmi"].count("U") == len(a["xgmi_kb"]), a
    assert a["xgmi_width"] == 16 and a["xgmi_speed_gbps"] == 38 and len(a["xgmi_hive"]) == 16, a
    assert set(a.get("throttle_acc") or {}) == set(b.get("throttle_acc") or {})


def test_native_probe_telemetry_and_throttle_window(dev):
    from k8s_gpu_node_checker_amd.agent.agent import Agent
    from k8s_gpu_node_checker_amd.ops import diag
    ag = Agent("n", source="native")
    g = ag.probe_once()["gpus"][0]
    print(json.dumps({k: g.get(k) for k in ("power_w", "power_cap_w", "hbm_temp_c", "gfxclk_mhz", "throttle_acc")}))
    assert 0 < g["power_w"] <= g["power_cap_w"] + 200 and 500 <= g["power_cap_w"] <= 2000, g
    assert 0 < g["hbm_temp_c"] < 110 and g["gfxclk_mhz"] > 0, g
    assert g["throttle_acc"]["n"] > 0 and "ppt" in g["throttle_acc"], g
    diag.run(1, 0)  # some load between the two samples
    g2 = ag.probe_once()["gpus"][0]
    w = g2["throttle"]
    assert w["s"] > 0 and all(0.0 <= w[k] <= 100.0 for k in ("thermal_pct", "power_pct", "prochot_pct")), w


@pytest.mark.parametrize("m,n,k", [(128, 128, 64), (256, 384, 192), (1024, 1024, 1024), (512, 2048, 4096),
                                   (2048, 1024, 256)])
def test_mfma_gemm_matches_fp32_reference(dev, m, n, k):
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m * 7 + n * 3 + k)
    a = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
    bt = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
    c = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
    diag.gemm_launch(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = a.float() @ bt.float().t()
    assert not torch.isnan(c).any()
    rel = ((c - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
    assert rel < 1e-4 * max(1, k / 512), rel


@pytest.mark.parametrize("variant", ["v1", "v2", "v3", "v3-lds-epilogue", "v4", "v4t"])
@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (256, 512, 128), (512, 256, 192), (768, 512, 256),
                                   (1024, 768, 4096)])
def test_mfma_gemm_variants_match_fp32_reference(dev, variant, m, n, k):
    """Every kernel variant on shapes that exercise 1, 2, 3, 4 and 64 K-tiles (prologue/epilogue
    paths of the staggered v3 pipeline) and non-square grids."""
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + 5 * n + 11 * k)
    a = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
    bt = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
    c = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
    before = diag.get_gemm_config()
    with diag.gemm_config(variant=variant.split("-")[0], epilogue=variant.endswith("lds-epilogue")):
        diag.gemm_launch(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    assert diag.get_gemm_config() == before  # restored, not reset to some other value
    ref = a.float() @ bt.float().t()
    assert not torch.isnan(c).any()
    rel = ((c - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
    assert rel < 1e-4 * max(1, k / 512), rel


@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (512, 256, 192), (768, 512, 256), (1024, 768, 4096),
                                   (2048, 2048, 2048)])
def test_v3_buffer_load_staging_matches(dev, m, n, k):
    """The buffer_load ... lds staging path of the v3 pipeline (bf16 and MX-fp8) computes exactly what
    the global_load_lds path computes, and matches the torch reference."""
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + 3 * n + 7 * k)
    st = torch.cuda.current_stream().cuda_stream
    a = torch.randn(m, k, device=dev, generator=g)
    bt = torch.randn(n, k, device=dev, generator=g)
    for (x, y, launch) in ((a.to(torch.bfloat16), bt.to(torch.bfloat16), diag.gemm_launch),
                           (a.to(torch.float8_e4m3fn), bt.to(torch.float8_e4m3fn), diag.gemm_fp8_launch)):
        if launch is diag.gemm_fp8_launch and k % 128:
            continue
        outs = []
        for buf in (False, True):
            with diag.gemm_config(variant="v3", buffer_loads=buf):
                c = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
                launch(x.data_ptr(), y.data_ptr(), c.data_ptr(), m, n, k, st)
                torch.cuda.synchronize()
                outs.append(c)
        assert torch.equal(outs[0], outs[1])
        if launch is diag.gemm_fp8_launch:  # the MX MFMA's own accumulation error, normalised by sum|a*b|
            ref = x.double() @ y.double().t()
            mag = x.double().abs() @ y.double().abs().t()
            err = ((outs[1].double() - ref).abs() / mag.clamp_min(1e-30)).max().item()
            assert err < diag.GEMM_FP8_MAX_ERR, err
        else:
            ref = x.float() @ y.float().t()
            rel = ((outs[1] - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
            assert rel < 1e-4 * max(1, k / 512), rel


@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (256, 512, 128), (512, 256, 192), (768, 512, 320),
                                   (1024, 768, 4096), (2048, 2048, 2048)])
def test_v3_restaging_schedules_compute_the_same(dev, m, n, k):
    """Both LDS-DMA restaging orders of the v3 pipeline (schedule 1, the default, and the earlier 0) give
    bit-identical outputs for bf16 and MX-fp8, including 1-5 K-tiles (prologue / tail paths), and match torch."""
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + 5 * n + 11 * k)
    st = torch.cuda.current_stream().cuda_stream
    a = torch.randn(m, k, device=dev, generator=g)
    bt = torch.randn(n, k, device=dev, generator=g)
    for (x, y, launch) in ((a.to(torch.bfloat16), bt.to(torch.bfloat16), diag.gemm_launch),
                           (a.to(torch.float8_e4m3fn), bt.to(torch.float8_e4m3fn), diag.gemm_fp8_launch)):
        if launch is diag.gemm_fp8_launch and k % 128:
            continue
        outs = []
        for sched in (0, 1):
            with diag.gemm_config(variant="v3", schedule=sched):
                c = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
                launch(x.data_ptr(), y.data_ptr(), c.data_ptr(), m, n, k, st)
                torch.cuda.synchronize()
                outs.append(c)
        assert torch.equal(outs[0], outs[1])
        if launch is diag.gemm_launch:
            ref = x.float() @ y.float().t()
            rel = ((outs[1] - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
            assert rel < 1e-4 * max(1, k / 512), rel
        else:
            ref = x.double() @ y.double().t()
            mag = x.double().abs() @ y.double().abs().t()
            assert ((outs[1].double() - ref).abs() / mag.clamp_min(1e-30)).max().item() < diag.GEMM_FP8_MAX_ERR
    with pytest.raises(ValueError):
        diag.set_gemm_schedule(2)


@pytest.mark.parametrize("m,n,k", [(256, 256, 128), (512, 256, 256), (768, 512, 384), (1024, 768, 4096),
                                   (2048, 2048, 2048)])
def test_v3_bf16_output_and_fused_checksums_match(dev, m, n, k):
    """The kernel the GEMM diagnostics time (``gemm_launch_ck``): bf16 C is the fp32 kernel's output rounded to
    bf16 (bit-exact, both restaging orders), and the fused column sums equal the fp64 sums of the fp32 kernel's
    output over every 128-row block, for bf16 and MX-fp8 operands, 1-64 K-tiles."""
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + 7 * n + 13 * k)
    st = torch.cuda.current_stream().cuda_stream
    a = torch.randn(m, k, device=dev, generator=g)
    bt = torch.randn(n, k, device=dev, generator=g)
    for dt, x, y, launch in (("bf16", a.to(torch.bfloat16), bt.to(torch.bfloat16), diag.gemm_launch),
                             ("fp8", a.to(torch.float8_e4m3fn), bt.to(torch.float8_e4m3fn), diag.gemm_fp8_launch)):
        with diag.gemm_config(variant="v3"):
            c32 = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
            launch(x.data_ptr(), y.data_ptr(), c32.data_ptr(), m, n, k, st)
            for sched in (0, 1):
                with diag.gemm_config(schedule=sched):
                    c16 = torch.full((m, n), float("nan"), device=dev, dtype=torch.bfloat16)
                    cs = torch.full((m // 128, n), float("nan"), device=dev, dtype=torch.float64)
                    diag.gemm_launch_ck(dt, x.data_ptr(), y.data_ptr(), c16.data_ptr(), cs.data_ptr(), m, n, k, st)
                    torch.cuda.synchronize()
                assert torch.equal(c16, c32.to(torch.bfloat16)), (dt, sched)
                want = c32.double().view(m // 128, 128, n).sum(dim=1)
                mag = c32.double().abs().view(m // 128, 128, n).sum(dim=1)
                assert ((cs - want).abs() / mag).max().item() < 1e-12, (dt, sched)
    with pytest.raises(ValueError):
        diag.gemm_launch_ck("fp8", 0, 0, 0, 0, 256, 256, 64)
    with pytest.raises(RuntimeError, match="null"):  # refused on the host, nothing launched
        diag.gemm_launch_ck("bf16", x.data_ptr(), y.data_ptr(), 0, 0, 256, 256, 128)


@pytest.mark.parametrize("m,n,k", [(256, 256, 128), (1024, 768, 4096), (2048, 2048, 2048)])
def test_fp8_gemm_mfma_forms_are_bit_identical(dev, m, n, k):
    """The fp8 v3 GEMM on the unscaled v_mfma_f32_16x16x128_f8f6f4 (the default, hipBLASLt's form) and on the
    scaled MX form with unit scales: the same fp32 C, bf16 C and fused column sums, bit for bit, and within the
    fp8 error bound of an fp64 reference."""
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + 3 * n + 5 * k)
    st = torch.cuda.current_stream().cuda_stream
    x = torch.randn(m, k, device=dev, generator=g).to(torch.float8_e4m3fn)
    y = torch.randn(n, k, device=dev, generator=g).to(torch.float8_e4m3fn)
    outs = {}
    for unscaled in (True, False):
        with diag.gemm_config(variant="v3", fp8_unscaled=unscaled):
            assert diag.get_gemm_fp8_unscaled() is unscaled
            c32 = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
            diag.gemm_fp8_launch(x.data_ptr(), y.data_ptr(), c32.data_ptr(), m, n, k, st)
            c16 = torch.full((m, n), float("nan"), device=dev, dtype=torch.bfloat16)
            cs = torch.full((m // 128, n), float("nan"), device=dev, dtype=torch.float64)
            diag.gemm_launch_ck("fp8", x.data_ptr(), y.data_ptr(), c16.data_ptr(), cs.data_ptr(), m, n, k, st)
            torch.cuda.synchronize()
            outs[unscaled] = (c32, c16, cs)
    assert diag.get_gemm_fp8_unscaled() is True  # restored
    for a, b in zip(outs[True], outs[False]):
        assert torch.equal(a, b)
    ref = x.double() @ y.double().t()
    mag = x.double().abs() @ y.double().abs().t()
    assert ((outs[True][0].double() - ref).abs() / mag.clamp_min(1e-30)).max().item() < diag.GEMM_FP8_MAX_ERR


def test_fp8_burn_in_kind_runs_the_unscaled_f8f6f4_path_exactly(dev):
    """The burn-in's fp8 kind (the unscaled f8f6f4 instruction) computes its exact integer sums on every CU at
    the fp8 rate -- well above the bf16 rate the gfx94x-era instruction it replaced ran at."""
    from k8s_gpu_node_checker_amd.ops import diag
    r = diag.mfma_burn(0)
    fp8, bf16 = r["kinds"]["fp8"], r["kinds"]["bf16"]
    assert fp8["errors"] == 0 and r["map"]["cus"] == 256
    assert fp8["tflops"] > 1.5 * bf16["tflops"], r["kinds"]


def test_mfma_gemm_large_auto_uses_v4_and_matches(dev):
    """4096^3 in auto mode runs the four-wave v4 kernel, bit-identical to v3; compare every output with a
    bf16-input, fp32-accumulate torch reference.  Runs with the production knobs (what the agent launches)."""
    from k8s_gpu_node_checker_amd.ops import diag
    assert diag.get_gemm_config() == {"variant": "auto", "epilogue": True, "buffer_loads": False, "schedule": 1,
                                     "fp8_unscaled": True, "tail": True}
    m = n = k = 4096
    g = torch.Generator(device=dev).manual_seed(4096)
    a = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
    bt = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
    c = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
    diag.gemm_launch(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = a.float() @ bt.float().t()
    rel = ((c - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
    assert rel < 1e-4 * (k / 512), rel
    with diag.gemm_config(variant="v3"):
        c3 = torch.full_like(c, float("nan"))
        diag.gemm_launch(a.data_ptr(), bt.data_ptr(), c3.data_ptr(), m, n, k, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    assert torch.equal(c, c3)


@pytest.mark.parametrize("m,n,k", [(256, 256, 64), (256, 512, 128), (512, 256, 192), (768, 512, 320),
                                   (1024, 768, 4096), (2048, 2048, 2048), (4096, 4096, 1024)])
def test_v4_gemm_is_bit_identical_to_v3(dev, m, n, k):
    """The four-wave v4 kernels (asm-ordered loop, 128x128 per wave; ``v4t`` with the MFMA operands swapped so the
    accumulators hold row pieces, stored without LDS) accumulate in v3's K order: fp32 C and bf16 C equal v3's bit
    for bit, over 1-64 K-tiles (the prologue, the re-fetch of the last tile and the stale final fragment reads) and
    non-square grids; the fused column sums are v3's (v4: bitwise; v4t sums in another order: to fp64 rounding)."""
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + 3 * n + 17 * k)
    st = torch.cuda.current_stream().cuda_stream
    a = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
    bt = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
    outs = {}
    for variant in ("v3", "v4", "v4t"):
        with diag.gemm_config(variant=variant):
            c32 = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
            diag.gemm_launch(a.data_ptr(), bt.data_ptr(), c32.data_ptr(), m, n, k, st)
            c16 = torch.full((m, n), float("nan"), device=dev, dtype=torch.bfloat16)
            cs = torch.full((m // 128, n), float("nan"), device=dev, dtype=torch.float64)
            diag.gemm_launch_ck("bf16", a.data_ptr(), bt.data_ptr(), c16.data_ptr(), cs.data_ptr(), m, n, k, st)
            torch.cuda.synchronize()
            outs[variant] = (c32, c16, cs)
    mag = outs["v3"][0].double().abs().view(m // 128, 128, n).sum(dim=1)
    for variant in ("v4", "v4t"):
        assert torch.equal(outs["v3"][0], outs[variant][0]), variant
        assert torch.equal(outs["v3"][1], outs[variant][1]), variant
        assert ((outs["v3"][2] - outs[variant][2]).abs() / mag).max().item() < 1e-14, variant
    assert torch.equal(outs["v3"][2], outs["v4"][2])
    c32, c16, cs = outs["v4t"]
    assert torch.equal(c16, c32.to(torch.bfloat16))
    ref = a.float() @ bt.float().t()
    assert ((c32 - ref).abs() / ref.abs().clamp_min(1.0)).max().item() < 1e-4 * max(1, k / 512)


@pytest.mark.parametrize("m,n,k", [(6144, 6144, 256), (2304, 7424, 192), (4352, 4096, 64)])
def test_v4_tail_wave_is_bit_identical(dev, m, n, k):
    """a grid whose last wave is short (576 tiles = 2.25 waves; 261 tiles, an uneven 5-per-XCD
    remainder; 272) runs its whole waves on v4 and the rest as 128x128 quadrants (gemm_v4_tail_kernel): fp32 C, bf16
    C and the fused column sums equal v3's and tail-off v4's bit for bit (v4t: C bitwise, sums to fp64 rounding)."""
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + 5 * n + 11 * k)
    st = torch.cuda.current_stream().cuda_stream
    a = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
    bt = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
    outs = {}
    for name, variant, tail in (("v3", "v3", True), ("v4", "v4", True), ("v4-notail", "v4", False),
                                ("v4t", "v4t", True)):
        with diag.gemm_config(variant=variant, tail=tail):
            c32 = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
            diag.gemm_launch(a.data_ptr(), bt.data_ptr(), c32.data_ptr(), m, n, k, st)
            c16 = torch.full((m, n), float("nan"), device=dev, dtype=torch.bfloat16)
            cs = torch.full((m // 128, n), float("nan"), device=dev, dtype=torch.float64)
            diag.gemm_launch_ck("bf16", a.data_ptr(), bt.data_ptr(), c16.data_ptr(), cs.data_ptr(), m, n, k, st)
            torch.cuda.synchronize()
            outs[name] = (c32, c16, cs)
    assert diag.get_gemm_config()["tail"] is True  # restored
    for name in ("v4", "v4-notail", "v4t"):
        assert not torch.isnan(outs[name][0]).any() and not torch.isnan(outs[name][2]).any(), name  # every tile
        assert torch.equal(outs["v3"][0], outs[name][0]), name
        assert torch.equal(outs["v3"][1], outs[name][1]), name
    assert torch.equal(outs["v3"][2], outs["v4"][2]) and torch.equal(outs["v3"][2], outs["v4-notail"][2])
    mag = outs["v3"][0].double().abs().view(m // 128, 128, n).sum(dim=1)
    assert ((outs["v3"][2] - outs["v4t"][2]).abs() / mag).max().item() < 1e-14


@pytest.mark.parametrize("m,n,k", [(256, 256, 128), (256, 512, 256), (512, 256, 384), (768, 512, 640),
                                   (1024, 768, 4096), (2048, 2048, 2048)])
def test_v4_fp8_gemm_is_bit_identical_to_v3(dev, m, n, k):
    """The four-wave fp8 kernel (quadrant-ordered 16x16x128 MFMAs, half the fragments reloaded per K-tile) issues the
    same MFMA per output block and K-tile as v3's unscaled fp8 path: fp32 C, bf16 C and the fused column sums equal
    v3's bit for bit over 1-32 K-tiles and non-square grids, within the fp8 error bound of an fp64 reference."""
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + 11 * n + 3 * k)
    st = torch.cuda.current_stream().cuda_stream
    x = torch.randn(m, k, device=dev, generator=g).to(torch.float8_e4m3fn)
    y = torch.randn(n, k, device=dev, generator=g).to(torch.float8_e4m3fn)
    outs = {}
    for variant in ("v3", "v4", "v4t"):
        with diag.gemm_config(variant=variant):
            assert diag.lib().diag_gemm_ck_path(1, m, n) == 1
            c32 = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
            diag.gemm_fp8_launch(x.data_ptr(), y.data_ptr(), c32.data_ptr(), m, n, k, st)
            c16 = torch.full((m, n), float("nan"), device=dev, dtype=torch.bfloat16)
            cs = torch.full((m // 128, n), float("nan"), device=dev, dtype=torch.float64)
            diag.gemm_launch_ck("fp8", x.data_ptr(), y.data_ptr(), c16.data_ptr(), cs.data_ptr(), m, n, k, st)
            torch.cuda.synchronize()
            outs[variant] = (c32, c16, cs)
    mag = outs["v3"][0].double().abs().view(m // 128, 128, n).sum(dim=1)
    for variant in ("v4", "v4t"):
        assert torch.equal(outs["v3"][0], outs[variant][0]), variant
        assert torch.equal(outs["v3"][1], outs[variant][1]), variant
        assert ((outs["v3"][2] - outs[variant][2]).abs() / mag).max().item() < 1e-14, variant
    ref = x.double() @ y.double().t()
    err = ((outs["v4"][0].double() - ref).abs() / (x.double().abs() @ y.double().abs().t()).clamp_min(1e-30)).max()
    assert err.item() < diag.GEMM_FP8_MAX_ERR


@pytest.mark.parametrize("m,n,k", [(6144, 6144, 512), (2304, 7424, 256)])
def test_v4_fp8_tail_wave_is_bit_identical(dev, m, n, k):
    """The fp8 tail (128x128 quadrants on the unscaled 16x16x128 MFMA, v3 / v4's fp8 fragments): fp32 C, bf16 C and
    the column sums equal v3's and tail-off v4's bit for bit."""
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + 7 * n + 13 * k)
    st = torch.cuda.current_stream().cuda_stream
    x = torch.randn(m, k, device=dev, generator=g).to(torch.float8_e4m3fn)
    y = torch.randn(n, k, device=dev, generator=g).to(torch.float8_e4m3fn)
    outs = {}
    for name, variant, tail in (("v3", "v3", True), ("v4", "v4", True), ("v4-notail", "v4", False)):
        with diag.gemm_config(variant=variant, tail=tail):
            c32 = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
            diag.gemm_fp8_launch(x.data_ptr(), y.data_ptr(), c32.data_ptr(), m, n, k, st)
            c16 = torch.full((m, n), float("nan"), device=dev, dtype=torch.bfloat16)
            cs = torch.full((m // 128, n), float("nan"), device=dev, dtype=torch.float64)
            diag.gemm_launch_ck("fp8", x.data_ptr(), y.data_ptr(), c16.data_ptr(), cs.data_ptr(), m, n, k, st)
            torch.cuda.synchronize()
            outs[name] = (c32, c16, cs)
    for name in ("v4", "v4-notail"):
        for i in range(3):
            assert torch.equal(outs["v3"][i], outs[name][i]), (name, i)


def test_v4_gemm_diagnostic_reports_bf16_output(dev):
    """The bf16 diagnostic at a size that fills the chip times v4 with bf16 C and fused sums, and passes."""
    from k8s_gpu_node_checker_amd.ops import diag
    assert diag.lib().diag_gemm_ck_path(0, 4096, 4096) == 1
    with diag.gemm_config(variant="v4", epilogue=False):  # v4 has one epilogue: the knob does not apply
        assert diag.lib().diag_gemm_ck_path(0, 4096, 4096) == 1
    with diag.gemm_config(variant="v3", epilogue=False):
        assert diag.lib().diag_gemm_ck_path(0, 4096, 4096) == 0
    r = diag.gemm(0, size=4096, warmup=1, iters=3, samples=512)
    assert r["numerics"] == "" and r["checksum_bad_tiles"] == 0, r
    assert r["output"] == "bf16+colsums" and r["tflops"] > 0, r


def test_mfma_gemm_identity_asymmetric(dev):
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    from k8s_gpu_node_checker_amd.ops import diag
    m = n = k = 128
    a = torch.eye(m, k, device=dev).to(torch.bfloat16)
    idx = torch.arange(n * k, device=dev, dtype=torch.float32).reshape(n, k)
    bt = (idx % 251).to(torch.bfloat16)  # exact in bf16, asymmetric
    c = torch.empty(m, n, device=dev, dtype=torch.float32)
    diag.gemm_launch(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(c, bt.float().t())


def test_gemm_rejects_bad_shapes():
    from k8s_gpu_node_checker_amd.ops import diag
    with pytest.raises(ValueError):
        diag.gemm_launch(0, 0, 0, 100, 128, 64)


def test_diag_gemm_burn_in(dev):
    from k8s_gpu_node_checker_amd.ops import diag
    r = _as_production(lambda: diag.gemm(0, size=4096, warmup=2, iters=10, samples=512))
    print(json.dumps(r))
    assert r["max_rel_err"] < diag.GEMM_MAX_REL_ERR
    assert r["pass"], r


def test_diag_hbm_bandwidth(dev):
    from k8s_gpu_node_checker_amd.ops import diag
    r = _as_production(lambda: diag.hbm(0, gib=2.0, iters=5))
    print(json.dumps(r))
    assert r["pass"], r
    assert r["copy_tbs"] < 8.5  # cannot beat the 8 TB/s HBM3E spec (sanity of the timing)


def test_diag_memtest_clean(dev):
    from k8s_gpu_node_checker_amd.ops import diag
    r = diag.memtest(0, gib=1.0, passes=1)
    print(json.dumps(r))
    assert r["errors"] == 0 and r["pass"], r


def test_memtest_counts_and_locates_an_injected_word(dev):
    """A 16-byte word overwritten between the pattern write and its check is counted once and located to its
    byte offset; the same run without the injection is clean."""
    from k8s_gpu_node_checker_amd.ops import diag
    r = diag.memtest(0, gib=1.0, inject_word=123457)
    assert not r["pass"] and r["errors"] == 1 and r["first_bad_byte"] == 123457 * 16, r
    assert diag.memtest(0, gib=1.0)["errors"] == 0
    with pytest.raises(RuntimeError, match="outside the buffer"):
        diag.memtest(0, gib=1.0, inject_word=1 << 40)


def _tile_xcd(tm, tn, tiles_m, tiles_n, group_m=4):
    """The XCD whose workgroup computes tile (tm, tn): blockIdx b runs on XCD b % 8 (the kernels' regrouping,
    written out independently of diag.hip's tile_xcds)."""
    nwg = tiles_m * tiles_n
    q, r = divmod(nwg, 8)
    for b in range(nwg):
        x = b % 8
        bid = (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + b // 8
        first = bid // (group_m * tiles_n) * group_m
        gsize = min(tiles_m - first, group_m)
        if (first + (bid % (group_m * tiles_n)) % gsize, (bid % (group_m * tiles_n)) // gsize) == (tm, tn):
            return x
    raise AssertionError("tile not computed by any workgroup")


@pytest.mark.parametrize("kind,n,tile,group_m", [("gemm", 4096, 256, 4), ("gemm", 2048, 128, 8),
                                                  ("gemm_fp8", 4096, 256, 4), ("gemm_fp8", 2048, 256, 4)])
def test_gemm_checksums_catch_and_locate_one_corrupted_output(dev, kind, n, tile, group_m):
    """The GEMM tests check every output through tile column checksums, not only the 4,096 sampled ones: a
    healthy run is clean, and one output overwritten after the timing is found in exactly one tile -- its own
    -- and attributed to the XCD that computed it (bf16 2048^2 runs the 128^2-tile kernel with fp32 C, the others
    the 256^2 one with bf16 C, where the hook overwrites the output and its share of the fused column sum)."""
    from k8s_gpu_node_checker_amd.ops import diag
    fn = getattr(diag, kind)
    tol = diag.GEMM_CK_TOL if kind == "gemm" else diag.GEMM_FP8_CK_TOL
    ok = fn(0, size=n, warmup=1, iters=2)  # (small sizes fall short of the 8192^3 rate: only numerics matter)
    assert ok["output"] == ("fp32" if tile == 128 else "bf16+colsums"), ok
    assert ok["checksum_bad_tiles"] == 0 and ok["checksum_err"] < tol / 10 and "checksum" not in ok["detail"], ok
    row, col = n // 2 + 297, n // 3 + 501
    r = fn(0, size=n, warmup=1, iters=2, inject_elem=row * n + col)
    assert not r["pass"] and r["checksum_bad_tiles"] == 1, r
    assert r["checksum_first_bad_tile"] == [row // tile, col // tile], r
    xcd = _tile_xcd(row // tile, col // tile, n // tile, n // tile, group_m)
    assert r["checksum_bad_xcds"] == {str(xcd): 1}, r
    assert "fail their checksums" in r["detail"], r
    with pytest.raises(RuntimeError, match="outside the output"):
        fn(0, size=n, warmup=0, iters=1, inject_elem=n * n)


def test_diag_failed_allocation_leaks_nothing(dev):
    """A diagnostic that runs out of device memory half-way (the agent's GPU got busy) frees what it
    already took and leaves no error behind for the next call: the agent calls these for the life
    of its pod."""
    import ctypes
    import torch
    from k8s_gpu_node_checker_amd.ops import diag
    L = diag.lib()
    torch.cuda.synchronize()
    free0, total = torch.cuda.mem_get_info(0)
    d = [ctypes.c_double() for _ in range(3)]
    big = int(free0 * 0.7) // (1 << 20) << 20  # the first buffer fits, the second cannot
    for _ in range(3):
        assert L.diag_hbm_bandwidth(0, big, 1, *(ctypes.byref(x) for x in d)) == -1
        assert b"out of memory" in L.diag_last_error().lower()
        m = 393216  # C alone is 618 GB; A and Bt (805 MB each) are allocated first
        assert L.diag_gemm_bf16(0, m, m, 1024, 0, 1, 16, *(ctypes.byref(x) for x in d)) == -1
    free1, _ = torch.cuda.mem_get_info(0)
    assert free0 - free1 < (256 << 20), (free0, free1)
    r = _as_production(lambda: diag.hbm(0, gib=0.5, iters=2))  # and the next call runs clean
    assert r["pass"], r


def test_agent_with_diagnostics_is_healthy(dev):
    from k8s_gpu_node_checker_amd.agent.agent import Agent
    from k8s_gpu_node_checker_amd.models.health import HealthExpectations, evaluate_report
    ag = Agent("gpu-node", source="native", diag_level=1, devices=[0], diag_when="always")
    rep = ag.probe_once()
    g = rep["gpus"][0]
    assert g["diag"]["gemm"]["pass"] and g["diag"]["hbm"]["pass"], g["diag"]
    v = evaluate_report(rep, len(rep["gpus"]), HealthExpectations(xgmi_links=g["xgmi"].count("U")))
    assert v.ok, v.to_dict()


def test_agent_self_baseline_forms_on_the_gpu_without_drift(dev, tmp_path):
    """models/baseline.py on real hardware: back-to-back level-1 cycles form the GPU's baseline from its first
    clean runs (2 here), persist it, and the next cycles sit within the drift line of it (run-to-run spread of a
    healthy MI355X: profiles/baseline_soak_l1_mi355x.json)."""
    from k8s_gpu_node_checker_amd.agent.agent import Agent
    from k8s_gpu_node_checker_amd.models import baseline as B
    path = tmp_path / "baseline.json"
    ag = Agent("gpu-node", source="native", diag_level=1, devices=[0], diag_when="always", diag_interval=0.0,
               baseline_file=str(path))
    ag.baselines.runs = 2
    for _ in range(4):
        rep = ag.probe_once()
    g = rep["gpus"][0]
    rated = {t: r for t, r in g["diag"].items() if isinstance(r, dict) and r.get("rates")}
    assert rated and all(r.get("baseline") for r in rated.values()), g["diag"]
    assert not any(r.get("drift") for r in rated.values()), {t: r.get("drift") for t, r in rated.items()}
    assert min(v for r in rated.values() for v in r["baseline"]["ratio"].values()) > B.DRIFT_RATIO
    doc = json.loads(path.read_text())
    assert doc["schema"] == B.SCHEMA and len(doc["gpus"]) == 1
    # the epoch is read off the real amd-smi report: the driver release and this GPU's firmware images
    epoch = next(iter(doc["gpus"].values()))["epoch"]
    assert epoch and epoch.startswith("driver ") and "; fw " in epoch and "pm=" in epoch, epoch
    assert epoch == B.epoch_of(g, rep["driver"]["version"])


def test_smoke(dev):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__
    __graft_entry__.smoke()


def test_bench_contract_on_gpu(repo):
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--steps", "50", "--warmup", "5"],
                       capture_output=True, text=True, timeout=600, cwd=repo)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["check_ok"] and d["n_gpus"] == 1 and d["value"] > 0
    assert d["probe"]["source"] == "native", d["probe"]
    # the line says where a step's time goes (medians; the parts add up to about the step)
    sm = d["step_ms"]
    assert set(sm) >= {"connect", "first_byte", "body", "scan", "client", "health", "render", "other", "step"}
    parts = [v for k, v in sm.items() if k not in ("step", "checker", "transport")]  # the last two are sums of parts
    assert abs(sum(parts) - sm["step"]) < 0.5 * sm["step"]
    assert abs(sm["checker"] + sm["transport"] - sm["step"]) < 0.5 * sm["step"] and d["checker_ms"] == sm["checker"]
    assert [r["nodes"] for r in d["curve"]] == [1, 2, 4, 8, 16, 1000] and all(r["check_ok"] for r in d["curve"])


def test_rccl_collective_single_rank(repo):
    """The RCCL (backend nccl) path of the xGMI diagnostic runs end to end on the GPU (world size 1 here;
    the 8-GPU hive runs it with --nproc-per-node 8)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "-m", "k8s_gpu_node_checker_amd.parallel.collectives",
           "--sizes", "1M,64M", "--iters", "5", "--warmup", "2"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=repo)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert d["backend"] == "nccl" and d["pass"] and all(r["correct"] for r in d["rows"])


def test_rccl_in_process_fabric_suite(dev):
    """libmi355x_fabric.so: ncclCommInitAll over the box's GPUs, all four collectives, every received
    element checked on its GPU against the rank-coded expectation."""
    from k8s_gpu_node_checker_amd.ops import diag, fabric
    n = min(diag.device_count(), 8)
    res = fabric.collective_suite(list(range(n)), sizes=[1 << 20, 64 << 20], iters=3, warmup=1)
    assert res["pass"], res
    assert [(r["op"], r["bytes"]) for r in res["rows"]] == [(op, b) for op in fabric.OPS for b in (1 << 20, 64 << 20)]
    assert all(r["errors"] == 0 and r["algbw_gbps"] > 0 for r in res["rows"]), res["rows"]
    assert res["rccl"] != "unknown"


def test_rccl_suite_with_a_deadline_and_an_abort(dev):
    """Non-blocking communicators: the suite under a generous deadline passes exactly as without one; a
    deadline too short for communicator setup aborts (ncclCommAbort) and comes back as a failed, aborted
    result instead of blocking; the process can build a fresh communicator afterwards."""
    from k8s_gpu_node_checker_amd.ops import diag, fabric
    n = diag.device_count()
    ok = fabric.collective_suite(list(range(n)), sizes=[1 << 20], iters=2, warmup=1, timeout_s=60)
    assert ok["pass"] and not ok.get("aborted"), ok
    t0 = time.monotonic()
    bad = fabric.collective_suite(list(range(n)), sizes=[64 << 20], iters=50, warmup=1, timeout_s=1e-6)
    assert time.monotonic() - t0 < 30
    print(json.dumps({k: bad.get(k) for k in ("pass", "aborted", "detail")}))
    assert bad["pass"] is False and bad["aborted"] is True and "ncclCommAbort" in bad["detail"], bad
    again = fabric.collective_suite(list(range(n)), sizes=[1 << 20], iters=2, warmup=1, timeout_s=60)
    assert again["pass"], again


def test_rccl_abort_while_collectives_are_in_flight(dev):
    """A deadline that passes in the middle of the timed collectives (not during setup): the communicators are
    aborted with kernels in flight, the suite reports which collective, and the process recovers."""
    from k8s_gpu_node_checker_amd.ops import diag, fabric
    n = diag.device_count()
    t0 = time.monotonic()
    warm = fabric.collective_suite(list(range(n)), sizes=[1 << 20], ops=["all_reduce"], iters=1, warmup=0,
                                   timeout_s=60)
    setup = time.monotonic() - t0
    assert warm["pass"], warm
    # 100k x 256 MiB all-reduces take ~10 s even on one GPU (~0.1 ms each); the deadline leaves the setup and
    # a fraction of a second of them
    t0 = time.monotonic()
    cut = fabric.collective_suite(list(range(n)), sizes=[256 << 20], ops=["all_reduce"], iters=100000, warmup=1,
                                  timeout_s=1.5 * setup + 0.3)
    took = time.monotonic() - t0
    print(json.dumps({"setup_s": round(setup, 3), "took_s": round(took, 3),
                      **{k: cut.get(k) for k in ("pass", "aborted", "detail")}}))
    assert cut["pass"] is False and cut["aborted"] is True, cut
    assert "all_reduce" in cut["detail"] and "ncclCommAbort" in cut["detail"]
    assert took < 1.5 * setup + 0.3 + 3.0, took  # the deadline holds while launches are still being issued
    again = fabric.collective_suite(list(range(n)), sizes=[1 << 20], iters=2, warmup=1, timeout_s=60)
    assert again["pass"], again


def test_fabric_cli_stdout_is_pure_json(repo):
    """RCCL prints a version banner during communicator init; the CLI's stdout must still parse as one
    JSON document (the banner goes to stderr)."""
    p = subprocess.run([sys.executable, "-m", "k8s_gpu_node_checker_amd.ops.fabric", "--device", "0",
                        "--sizes", "1M", "--iters", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, cwd=repo)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout)
    assert d["pass"] and d["rows"]


def test_probe_sees_a_workload_and_agent_skips_diagnostics(dev, repo):
    """A second process holding 4 GiB of VRAM shows up in the native probe's per-process list, and an
    idle-only agent (the default) leaves that GPU's diagnostics alone while it is held."""
    from k8s_gpu_node_checker_amd.agent.agent import Agent, gpu_busy
    from k8s_gpu_node_checker_amd.ops.amdsmi_probe import probe_native
    holder = subprocess.Popen([sys.executable, "-c",
                               "import sys, time, torch; x = torch.empty(4 << 30, dtype=torch.uint8, device='cuda:0');"
                               "x.fill_(1); torch.cuda.synchronize(); print('held', flush=True); time.sleep(60)"],
                              stdout=subprocess.PIPE, text=True, cwd=repo)
    try:
        assert holder.stdout.readline().strip() == "held"
        g = probe_native("n")["gpus"][0]
        print(json.dumps({k: g.get(k) for k in ("processes", "procs", "gfx_activity", "vram_used_mb")}))
        assert any(p["pid"] == holder.pid and p["vram_mb"] >= 4096 for p in g["procs"]) or \
            any(p["vram_mb"] >= 4096 for p in g["procs"]), g.get("procs")  # PIDs may be of another namespace
        assert gpu_busy(g) and "in use" in gpu_busy(g)
        ag = Agent("n", source="native", diag_level=1, devices=[0])
        g2 = ag.probe_once()["gpus"][0]
        assert "diag" not in g2 and g2["diag_skipped"].startswith("in use"), g2.get("diag_skipped")
    finally:
        holder.kill()
        holder.wait(timeout=30)
        # the driver frees a killed process's VRAM asynchronously: leave the GPU idle for the next test
        _wait_until_idle()


def _foreign_holders(busy_mb=2048):
    from k8s_gpu_node_checker_amd.ops.amdsmi_probe import probe_native
    g = probe_native("n")["gpus"][0]
    return [p for p in g.get("procs") or [] if p.get("pid") != os.getpid() and p.get("vram_mb", 0) >= busy_mb]


def _wait_until_idle(timeout_s=30.0, busy_mb=2048):
    """Release this process's cached VRAM and poll (bounded) until no other process holds busy_mb."""
    import time
    torch.cuda.empty_cache()
    deadline = time.monotonic() + timeout_s
    held = _foreign_holders(busy_mb)
    while held and time.monotonic() < deadline:
        time.sleep(0.5)
        held = _foreign_holders(busy_mb)
    return held


def test_agent_cli_once_runs_idle_diagnostics(repo):
    """The DaemonSet's entry point end to end: one probe + level-1 diagnostics with the default
    idle-only policy on an idle GPU, the report on stdout."""
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    # earlier tests leave cached VRAM in this process and a killed holder's VRAM is freed late: wait for
    # an idle GPU (bounded), and tell the agent that its parent (this runner) is not a workload
    held = _wait_until_idle()
    assert not held, f"GPU still held by another process: {held}"
    p = subprocess.run([sys.executable, "-m", "k8s_gpu_node_checker_amd.agent.agent", "--once", "--publish", "stdout",
                        "--source", "native", "--diag-level", "1", "--node", "gpu-node",
                        "--ignore-pid", str(os.getpid())],
                       capture_output=True, text=True, timeout=300, cwd=repo)
    assert p.returncode == 0, p.stderr[-2000:]
    rep = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    g = rep["gpus"][0]
    assert "diag_skipped" not in g, g.get("diag_skipped")
    assert g["diag"]["gemm"]["pass"] and g["diag"]["hbm"]["pass"] and g["diag_at"] > 0, g.get("diag")
    assert rep["state"] in ("healthy", "degraded"), rep["state"]


_ISOLATED_AGENT = r"""
import json, os, sys
from k8s_gpu_node_checker_amd.agent.agent import Agent
ag = Agent("gpu-node", source="native", diag_level=1, devices=[0], diag_when="always", diag_interval=0.0,
           isolation="process")
reps = [ag.probe_once() for _ in range(2)]
maps = open("/proc/self/maps").read()
with open(f"/proc/{os.getpid()}/status") as f:
    rss = next(int(l.split()[1]) // 1024 for l in f if l.startswith("VmRSS:"))
print(json.dumps({"pid": os.getpid(), "rss_mib": rss, "reps": reps, "started": ag.workers.started,
                  "hip_in_agent": "libamdhip64" in maps, "diag_in_agent": "libmi355x_diag" in maps}))
"""


def test_agent_process_isolation_keeps_hip_out_of_the_agent(repo):
    """VERDICT r5 #2 on the GPU: the agent's level-1 diagnostics run in forkserver children; the agent process
    itself never maps the HIP runtime or the diagnostics library, stays small, and each cycle's child is new."""
    import torch as _t
    if not _t.cuda.is_available():
        pytest.skip("no GPU")
    _wait_until_idle()
    p = subprocess.run([sys.executable, "-c", _ISOLATED_AGENT], capture_output=True, text=True, timeout=300, cwd=repo,
                       env=dict(os.environ, PYTHONPATH=repo))
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    print(json.dumps({k: d[k] for k in ("rss_mib", "started", "hip_in_agent", "diag_in_agent")}))
    assert not d["hip_in_agent"] and not d["diag_in_agent"], d
    procs = [r["gpus"][0]["diag_proc"] for r in d["reps"]]
    print(json.dumps(procs))
    for r in d["reps"]:
        g = r["gpus"][0]
        assert g["diag"]["gemm"]["pass"] and g["diag"]["hbm"]["pass"], g["diag"]
    assert procs[0]["pid"] != procs[1]["pid"] and d["pid"] not in (procs[0]["pid"], procs[1]["pid"])
    assert procs[0]["peak_rss_mib"] > d["rss_mib"]  # the HIP work's memory was the child's, not the agent's
    assert d["rss_mib"] < 100, d["rss_mib"]
    # a level-1 child starts HIP without the SDMA engines (no level-1 test times a DMA copy): ~445 MiB, against
    # ~630 with them -- the DaemonSet's limit is sized on it (agent.MEM_CHILD_PEAK_MIB)
    from k8s_gpu_node_checker_amd.agent import agent as A
    assert all(p["peak_rss_mib"] <= A.MEM_CHILD_PEAK_MIB[1] * 1.25 for p in procs), procs  # SDMA on: 630-685


def test_agent_diagnostics_threads_per_device(dev):
    from k8s_gpu_node_checker_amd.agent.agent import Agent
    from k8s_gpu_node_checker_amd.ops import diag
    ag = Agent("n", source="native", diag_level=1, diag_when="always")
    rep = ag.probe_once()
    assert len(rep["gpus"]) >= 1
    assert all("diag" in g for g in rep["gpus"][: diag.device_count()])


def test_polled_deadline_returns_at_its_deadline(dev):
    """The wait the xGMI pair copies use (diag_p2p_copy_t) on real HIP: ~150 ms of queued work waited for with a
    20 ms deadline comes back at the deadline, and the work then drains; with a generous deadline it completes."""
    from k8s_gpu_node_checker_amd.ops import diag
    r = diag.poll_selftest(0, launches=1000, deadline_ms=20.0)
    assert r["timed_out"] and 19.0 <= r["waited_ms"] < 60.0 and r["drained_ms"] > 10.0, r
    r = diag.poll_selftest(0, launches=10, deadline_ms=5000.0)
    assert not r["timed_out"] and r["waited_ms"] < 1000.0, r
    with pytest.raises(RuntimeError, match="positive deadline"):
        diag.poll_selftest(0, launches=10, deadline_ms=0.0)


def test_burn_in_on_this_box(dev):
    """``mi355x-diag --duration``: the level-1 suite round after round on the real GPU, every round passing,
    each rate reported as a min / median / max spread."""
    from k8s_gpu_node_checker_amd.ops import diag
    b = diag.burn_in(1, [0], minutes=0.05)
    assert b["pass"], b["failures"]
    assert b["rounds"] >= 2 and b["wall_s"] >= 3.0
    g = b["devices"][0]["gemm.tflops"]
    assert 0 < g["min"] <= g["median"] <= g["max"]
    assert b["devices"][0]["gemm.fraction"]["min"] > diag.FAIL_FRACTION


def test_p2p_diag_on_this_box(dev):
    """The pair matrix is a node-level xGMI test: with one visible GPU it is skipped, and the C ABI
    rejects a pair that is not two distinct devices instead of faulting."""
    from k8s_gpu_node_checker_amd.ops import diag
    n = diag.device_count()
    if n < 2:
        assert diag.p2p_matrix()["skipped"]
        with pytest.raises(RuntimeError, match="two distinct devices"):
            diag.p2p_copy(0, 0)
        with pytest.raises(RuntimeError, match="two distinct devices"):  # the polled (deadline) entry point
            diag.p2p_copy(0, 0, timeout_s=5.0)
    else:
        m = diag.p2p_matrix([0, 1], mib=64, iters=3)
        assert all(p["errors"] == 0 for p in m["pairs"]) and m["min_gbps"] > 1.0, m
        t = diag.p2p_matrix([0, 1], mib=64, iters=3, timeout_s=60.0)  # polled completion: same result
        assert t["pass"] and "stopped" not in t and abs(t["median_gbps"] - m["median_gbps"]) < 0.5 * m["median_gbps"]


def test_mfma_burn_every_precision(dev):
    """bf16 / fp8 / MX-fp8 / MX-fp4 matrix cores: exact results on every wave, rates above the floors."""
    from k8s_gpu_node_checker_amd.ops import diag
    r = _as_production(lambda: diag.mfma_burn(0))
    assert r["pass"], r
    k = r["kinds"]
    assert all(v["errors"] == 0 for v in k.values())
    assert k["mxfp8"]["tflops"] > 1.5 * k["bf16"]["tflops"] and k["mxfp4"]["tflops"] > 1.5 * k["mxfp8"]["tflops"]
    # where the waves ran: every CU of the SPX device, 32 in each of the 8 XCDs, none lagging
    m = r["map"]
    info = diag.device_info(0)
    assert m["cus"] == info["cus"] and "bad_cus" not in m, m
    if info["cus"] == 256:
        assert sorted(m["xcds"]) == [str(x) for x in range(8)] and all(x["cus"] == 32 for x in m["xcds"].values()), m
    assert m.get("slowest_rel", 1.0) <= diag.XCD_SLOW_RATIO, m
    # the hardware deals every CU the same number of workgroups, and no CU lags its XCD
    assert m["waves_per_cu"][0] == m["waves_per_cu"][1] and m["slowest_cu_rel"] <= diag.CU_SLOW_RATIO, m


def test_mfma_burn_rejects_inexact_iteration_counts():
    from k8s_gpu_node_checker_amd.ops import diag
    with pytest.raises(RuntimeError, match="exact fp32"):
        diag.mfma_burn(0, kinds=("mxfp4",), iters=4096, reps=1)


@pytest.mark.parametrize("lds_epilogue", [False, True])
@pytest.mark.parametrize("m,n,k", [(256, 256, 128), (256, 512, 256), (512, 256, 384), (768, 512, 512),
                                   (1024, 768, 8192), (4096, 4096, 4096)])
def test_mxfp8_gemm_matches_fp32_reference(dev, m, n, k, lds_epilogue):
    """MX-fp8 (E4M3) GEMM on the staggered v3 pipeline vs torch on the same fp8 values in fp32."""
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + 3 * n + 7 * k)
    a = torch.randn(m, k, device=dev, generator=g).to(torch.float8_e4m3fn)
    bt = torch.randn(n, k, device=dev, generator=g).to(torch.float8_e4m3fn)
    c = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
    with diag.gemm_config(epilogue=lds_epilogue):
        diag.gemm_fp8_launch(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k,
                             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    ref = a.double() @ bt.double().t()
    mag = a.double().abs() @ bt.double().abs().t()
    assert not torch.isnan(c).any()
    # The MX MFMA does not accumulate a 128-long block in exact fp32: hipBLASLt's fp8 GEMM
    # (torch._scaled_mm) shows the identical error, <= 1.6e-5 of sum|a*b| (tools/fp8_numerics.py,
    # profiles/fp8_numerics_mi355x.jsonl); a layout or staging bug is off by O(1).
    worst = ((c.double() - ref).abs() / mag.clamp_min(1e-30)).max().item()
    assert worst < 4e-5, worst


def test_mxfp8_gemm_identity_asymmetric(dev):
    from k8s_gpu_node_checker_amd.ops import diag
    m = n = 256
    k = 256
    a = torch.eye(m, k, device=dev).to(torch.float8_e4m3fn)
    bt = ((torch.arange(n * k, device=dev, dtype=torch.float32).reshape(n, k) % 13) - 6).to(torch.float8_e4m3fn)
    c = torch.empty(m, n, device=dev, dtype=torch.float32)
    diag.gemm_fp8_launch(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(c, bt.float().t()[:m, :n])


def test_diag_gemm_fp8_burn_in(dev):
    from k8s_gpu_node_checker_amd.ops import diag
    r = _as_production(lambda: diag.gemm_fp8(0, size=4096, warmup=2, iters=5, samples=512))
    assert r["pass"], r
    assert r["max_err_over_mag"] < 4e-5 and r["tflops"] > 1200


FP4_VALUES = [0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0, -0.0, -0.5, -1.0, -1.5, -2.0, -3.0, -4.0, -6.0]


def _fp4_operand(rows, k, gen, dev):
    """Random E2M1 codes -> (packed bytes [rows, k/2], decoded float32 values [rows, k])."""
    codes = torch.randint(0, 16, (rows, k), generator=gen, device=dev, dtype=torch.int32)
    table = torch.tensor(FP4_VALUES, device=dev)
    packed = (codes[:, 0::2] | (codes[:, 1::2] << 4)).to(torch.uint8)
    return packed.contiguous(), table[codes]


@pytest.mark.parametrize("m,n,k", [(256, 256, 256), (512, 256, 768), (768, 512, 1024), (1024, 1024, 8192)])
def test_mxfp4_gemm_matches_fp64_reference(dev, m, n, k):
    from k8s_gpu_node_checker_amd.ops import diag
    g = torch.Generator(device=dev).manual_seed(m + n + k)
    a, av = _fp4_operand(m, k, g, dev)
    bt, bv = _fp4_operand(n, k, g, dev)
    c = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
    diag.gemm_fp4_launch(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = av.double() @ bv.double().t()
    mag = av.double().abs() @ bv.double().abs().t()
    assert not torch.isnan(c).any()
    worst = ((c.double() - ref).abs() / mag.clamp_min(1e-30)).max().item()
    assert worst < 4e-5, worst


def test_host_link_bandwidth_and_pcie_fields(dev):
    from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag
    r = diag.host_link(0, mib=128, iters=3)
    print(json.dumps(r))
    assert r["h2d_gbps"] > 1.0 and r["d2h_gbps"] > 1.0
    g = amdsmi_probe.probe_native("n")["gpus"][0]
    assert g.get("pcie_max_width", 0) >= 1 and g.get("pcie_width", 0) >= 1, g


def test_lds_test_every_cu_and_injected_fault(dev):
    """Every CU's 160 KiB LDS holds all four patterns; one word flipped in one workgroup is counted
    once and located to that workgroup's CU."""
    from k8s_gpu_node_checker_amd.ops import diag
    info = diag.device_info(0)
    r = diag.lds_test(0)
    assert r["pass"] and r["errors"] == 0 and r["cus"] == info["cus"], r
    assert r["bytes_per_cu"] >= 160 * 1024 - 64, r  # gfx950: the whole 160 KiB per workgroup
    bad = diag.lds_test(0, rounds=1, inject_block=5)
    assert not bad["pass"] and bad["errors"] == 1 and len(bad["bad_cus"]) == 1, bad
    assert bad["bad_cus"][0].endswith("(1 words)") and bad["bad_cus"][0].startswith("xcd"), bad


def _as_production(measure):
    """A rate diagnostic as ``ops/diag.run`` takes it: a slow-only result (rate or one lagging XCD, numerics fine)
    is measured again, up to REMEASURE times, the best kept.  One box showed a single XCD reading HBM at 0.41x
    of the others once and 1.33 TB/s like the rest in the next three runs
    (profiles/pytest_gpu_r05_hbm_xcd_transient.log)."""
    from k8s_gpu_node_checker_amd.ops import diag
    r = measure()
    for _ in range(diag.REMEASURE):
        if not diag._slow_only(r):
            break
        again = measure()
        r = again if diag._goodness(again) > diag._goodness(r) else r
    return r


def test_hbm_per_xcd_together_and_alone(dev):
    from k8s_gpu_node_checker_amd.ops import diag
    r = _as_production(lambda: diag.hbm_xcd(0))
    print(json.dumps(r))
    assert r["pass"] and r["errors"] == 0, r
    info = diag.device_info(0)
    if info["cus"] >= 256:
        assert len(r["alone_tbs"]) == 8 and r["slowest_xcd_rel"] >= diag.XCD_ALONE_MIN_RATIO
        assert r["read_tbs"] < 8.5  # cannot beat the HBM3E spec


def test_l2_bandwidth_per_xcd(dev):
    """Each XCD reads its own L2-resident slice: aggregate rate above the floor, every CU and XCD seen,
    no XCD lagging, every word intact."""
    from k8s_gpu_node_checker_amd.ops import diag
    r = _as_production(lambda: diag.l2_bandwidth(0))
    info = diag.device_info(0)
    assert r["pass"] and r["errors"] == 0 and r["map"]["cus"] == info["cus"], r
    if info["cus"] == 256:
        assert len(r["map"]["xcds"]) == 8 and r["read_tbs"] > 25.0, r


def test_gemm_knobs_are_thread_local_and_concurrent_threads_agree(dev):
    """The agent runs one diagnostic thread per GPU: a knob set in one thread must not change what
    another launches, and concurrent first launches of the 128 KiB-LDS v3 kernel (whose dynamic-LDS
    attribute is set once per device) all succeed and match."""
    import threading
    from k8s_gpu_node_checker_amd.ops import diag
    m = n = k = 4096
    g = torch.Generator(device=dev).manual_seed(77)
    a = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
    bt = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
    ref = a.float() @ bt.float().t()
    seen, errs, outs = [], [], []
    with diag.gemm_config(variant="v1", epilogue=False):
        def worker():
            try:
                torch.cuda.set_device(dev)
                seen.append(diag.get_gemm_config())
                s = torch.cuda.Stream(device=dev)
                c = torch.full((m, n), float("nan"), device=dev, dtype=torch.float32)
                # the NaN fill ran on this thread's current stream: order it before the GEMM on s (torch's
                # streams do not synchronize with it by themselves; a fill finishing late overwrote C with NaN)
                s.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(s):
                    diag.gemm_launch(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, s.cuda_stream)
                s.synchronize()
                outs.append(c)
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))
        ts = [threading.Thread(target=worker) for _ in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        assert diag.get_gemm_config()["variant"] == "v1"  # this thread's own setting survives
    assert not errs, errs
    assert seen == [{"variant": "auto", "epilogue": True, "buffer_loads": False, "schedule": 1,
                     "fp8_unscaled": True, "tail": True}] * 4
    for c in outs:
        rel = ((c - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
        assert rel < 1e-4 * (k / 512), rel
        assert torch.equal(c, outs[0])


def test_xgmi_fan_entry_point_on_one_gpu(dev):
    """diag_p2p_fan_t loads and validates on real HIP (a one-GPU box has no peers to fan to): a fan to the source
    itself is refused before anything is allocated; the matrix skips a lone GPU."""
    from k8s_gpu_node_checker_amd.ops import diag
    with pytest.raises(RuntimeError, match="every peer must be a device other than the source"):
        diag.p2p_fan(0, [0], mib=1, iters=1)
    with pytest.raises(RuntimeError, match="1..64 peers"):
        diag.p2p_fan(0, [], mib=1, iters=1)
    if diag.device_count() == 1:
        m = diag.p2p_matrix([0])
        assert m["pass"] and m["skipped"]
