"""Active MI355X diagnostics: ctypes front-end of ``libmi355x_diag.so`` (``csrc/diag/diag.hip``).

Each test returns a dict that the node agent folds into its probe report
under ``gpus[i].diag.<test>`` and that :func:`models.health.evaluate_gpu`
turns into a failure when ``pass`` is false.

Rate tests are judged against the measured rates of a healthy MI355X, scaled to
the device's partition (see the threshold block below): under 85 % fails, 85-95 %
passes as *degraded*.

The library is *required* on a GPU box: a missing build raises
:class:`~k8s_gpu_node_checker_amd.ops.native.NativeUnavailable` instead of
silently skipping the diagnostic.
"""

from __future__ import annotations

import ctypes
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

from .native import NativeUnavailable, load_cdll

# --- Pass / degraded thresholds --------------------------------------------------------------------
# Every rate test is judged against the *reference rate* of a healthy, unpartitioned MI355X (256 CUs,
# SPX/NPS1, 1400 W cap): the lower of (a) the median of a sustained soak and (b) what one cold run
# measures, since the agent runs the suite once per --diag-interval on an idle (clocked-down) GPU:
#   8192^3 (level 2): profiles/soak_level2_5min_mi355x.json, 589 rounds of the full level-2 suite in 5 min
#       hbm copy 6.55 / read 6.98 TB/s, mfma bf16 1901, fp8 1940, mxfp8 4326, mxfp4 7610 TFLOP/s, host link
#       h2d 57.2 / d2h 56.8 GB/s; the GEMMs since the v3 restaging order 1 (round 3):
#       profiles/soak_level2_sched1_mi355x.json (314 rounds, 3 min) gemm 1232 (min 1214), gemm_fp8 2440
#       (min 2337); cold single runs (profiles/diag_cold_sched1_mi355x.jsonl) 1228-1240 / 2376-2457
#   4096^3 (level 1): profiles/soak_level1_mi355x.json, 970 rounds in 2 min: hbm copy 6.49 / read 6.96 TB/s,
#       mfma bf16 1978, fp8 2009, mxfp8 4493, mxfp4 7834; GEMMs with order 1:
#       profiles/soak_level1_sched1_mi355x.json (963 rounds, 3 min) gemm 1343 warm but 1275-1294 in single
#       cold runs, gemm_fp8 2300 warm / 2208-2242 cold (order 0 measured 1207-1226 / 2098-2108 cold)
#   bf16 GEMM since the four-wave v4 kernel (round 5): the v3 references scaled by the measured v4/v3 ratio
#       (REFERENCE_RATES["gemm"] below), then lowered so the slowest healthy device measured sits at >= 0.97
#   Devices differ: two MI355X of the round-5 pool, same tree, cold level-1 runs (profiles/
#       diag_box_spread_r05_mi355x.jsonl): 0000:8e:00.0 gemm 1,278-1,280 / gemm_fp8 2,318-2,332 / MX-fp4 burn
#       6,977-7,035 against 0000:d9:00.0's 1,457-1,487 / 2,585-2,635 / 8,004-8,252 (0.86-0.89 of it, with HBM,
#       L2 and the bf16 burn-in alike).  A reference set on a fast device flags slow healthy ones "degraded"
#       for life, so every compute reference is at most the slowest healthy device / 0.97
# A result below FAIL_FRACTION of its reference fails (a GPU at 55 % clock or power is unhealthy); one
# between FAIL_FRACTION and DEGRADED_FRACTION passes as *degraded* (a warning on the node, still Ready).
# The 85 % floor sits under every soak minimum (worst: gemm_fp8 8192^3 at 90 % of its median) and under
# the ~10 % box-to-box DVFS spread; a rate that lands below 95 % is measured again (REMEASURE) before it is
# reported (best of three), so a noisy sample does not flap the node's verdict.
#
# Partitions: the reference rates are scaled by the share of the physical GPU the HIP device is.
#   compute (GEMM, MFMA burn-in):   cus / 256       (CPX: 32 CUs -> 1/8)
#   memory (HBM copy / read):       min(mem_bytes / 288 GiB, 1/NPS, cus / 256)
#   host link (PCIe):               cus / 256       (every partition of one GPU shares its x16 link)
# Power: a GPU whose power cap was lowered below its default runs its matrix cores at lower clocks; the
# compute references are scaled by cap / default (run(power_fraction=...), from amd-smi), which is lenient
# (rate falls slower than power), so a deliberately capped GPU is judged against its cap, not failed for it.
#
# Concurrency: the node agent runs every GPU's suite at once (--diag-parallel).  Per-GPU resources (CUs, HBM,
# the GPU's own power budget) are not shared between GPUs; the host side is, so the tests that measure it --
# SHARED_TESTS, the PCIe host link (pinned host memory, the CPU root complex, switch uplinks two GPUs may share)
# -- run one device at a time under a process-wide lock, each against the single-GPU reference.  The rate
# references themselves were measured on one MI355X running alone; the same suite on all 8 GPUs of a node at
# once is unmeasured (parity unpinned: no 8-GPU box was available to this project).
# The partition scaling is proportional, not measured (no partitioned MI355X was available): it is the
# lenient bound, so a healthy partition never fails; a partitioned GPU's degraded band is advisory.
#
# These absolute lines judge a GPU *alone*.  GPUs measured together on one node are judged against each other
# (models/peers.judge_node, applied by the node agent, `mi355x-diag` and the burn-in): a GPU under 85 % of its
# node's other GPUs fails by name, a shortfall every GPU shares alike is one node-level *degraded* finding (the
# platform's cooling / power / firmware, never `unhealthy`), and each GPU also keeps a self-baseline of its first
# clean runs (models/baseline.py) whose drift is a warning.  So the references below are not re-tuned to
# whichever box ran last: a slower healthy platform shows as a node-level note, not as failed GPUs.
FAIL_FRACTION = 0.85
SHARED_TESTS = frozenset(("host_link",))
# tests that time the DMA (SDMA) engines: every other test keeps its copies to a few KiB or on the device.  A process
# that runs none of them can start its HIP runtime with HSA_ENABLE_SDMA=0 -- copies then run as blit kernels, and the
# runtime never sets up its SDMA queues, which hold ~180 MiB of host memory from the first copy of 32 KiB or more on
# (tools/hip_rss_probe.hip, tools/copy_threshold.sh).  The agent's isolated children do (agent/isolation.py).
DMA_TESTS = frozenset(("host_link",))


def uses_dma(level: int) -> bool:
    """Whether the suite of ``level`` times a DMA-engine copy (:data:`DMA_TESTS`)."""
    return any(t.replace("_quick", "") in DMA_TESTS for t in LEVELS.get(level, ()))
_HOST_SHARED: Any = threading.Lock()  # held by the one device measuring a SHARED_TESTS test
_HOST_HOLDER: Dict[str, Any] = {}  # who holds it: {"device": d, "since": monotonic time}
# per-device diagnostic *processes* (agent/isolation.py) share a multiprocessing lock instead, and say who holds it
# in a shared (device, since) cell: CLOCK_MONOTONIC is one clock for every process of the host
_HOST_CELL: Any = None
_HOST_LABEL: Optional[int] = None  # the device a narrowed child (one visible GPU, ordinal 0) stands for
# how long a device waits for the host-resource lock when run() is given no deadline (s): a healthy 8-GPU turn
# at the host link is ~8 x 0.1 s, so this only ever expires behind a device stuck inside its host-link test
SHARED_WAIT_S = 120.0
# A rate below the degraded line (numerics fine) is measured again, up to REMEASURE more times, and the best
# is kept: under sustained load the burn-in dips below 95 % in ~10 % of single runs (power management),
# two dips in a row were 19 of 1,913 soak rounds (profiles/soak_level1_r2_mi355x.json); three in a row
# would be ~0.1 %.
REMEASURE = 2
DEGRADED_FRACTION = 0.95
FULL_CUS = 256
FULL_MEM_BYTES = 288 << 30
REFERENCE_RATES: Dict[str, Dict[Any, float]] = {
    # bf16 MFMA GEMM, TFLOP/s.  The diagnostics run the four-wave v4 kernel since round 5; its references are the
    # v3 kernel's (4096: 1280, 8192: 1228, above) times the v4/v3 ratio of cold diagnostic runs on one box,
    # alternated run by run (profiles/diag_cold_v3v4_mi355x.jsonl, second block): medians 1310 / 1217 = 1.076 at
    # level 1 and 1308 / 1203 = 1.087 at level 2, rounded down -- the same relative margin for every box as before.
    # That box is a slow one (v3 at 0.95 of its old reference); its v4 soaks: level 2, 322 rounds, 1300-1326, level 1,
    # 669 rounds, 1309-1332 (profiles/soak_l{1,2}_v4_mi355x.json).  Lowered from 1,370 / 1,330 after a slower
    # healthy device (8e:00.0 above) measured 1,278-1,280 cold at 4096^3 (0.93: degraded): 1,280 / 0.97 -> 1,310.
    # Its 8192^3 rate was not measured (the pool did not hand it out again); level 2 / level 1 is 0.93-0.99 on
    # the devices that were (d9, 26, 5d: 1,355-1,405 at level 2 against 1,419-1,487 at level 1; the calibration
    # box above), so 1,190-1,267 expected -> 1,240 puts even the low end at 0.96.  The others sit at 1.08-1.13.
    "gemm": {4096: 1310.0, 8192: 1240.0},
    # MX-fp8 GEMM, TFLOP/s.  8192^3 with the bf16-output kernel: 2,294-2,450 over a 6-minute level-2 burn-in
    # (median 2,402, profiles/diag_burn_in_level2_6min_bf16out_mi355x.json), 2,199 as the best of three on the
    # slowest box's cold node cycle (profiles/node_cycle_1gpu_mi355x.json) -> 2,300 puts that healthy run at
    # 0.956, above the degraded line (the fp32-output 2,380 left a slow healthy box degraded in most rounds)
    # v3's 2,210 / 2,300 times the same box's fp8 v4/v3 cold ratio, 2,377 / 2,269 = 1.047 (level 1) and 2,386 / 2,277
    # = 1.048 (level 2), rounded down; its v4 soaks 2,373-2,438.  8192^3 lowered from 2,400: the slow device 8e:00.0
    # (2,318-2,332 at 4096^3, level 2 not measured) at the level-2 / level-1 ratio of the measured devices
    # (0.99-1.0) would sit at 0.96-0.97 of 2,400 -> 2,350
    "gemm_fp8": {4096: 2300.0, 8192: 2350.0},
    "hbm": {"copy_tbs": 6.49, "read_tbs": 6.96},   # 16-byte copy (read + write bytes counted) / read, TB/s
    # register-resident burn-in.  fp8 is the unscaled f8f6f4 instruction since round 4 (it was the gfx94x
    # v_mfma_f32_16x16x32_fp8_fp8, 1,940): 40 runs median 4,872 vs MX-fp8's 4,844 in the same runs, first (cold)
    # run 4,058 (profiles/mfma_kinds_mi355x.json) -> MX-fp8's reference x 4,872 / 4,844.  MX-fp4 lowered from 7,610:
    # the slow device 8e:00.0 burns 6,977-7,035 (0.92, degraded) while its other kinds sit at 0.98-1.02 ->
    # 6,977 / 0.97 -> 7,190 (d9:00.0: 7,982-8,259)
    "mfma": {"bf16": 1901.0, "fp8": 4350.0, "mxfp8": 4326.0, "mxfp4": 7190.0},
    "host_link": {"h2d_gbps": 57.0, "d2h_gbps": 56.8},  # pinned copies over PCIe Gen5 x16
    # per-XCD HBM reads, 8 x 256 MiB slices (read 4x since profiles/hbm_xcd_passes_mi355x.json: lone-XCD
    # spread 0.994 at 4 passes vs 0.987 at 2, +5 ms); at 2 passes all XCDs together 5.83-6.27 TB/s (a cold level-2
    # run and 1,299 level-1 soak rounds), each XCD alone 1.23-1.33 TB/s (profiles/hbm_xcd_explore_mi355x.json,
    # profiles/soak_level1_hbm_xcd_mi355x.json)
    "hbm_xcd": {"read_tbs": 5.8, "alone_tbs": 1.28},
    "l2": {"read_tbs": 30.5},                      # per-XCD L2 reads, 2 MiB slices, 8 WG/CU: 31.6-31.9 measured
                                                   # (profiles/l2_explore_mi355x.json; 34.5 TB/s is the L2's own figure)
}
# What produced each test's rates besides the references above: the kernel (and shape policy) that runs it.  Bump a
# test's entry when a kernel change moves its rates; a self-baseline (models/baseline.py) formed under another
# revision -- or under other REFERENCE_RATES for the test, since a baseline is a fraction of them -- re-forms.
KERNEL_REVISION: Dict[str, str] = {
    "gemm": "bf16-v4",           # four-wave v4 MFMA GEMM since round 5 (v3 before)
    "gemm_fp8": "mxfp8-v4",
    "hbm": "copy16-r1", "hbm_xcd": "xcd-slices-4pass", "l2": "xcd-l2-2mib",
    "mfma": "burn-f8f6f4-r4",    # fp8 as the unscaled f8f6f4 instruction since round 4
    "host_link": "pinned-r1",
}


def rate_revision(test: str) -> str:
    """A short stamp of what a test's rate fractions are relative to: its kernel revision and its reference rates."""
    import hashlib
    import json as _json
    ref = REFERENCE_RATES.get(test)
    doc = {"kernel": KERNEL_REVISION.get(test, ""),
           "ref": {str(k): v for k, v in ref.items()} if isinstance(ref, dict) else None}
    return hashlib.sha256(_json.dumps(doc, sort_keys=True).encode()).hexdigest()[:12]


# Sampled errors.  The v4 / v3 kernels the diagnostics time write bf16 C (diag.hip OUT_BF16_CK): there the error is
# what lies beyond the output's own rounding (half a bf16 ulp), so the limits below hold for both outputs.
GEMM_MAX_REL_ERR = 2e-3       # vs fp32 reference; bf16 inputs are exact in fp32, so ~1e-5 is typical
GEMM_FP8_MAX_ERR = 4e-5       # |C - ref| / sum|a*b|: the MX MFMA's own accumulation error is <= 1.6e-5
# whole-output tile checksums (diag.hip gemm_checksum): |column sum of a tile - fp64 reference| / sum|a*b| over
# the same outputs.  Healthy MI355X maxima (profiles/gemm_checksum_mi355x.jsonl, deterministic run to run): bf16
# 2.3e-9, MX-fp8 5.4e-7, so 43x / 18x margins.  At 8192^3 bf16 a tile column's sum|a*b| is ~5.2e5, so one output
# off by more than ~0.05 (a typical output is ~30) fails its tile.
GEMM_CK_TOL = 1e-7
GEMM_FP8_CK_TOL = 1e-5
MEMTEST_MAX_ERRORS = 0
MFMA_KINDS = ("bf16", "fp8", "mxfp8", "mxfp4")
P2P_MIN_FRACTION_OF_MEDIAN = 0.5  # a GPU pair slower than half the node's median pair: suspect link
# The absolute anchor of the xGMI pair matrix: one direction of one link carries lanes x Gb/s / 8 GB/s -- x16 at
# 38 Gb/s on MI355X (amd-smi's xgmi_link_width / xgmi_link_speed, profiles/amdsmi_xgmi_link_metrics_mi355x.json), 76
# GB/s -- and a pair copying under half of that fails whatever its node's median is, so a hive whose links are all
# degraded alike fails too.  The fan pass (every peer of a source at once) is judged against half of the fan's median
# destination and a quarter of the link: under load the copy engines, not only the links, set the pace.  Both floors
# are set from the link's signalling rate, not from a measurement: no 8-GPU node was available to this project.
P2P_MIN_FRACTION_OF_LINK = 0.5
P2P_FAN_MIN_FRACTION_OF_LINK = 0.25
# burn-in waves of one XCD taking this much longer than the median XCD's: that XCD's clock domain (or a
# CU in it) lags -- degraded, not failed (the rate floors above judge the chip as a whole).  A healthy
# MI355X spreads 1.003-1.024 (20 burn-ins, profiles/mfma_xcd_map_mi355x.json), so 1.15 is ~6x its noise.
XCD_SLOW_RATIO = 1.15
# the same for one CU against the median CU of its own XCD (so an XCD-wide lag names the XCD, not its
# CUs).  Healthy MI355X (profiles/mfma_xcd_map_mi355x.json, every CU dealt the same workgroup count): the
# burn-in's register-resident waves take the same time to the 10 ns tick on every CU of an XCD (1.000 in
# 20 runs: one clock per XCD, no memory traffic); the L2 test's 1.016-1.022
CU_SLOW_RATIO = 1.15
# an XCD reading HBM alone at less than this share of the median XCD alone: its path to the memory stacks is
# slow (healthy spread < 3 %, profiles/hbm_xcd_explore_mi355x.json)
XCD_ALONE_MIN_RATIO = 0.9


class Scale:
    """Share of a full MI355X that one HIP device is (1.0 / 1.0 unpartitioned)."""

    def __init__(self, compute: float = 1.0, memory: float = 1.0):
        self.compute = compute
        self.memory = memory

    @classmethod
    def of(cls, cus: Optional[int] = None, mem_bytes: Optional[int] = None,
           memory_partition: Optional[str] = None, power_fraction: Optional[float] = None) -> "Scale":
        c = min(1.0, cus / FULL_CUS) if isinstance(cus, int) and cus > 0 else 1.0
        m = c
        if isinstance(power_fraction, (int, float)) and 0.0 < power_fraction < 1.0:
            c *= power_fraction  # compute only: HBM and the host link do not follow the core clock
        if isinstance(mem_bytes, int) and mem_bytes > 0:
            m = min(m, mem_bytes / FULL_MEM_BYTES)
        if isinstance(memory_partition, str) and memory_partition.upper().startswith("NPS"):
            try:
                m = min(m, 1.0 / max(1, int(memory_partition[3:])))
            except ValueError:
                pass
        return cls(c, min(1.0, m))

    def to_dict(self) -> Dict[str, float]:
        return {"compute": round(self.compute, 4), "memory": round(self.memory, 4)}


FULL = Scale()


def judge_rate(value: float, expected: float) -> str:
    """``pass``, ``degraded`` or ``fail`` for a measured rate against its (scaled) reference."""
    if value < FAIL_FRACTION * expected:
        return "fail"
    if value < DEGRADED_FRACTION * expected:
        return "degraded"
    return "pass"


def _rated(res: Dict[str, Any], rates: Dict[str, float], expected: Dict[str, float], unit: str,
           numerics_ok: bool = True, numerics_detail: str = "") -> Dict[str, Any]:
    """Record a rate test's raw findings in ``res`` -- ``rates``, ``expect`` (the scaled references), ``unit``
    and ``numerics`` (what was wrong with the results, "" when nothing) -- and judge them against the
    references (:func:`judge_absolute`).  The raw fields stay so a node-level judgement
    (``models/peers.judge_node``: the GPU against the node's other GPUs) can re-judge the same result."""
    res["rates"] = {k: round(float(v), 4) for k, v in rates.items()}
    res["expect"] = {k: round(v, 3) for k, v in expected.items()}
    res["unit"] = unit
    res["numerics"] = "" if numerics_ok else (numerics_detail or "wrong results")
    return judge_absolute(res)


def _notes(res: Dict[str, Any]) -> List[str]:
    """The degraded-only notes of a result: lagging XCDs / CUs (``lag``), drift from the GPU's own
    baseline (``drift``, models/baseline.py)."""
    return [str(x) for key in ("lag", "drift") for x in (res.get(key) or []) if x]


def judge_absolute(res: Dict[str, Any]) -> Dict[str, Any]:
    """``pass`` / ``degraded`` / ``fraction`` / ``detail`` of a rate test from its raw fields: numerics wrong ->
    failed; a rate under FAIL_FRACTION of its reference -> failed, under DEGRADED_FRACTION -> degraded; a lag or
    drift note -> degraded.  How a lone GPU (or one with no peers this cycle) is judged."""
    worst, problems, slow = 1e9, [], []
    unit = res.get("unit", "")
    expected = res.get("expect") or {}
    for k, v in (res.get("rates") or {}).items():
        exp = expected.get(k, 0.0)
        frac = v / exp if exp > 0 else 1.0
        worst = min(worst, frac)
        j = judge_rate(v, exp)
        txt = f"{k} {v:.3g} {unit} = {frac:.0%} of {exp:.3g}"
        if j == "fail":
            problems.append(txt)
        elif j == "degraded":
            slow.append(txt)
    if res.get("numerics"):
        problems.insert(0, res["numerics"])
    notes = _notes(res)
    res["pass"] = not problems
    res["degraded"] = bool(slow or notes) and not problems
    res["fraction"] = round(worst, 3) if worst < 1e9 else 1.0
    res["detail"] = "; ".join(problems or (slow + notes))
    res.pop("peers", None)
    return res


_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        L = load_cdll("libmi355x_diag.so", required=True)
        assert L is not None
        L.diag_last_error.restype = ctypes.c_char_p
        L.diag_set_gemm_variant.argtypes = [ctypes.c_int]
        L.diag_set_gemm_epilogue.argtypes = [ctypes.c_int]
        L.diag_set_gemm_buffer_loads.argtypes = [ctypes.c_int]
        L.diag_set_gemm_schedule.argtypes = [ctypes.c_int]
        L.diag_set_gemm_fp8_unscaled.argtypes = [ctypes.c_int]
        L.diag_set_gemm_tail.argtypes = [ctypes.c_int]
        L.diag_get_gemm_tail.restype = ctypes.c_int
        for getter in ("diag_get_gemm_variant", "diag_get_gemm_epilogue", "diag_get_gemm_buffer_loads",
                       "diag_get_gemm_schedule", "diag_get_gemm_fp8_unscaled"):
            getattr(L, getter).restype = ctypes.c_int
        L.diag_device_count.restype = ctypes.c_int
        L.diag_device_arch.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.diag_gemm_bf16_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.diag_gemm_bf16.argtypes = [ctypes.c_int] * 7 + [ctypes.POINTER(ctypes.c_double)] * 3
        L.diag_gemm_fp8.argtypes = [ctypes.c_int] * 7 + [ctypes.POINTER(ctypes.c_double)] * 3
        for f in ("diag_gemm_bf16_x", "diag_gemm_fp8_x"):
            getattr(L, f).argtypes = [ctypes.c_int] * 7 + [ctypes.c_longlong, ctypes.c_double] + \
                [ctypes.POINTER(ctypes.c_double)] * 4 + [ctypes.POINTER(ctypes.c_longlong)]
        L.diag_gemm_fp4_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.diag_gemm_fp8_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.diag_gemm_ck_path.argtypes = [ctypes.c_int] * 3
        L.diag_gemm_ck_path.restype = ctypes.c_int
        L.diag_gemm_launch_ck.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.diag_hbm_bandwidth.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int] + \
            [ctypes.POINTER(ctypes.c_double)] * 3
        L.diag_memtest.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong),
                                   ctypes.POINTER(ctypes.c_double)]
        L.diag_mfma_burn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_ulonglong)]
        L.diag_mfma_burn_map.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_ulonglong),
                                         ctypes.POINTER(ctypes.c_ulonglong)]
        L.diag_mfma_burn_slots.restype = ctypes.c_int
        L.diag_l2_bandwidth.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_ulonglong),
                                        ctypes.POINTER(ctypes.c_ulonglong)]
        L.diag_hbm_xcd.argtypes = list(L.diag_l2_bandwidth.argtypes) + [ctypes.POINTER(ctypes.c_double)]
        L.diag_lds_test.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong),
                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)]
        L.diag_host_link.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double)]
        L.diag_p2p_copy.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_ulonglong),
                                    ctypes.POINTER(ctypes.c_int)]
        L.diag_memtest_x.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int, ctypes.c_longlong,
                                     ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong),
                                     ctypes.POINTER(ctypes.c_double)]
        L.diag_poll_selftest.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_int),
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.diag_p2p_copy_t.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_double,
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_ulonglong),
                                      ctypes.POINTER(ctypes.c_int)]
        L.diag_p2p_fan_t.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_size_t,
                                     ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_int),
                                     ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != 0:
        raise RuntimeError(f"mi355x diag failed ({rc}): {lib().diag_last_error().decode(errors='replace')}")


def device_count() -> int:
    return int(lib().diag_device_count())


def device_info(device: int = 0) -> Dict[str, Any]:
    buf = ctypes.create_string_buffer(512)
    _check(lib().diag_device_arch(device, buf, len(buf)))
    arch, name, cus, mem, bdf = buf.value.decode().split("|")
    return {"arch": arch, "name": name, "cus": int(cus), "mem_bytes": int(mem), "bdf": bdf}


GEMM_VARIANTS = {"auto": 0, "v1": 1, "v2": 2, "v3": 3, "v4": 4, "v4t": 5}


def set_gemm_variant(variant: str = "auto") -> None:
    """Select the bf16 GEMM kernel: ``auto`` (v4 for 256-multiples that fill the chip, else v1),
    ``v1`` 128x128 register-staged, ``v2`` 256x256 LDS-DMA, ``v3`` 256x256 staggered LDS-DMA (8 waves),
    ``v4`` 256x256 with 4 waves of 128x128 and the loop's instruction order written out (diag.hip
    ``gemm_v4_kernel``).  v2-v4 need M, N multiples of 256.  fp8 / fp4 GEMMs always run v3."""
    lib().diag_set_gemm_variant(GEMM_VARIANTS[variant])


def set_gemm_epilogue(lds_staged: bool) -> None:
    """v3 kernels: write C with 4-byte stores straight from the MFMA layout (False) or staged
    through LDS as 16-byte row pieces (True)."""
    lib().diag_set_gemm_epilogue(1 if lds_staged else 0)


def set_gemm_buffer_loads(buffer_loads: bool) -> None:
    """v3 kernels: stage operands with ``global_load_lds_dwordx4`` (False) or ``buffer_load_dwordx4 ...
    lds`` from two per-tile buffer resources (True: loop-invariant per-lane offsets, the K step in a
    scalar register)."""
    lib().diag_set_gemm_buffer_loads(1 if buffer_loads else 0)


def set_gemm_schedule(schedule: int) -> None:
    """v3 kernels: the K-tile phase that issues each LDS-DMA restaging piece (``V3_PHASE`` in diag.hip):
    1 (default) = 0/2/2/4 pieces over the four phases, 0 = the earlier 2/0/4/2 order, kept for A/B."""
    if schedule not in (0, 1):
        raise ValueError(f"gemm schedule must be 0 or 1, not {schedule!r}")
    lib().diag_set_gemm_schedule(schedule)


def set_gemm_fp8_unscaled(unscaled: bool) -> None:
    """fp8 v3 GEMMs: the MFMA form -- the unscaled ``v_mfma_f32_16x16x128_f8f6f4`` hipBLASLt's fp8 GEMMs issue
    (True, the default: 5.6 % faster, 92 % of hipBLASLt at 8192^3) or ``v_mfma_scale_f32_16x16x128_f8f6f4`` with
    unit E8M0 scales (False, the MX path).  Unit scales make the two compute the same products (bit-identical C);
    the knob picks the matrix-core path timed.  Per calling thread."""
    lib().diag_set_gemm_fp8_unscaled(1 if unscaled else 0)


def get_gemm_fp8_unscaled() -> bool:
    f = getattr(lib(), "diag_get_gemm_fp8_unscaled", None)  # (absent from the test doubles of the library)
    return bool(f()) if f is not None else True


def set_gemm_tail(tail: bool) -> None:
    """v4 (bf16 and fp8): run a short last wave of 256x256 tiles (at most a quarter of the chip's 256 CUs, e.g.
    6144^3's 576 tiles) as 128x128 quadrants with v1's K loop (True, the default) or leave it to v4 (False, kept for
    A/B).  C and the fused column sums are bit-identical either way.  Per calling thread."""
    lib().diag_set_gemm_tail(1 if tail else 0)


def get_gemm_tail() -> bool:
    f = getattr(lib(), "diag_get_gemm_tail", None)  # (absent from the test doubles of the library)
    return bool(f()) if f is not None else True


def get_gemm_config() -> Dict[str, Any]:
    """The calling thread's GEMM knobs (they are thread-local in the library: every agent thread
    starts from the production defaults ``auto`` / LDS-staged epilogue / ``global_load_lds`` / schedule 1)."""
    L = lib()
    inv = {v: k for k, v in GEMM_VARIANTS.items()}
    return {"variant": inv.get(int(L.diag_get_gemm_variant()), "auto"),
            "epilogue": bool(L.diag_get_gemm_epilogue()),
            "buffer_loads": bool(L.diag_get_gemm_buffer_loads()),
            "schedule": int(L.diag_get_gemm_schedule()),
            "fp8_unscaled": get_gemm_fp8_unscaled(), "tail": get_gemm_tail()}


def get_gemm_epilogue() -> bool:
    return bool(lib().diag_get_gemm_epilogue())


class gemm_config:
    """``with gemm_config(variant="v3", epilogue=False): ...`` -- set knobs for the calling thread
    and restore the previous values on exit (not the library defaults)."""

    def __init__(self, variant: Optional[str] = None, epilogue: Optional[bool] = None,
                 buffer_loads: Optional[bool] = None, schedule: Optional[int] = None,
                 fp8_unscaled: Optional[bool] = None, tail: Optional[bool] = None):
        self.want = {"variant": variant, "epilogue": epilogue, "buffer_loads": buffer_loads, "schedule": schedule,
                     "fp8_unscaled": fp8_unscaled, "tail": tail}
        self.saved: Dict[str, Any] = {}

    @staticmethod
    def _apply(cfg: Dict[str, Any]) -> None:
        if cfg.get("variant") is not None:
            set_gemm_variant(cfg["variant"])
        if cfg.get("epilogue") is not None:
            set_gemm_epilogue(cfg["epilogue"])
        if cfg.get("buffer_loads") is not None:
            set_gemm_buffer_loads(cfg["buffer_loads"])
        if cfg.get("schedule") is not None:
            set_gemm_schedule(cfg["schedule"])
        if cfg.get("fp8_unscaled") is not None:
            set_gemm_fp8_unscaled(cfg["fp8_unscaled"])
        if cfg.get("tail") is not None and getattr(lib(), "diag_set_gemm_tail", None) is not None:
            set_gemm_tail(cfg["tail"])

    def __enter__(self) -> "gemm_config":
        self.saved = get_gemm_config()
        self._apply(self.want)
        return self

    def __exit__(self, *exc: Any) -> None:
        self._apply(self.saved)


def gemm_launch(a_ptr: int, bt_ptr: int, c_ptr: int, m: int, n: int, k: int, stream: int = 0) -> None:
    """Launch the MFMA GEMM on caller-owned device memory: ``C = A @ Bt.T`` (bf16 in, fp32 out)."""
    if m % 128 or n % 128 or k % 64:
        raise ValueError("gemm: M, N must be multiples of 128 and K a multiple of 64")
    _check(lib().diag_gemm_bf16_launch(a_ptr, bt_ptr, c_ptr, m, n, k, stream))


def gemm_fp8_launch(a_ptr: int, bt_ptr: int, c_ptr: int, m: int, n: int, k: int, stream: int = 0) -> None:
    """MX-fp8 GEMM on caller-owned memory: ``C = A @ Bt.T`` with OCP E4M3 operands (1 byte each,
    unit block scales) and fp32 output, on ``v_mfma_scale_f32_16x16x128_f8f6f4``."""
    if m % 256 or n % 256 or k % 128:
        raise ValueError("gemm_fp8: M, N must be multiples of 256 and K a multiple of 128")
    _check(lib().diag_gemm_fp8_launch(a_ptr, bt_ptr, c_ptr, m, n, k, stream))


def gemm_fp4_launch(a_ptr: int, bt_ptr: int, c_ptr: int, m: int, n: int, k: int, stream: int = 0) -> None:
    """MX-fp4 GEMM on caller-owned memory: OCP E2M1 operands packed two per byte (element 2i in the
    low nibble), unit block scales, fp32 ``C = A @ Bt.T``; ``k`` counts elements."""
    if m % 256 or n % 256 or k % 256:
        raise ValueError("gemm_fp4: M, N must be multiples of 256 and K a multiple of 256")
    _check(lib().diag_gemm_fp4_launch(a_ptr, bt_ptr, c_ptr, m, n, k, stream))


def gemm_launch_ck(dtype: str, a_ptr: int, bt_ptr: int, c_ptr: int, csum_ptr: int, m: int, n: int, k: int,
                   stream: int = 0) -> None:
    """The kernel the ``gemm`` / ``gemm_fp8`` diagnostics time: ``C = A @ Bt.T`` written as bf16 (the output
    hipBLASLt writes) plus ``csum[m // 128][n]`` (fp64), each column's sum over every 128-row block formed from
    the fp32 accumulators.  ``dtype`` ``"bf16"`` or ``"fp8"`` (OCP E4M3, unit block scales); 256-multiples."""
    dt = {"bf16": 0, "fp8": 1}[dtype]
    if m % 256 or n % 256 or k % (128 if dt else 64):
        raise ValueError("gemm_ck: M, N must be multiples of 256 and K of 64 (bf16) or 128 (fp8)")
    _check(lib().diag_gemm_launch_ck(dt, a_ptr, bt_ptr, c_ptr, csum_ptr, m, n, k, stream))


def _ref(test: str, key: Any, scale: float) -> float:
    table = REFERENCE_RATES[test]
    if key not in table:  # a size without its own measurement: the nearest measured one
        key = min(table, key=lambda k: abs(k - key))
    return table[key] * scale


def _checked_gemm(fn: str, device: int, size: int, warmup: int, iters: int, samples: int,
                  inject_elem: Optional[int], ck_tol: float) -> Tuple[float, float, float, float, List[int]]:
    tf, err, ms, ck = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    out = (ctypes.c_longlong * 12)()
    _check(getattr(lib(), fn)(device, size, size, size, warmup, iters, samples,
                              -1 if inject_elem is None else int(inject_elem), ck_tol, ctypes.byref(tf),
                              ctypes.byref(err), ctypes.byref(ms), ctypes.byref(ck), out))
    return tf.value, err.value, ms.value, ck.value, list(out)


def _gemm_output(dt: int, size: int) -> str:
    """What the timed GEMM wrote (the library decides, under this thread's knobs): ``bf16+colsums`` -- bf16 C,
    what hipBLASLt writes, with the column sums formed in the kernel -- or ``fp32``."""
    probe = getattr(lib(), "diag_gemm_ck_path", None)  # (absent from the test doubles of the library)
    if probe is None:
        return "unknown"
    return "bf16+colsums" if probe(dt, size, size) else "fp32"


def _checksum_verdict(res: Dict[str, Any], ck_err: float, out: List[int], tol: float) -> str:
    """Record the tile checksums in ``res``; a non-empty string describes the tiles that failed them."""
    res["checksum_err"] = ck_err
    res["checksum_bad_tiles"] = out[0]
    if not out[0]:
        return ""
    xcds = {x: n for x, n in enumerate(out[2:10]) if n}
    res["checksum_bad_columns"] = out[1]
    res["checksum_bad_xcds"] = {str(x): n for x, n in xcds.items()}
    res["checksum_first_bad_tile"] = [out[10], out[11]]
    where = ", ".join(f"XCD {x}: {n}" for x, n in xcds.items())
    return (f"{out[0]} output tile(s) fail their checksums ({where}; first at tile row {out[10]}, column "
            f"{out[11]}; err {ck_err:.2e} > {tol:g})")


def gemm(device: int = 0, size: int = 8192, warmup: int = 3, iters: int = 20, samples: int = 4096,
         scale: Scale = FULL, inject_elem: Optional[int] = None) -> Dict[str, Any]:
    """bf16 GEMM burn-in: rate, sampled fp32-reference error, and every output tile checked by its column
    checksums (a bad tile is named with the XCD that computed it).  ``inject_elem`` (a test hook) overwrites
    that output between the timing and the checks.

    At 256-multiple sizes that fill the chip the timed kernel writes bf16 C -- the output hipBLASLt writes, so
    the rate compares like for like -- and forms the column sums itself, in fp64 from its fp32 accumulators
    (``gemm_launch_ck``); the sampled error is then what lies beyond the bf16 rounding of the output."""
    t0 = time.perf_counter()
    tf, err, ms, ck, out = _checked_gemm("diag_gemm_bf16_x", device, size, warmup, iters, samples, inject_elem,
                                         GEMM_CK_TOL)
    res = {"tflops": round(tf, 1), "max_rel_err": err, "ms_per_gemm": round(ms, 4),
           "shape": [size, size, size], "output": _gemm_output(0, size),
           "wall_s": round(time.perf_counter() - t0, 3)}
    problems = [f"rel err {err:.2e} > {GEMM_MAX_REL_ERR:g}"] if not err <= GEMM_MAX_REL_ERR else []
    bad = _checksum_verdict(res, ck, out, GEMM_CK_TOL)
    problems += [bad] if bad else []
    return _rated(res, {"tflops": tf}, {"tflops": _ref("gemm", size, scale.compute)}, "TFLOP/s",
                  not problems, "; ".join(problems))


def gemm_fp8(device: int = 0, size: int = 8192, warmup: int = 3, iters: int = 20,
             samples: int = 4096, scale: Scale = FULL, inject_elem: Optional[int] = None) -> Dict[str, Any]:
    """MX-fp8 GEMM burn-in: rate, sampled fp64-reference error (normalised by sum|a*b|) and the tile
    checksums of every output, as ``gemm`` (bf16 C with fused column sums)."""
    t0 = time.perf_counter()
    tf, err, ms, ck, out = _checked_gemm("diag_gemm_fp8_x", device, size, warmup, iters, samples, inject_elem,
                                         GEMM_FP8_CK_TOL)
    res = {"tflops": round(tf, 1), "max_err_over_mag": err, "ms_per_gemm": round(ms, 4),
           "shape": [size, size, size], "output": _gemm_output(1, size),
           "wall_s": round(time.perf_counter() - t0, 3)}
    problems = [f"err {err:.2e} > {GEMM_FP8_MAX_ERR:g}"] if not err <= GEMM_FP8_MAX_ERR else []
    bad = _checksum_verdict(res, ck, out, GEMM_FP8_CK_TOL)
    problems += [bad] if bad else []
    return _rated(res, {"tflops": tf}, {"tflops": _ref("gemm_fp8", size, scale.compute)}, "TFLOP/s",
                  not problems, "; ".join(problems))


def hbm(device: int = 0, gib: float = 4.0, iters: int = 10, scale: Scale = FULL) -> Dict[str, Any]:
    c, r, w = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    t0 = time.perf_counter()
    _check(lib().diag_hbm_bandwidth(device, int(gib * (1 << 30)), iters, ctypes.byref(c), ctypes.byref(r),
                                    ctypes.byref(w)))
    res = {"copy_tbs": round(c.value, 3), "read_tbs": round(r.value, 3), "write_tbs": round(w.value, 3),
           "gib": gib, "wall_s": round(time.perf_counter() - t0, 3)}
    exp = {k: v * scale.memory for k, v in REFERENCE_RATES["hbm"].items()}
    return _rated(res, {"copy_tbs": c.value, "read_tbs": r.value}, exp, "TB/s")


def memtest(device: int = 0, gib: float = 8.0, passes: int = 1, seed: int = 0x5EED,
            inject_word: Optional[int] = None) -> Dict[str, Any]:
    """Pattern + inverse over ``gib`` of HBM, every word checked.  ``inject_word`` (a test hook) overwrites that
    16-byte word between the first write and its check, to show a corrupted word is counted and located."""
    errs, first, gbps = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_double()
    t0 = time.perf_counter()
    if inject_word is None:
        _check(lib().diag_memtest(device, int(gib * (1 << 30)), seed, passes, ctypes.byref(errs),
                                  ctypes.byref(first), ctypes.byref(gbps)))
    else:
        _check(lib().diag_memtest_x(device, int(gib * (1 << 30)), seed, passes, inject_word, ctypes.byref(errs),
                                    ctypes.byref(first), ctypes.byref(gbps)))
    ok = errs.value <= MEMTEST_MAX_ERRORS
    res: Dict[str, Any] = {"pass": ok, "errors": errs.value, "gib": gib, "passes": passes,
                           "gbps": round(gbps.value, 1), "wall_s": round(time.perf_counter() - t0, 3),
                           "detail": "" if ok else f"{errs.value} bad 16-byte words"}
    if errs.value:
        res["first_bad_byte"] = first.value
    return res


def slot_name(slot: int) -> str:
    """``xcd3/se1/cu5`` (``/sh1`` when the wave sat in shader array 1) of a burn-in CU slot
    (``wave_slot()`` in csrc/diag/diag.hip: xcd<<7 | se<<5 | sh<<4 | cu)."""
    sh = (slot >> 4) & 1
    return f"xcd{slot >> 7}/se{(slot >> 5) & 3}/cu{slot & 15}" + ("/sh1" if sh else "")


def cu_map_summary(maps: Dict[str, Any]) -> Dict[str, Any]:
    """Fold the burn-in's per-CU tables (kind -> flat [waves, wrong lanes, wave ticks] x slots) into
    where the work ran and how each XCD kept up.

    * ``cus``: distinct physical CUs that ran waves; ``xcds``: per XCD its CUs and ``rel_time``, its
      mean wave time over the median XCD's (median over the precisions, so one noisy kind does not
      move it);
    * ``bad_cus``: CUs with wrong results and the kinds they got wrong -- a miscomputing matrix core is
      named down to its CU, so the node can be drained with the fault located;
    * ``slowest_xcd`` / ``slowest_rel``: the XCD furthest behind (each XCD is its own clock domain).
    """
    per_kind_rel: Dict[int, List[float]] = {}
    per_cu_rel: Dict[int, List[float]] = {}
    cu_waves: Dict[int, List[int]] = {}
    cus: Dict[int, set] = {}
    bad: Dict[int, Dict[str, int]] = {}
    for kind, flat in maps.items():
        waves: Dict[int, int] = {}
        ticks: Dict[int, int] = {}
        cu_mean: Dict[int, float] = {}
        for slot in range(len(flat) // 3):
            w, e, t = flat[3 * slot], flat[3 * slot + 1], flat[3 * slot + 2]
            if not w:
                continue
            x = slot >> 7
            cus.setdefault(x, set()).add(slot)
            waves[x] = waves.get(x, 0) + w
            ticks[x] = ticks.get(x, 0) + t
            cu_mean[slot] = t / w
            cu_waves.setdefault(slot, []).append(int(w))
            if e:
                bad.setdefault(slot, {})[kind] = int(e)
        mean = {x: ticks[x] / waves[x] for x in waves if waves[x]}
        if mean:
            med = sorted(mean.values())[len(mean) // 2]
            for x, m in mean.items():
                per_kind_rel.setdefault(x, []).append(m / med if med > 0 else 1.0)
        # each CU against the median CU of its own XCD, so a whole XCD running behind (reported above)
        # does not also name its CUs
        by_xcd: Dict[int, List[float]] = {}
        for slot, m in cu_mean.items():
            by_xcd.setdefault(slot >> 7, []).append(m)
        xmed = {x: sorted(v)[len(v) // 2] for x, v in by_xcd.items()}
        for slot, m in cu_mean.items():
            med = xmed[slot >> 7]
            per_cu_rel.setdefault(slot, []).append(m / med if med > 0 else 1.0)
    xcds = {}
    for x in sorted(cus):
        rels = sorted(per_kind_rel.get(x, [1.0]))
        xcds[str(x)] = {"cus": len(cus[x]), "rel_time": round(rels[len(rels) // 2], 3)}
    out: Dict[str, Any] = {"cus": sum(len(v) for v in cus.values()), "xcds": xcds}
    if len(xcds) >= 2:
        slow = max(xcds, key=lambda k: xcds[k]["rel_time"])
        out["slowest_xcd"], out["slowest_rel"] = int(slow), xcds[slow]["rel_time"]
    if per_cu_rel:
        # the CU furthest behind its XCD's median CU (median over the kinds), and how evenly the hardware
        # dealt the workgroups out (waves per CU per kind, min..max)
        rel_cu = {slot: sorted(r)[len(r) // 2] for slot, r in per_cu_rel.items()}
        worst = max(rel_cu, key=rel_cu.get)
        out["slowest_cu"], out["slowest_cu_rel"] = slot_name(worst), round(rel_cu[worst], 3)
        ws = [w for lst in cu_waves.values() for w in lst]
        out["waves_per_cu"] = [min(ws), max(ws)]
    if bad:
        out["bad_cus"] = [f"{slot_name(s)} (" + ", ".join(f"{k} {n}" for k, n in kinds.items()) + ")"
                          for s, kinds in sorted(bad.items())]
    return out


def mfma_burn(device: int = 0, kinds=MFMA_KINDS, iters: int = 2000, reps: int = 5,
              scale: Scale = FULL) -> Dict[str, Any]:
    """Every matrix-core precision of the MI355X: dense TFLOP/s and exact-result errors per kind, plus
    where on the chip the waves ran (:func:`cu_map_summary`): the CU behind any wrong result, and an XCD
    whose waves fall more than ``XCD_SLOW_RATIO`` behind the others (degraded)."""
    t0 = time.perf_counter()
    rows: Dict[str, Any] = {}
    rates: Dict[str, float] = {}
    wrong = []
    L = lib()
    nslots = L.diag_mfma_burn_slots()
    maps: Dict[str, Any] = {}
    for kind in kinds:
        tf, errs = ctypes.c_double(), ctypes.c_ulonglong()
        m = (ctypes.c_ulonglong * (3 * nslots))()
        _check(L.diag_mfma_burn_map(device, MFMA_KINDS.index(kind), iters, reps, ctypes.byref(tf),
                                    ctypes.byref(errs), m))
        maps[kind] = list(m)
        rows[kind] = {"tflops": round(tf.value, 1), "errors": errs.value}
        rates[kind] = tf.value
        if errs.value:
            wrong.append(f"{kind}: {errs.value} wrong results")
    where = cu_map_summary(maps)
    if where.get("bad_cus"):
        wrong.append("on " + ", ".join(where["bad_cus"][:4]) + (" ..." if len(where["bad_cus"]) > 4 else ""))
    exp = {k: REFERENCE_RATES["mfma"][k] * scale.compute for k in kinds}
    res = _rated({"kinds": rows, "map": where, "wall_s": round(time.perf_counter() - t0, 3)}, rates, exp,
                 "TFLOP/s", not wrong, "; ".join(wrong))
    return _lag_verdict(res, where, "waves")


def _lag_notes(where: Dict[str, Any], what: str) -> List[str]:
    """An XCD, or a single CU, falling behind the rest of the chip on identical work (cu_map_summary).
    The per-CU comparison needs an even deal of workgroups (measured: every CU gets the same count);
    with an uneven one the co-resident waves differ and the times are not comparable."""
    notes = []
    rel = where.get("slowest_rel")
    if isinstance(rel, float) and rel > XCD_SLOW_RATIO:
        notes.append(f"xcd{where['slowest_xcd']} {what} take {rel:.2f}x the median XCD's time")
    crel, wpc = where.get("slowest_cu_rel"), where.get("waves_per_cu")
    if isinstance(crel, float) and crel > CU_SLOW_RATIO and isinstance(wpc, list) and wpc[0] == wpc[-1]:
        notes.append(f"{where['slowest_cu']} {what} take {crel:.2f}x its XCD's median CU's time")
    return notes


def _lag_verdict(res: Dict[str, Any], where: Dict[str, Any], what: str) -> Dict[str, Any]:
    notes = _lag_notes(where, what)
    if notes:
        res["lag"] = notes
        judge_absolute(res)
    return res


def lds_test(device: int = 0, rounds: int = 4, seed: int = 0x1D5, inject_block: int = -1) -> Dict[str, Any]:
    """Every CU's whole LDS (160 KiB on gfx950) under four patterns, each word read back by another
    thread than its writer; errors are located to their CU.  ``inject_block`` corrupts one word of that
    workgroup (self-check of the detection path)."""
    L = lib()
    nslots = L.diag_mfma_burn_slots()
    errs, nbytes, ms = ctypes.c_ulonglong(), ctypes.c_int(), ctypes.c_double()
    m = (ctypes.c_ulonglong * (2 * nslots))()
    t0 = time.perf_counter()
    _check(L.diag_lds_test(device, rounds, seed, inject_block, ctypes.byref(errs), m, ctypes.byref(nbytes),
                           ctypes.byref(ms)))
    cus = [s for s in range(nslots) if m[2 * s]]
    bad = [f"{slot_name(s)} ({m[2 * s + 1]} words)" for s in cus if m[2 * s + 1]]
    res: Dict[str, Any] = {"pass": errs.value == 0, "errors": errs.value, "cus": len(cus),
                           "bytes_per_cu": nbytes.value, "workgroups": sum(m[2 * s] for s in cus),
                           "ms": round(ms.value, 3), "wall_s": round(time.perf_counter() - t0, 3), "detail": ""}
    if bad:
        res["bad_cus"] = bad
    if errs.value:
        res["detail"] = f"{errs.value} LDS words wrong on " + ", ".join(bad[:4]) + (" ..." if len(bad) > 4 else "")
    return res


def l2_bandwidth(device: int = 0, slice_kib: int = 2048, passes: int = 32, blocks_per_cu: int = 8,
                 seed: int = 0x12C3, scale: Scale = FULL) -> Dict[str, Any]:
    """Each XCD's 4 MiB L2, read by that XCD's own CUs (a ``slice_kib`` slice per XCD, every word checked):
    aggregate TB/s against the reference, per-XCD wave time against the median XCD (degraded beyond
    ``XCD_SLOW_RATIO``: an L2 that lost ways or a slow XCD), wrong words located to the CU."""
    L = lib()
    nslots = L.diag_mfma_burn_slots()
    tbs, errs = ctypes.c_double(), ctypes.c_ulonglong()
    m = (ctypes.c_ulonglong * (3 * nslots))()
    t0 = time.perf_counter()
    _check(L.diag_l2_bandwidth(device, slice_kib << 10, passes, blocks_per_cu, seed, ctypes.byref(tbs),
                               ctypes.byref(errs), m))
    where = cu_map_summary({"l2": list(m)})
    wrong = f"{errs.value} wrong words on " + ", ".join(where.get("bad_cus", [])[:4]) if errs.value else ""
    exp = {"read_tbs": REFERENCE_RATES["l2"]["read_tbs"] * scale.compute}
    res = _rated({"read_tbs": round(tbs.value, 2), "errors": errs.value, "map": where,
                  "wall_s": round(time.perf_counter() - t0, 3)}, {"read_tbs": tbs.value}, exp, "TB/s",
                 not errs.value, wrong)
    return _lag_verdict(res, where, "L2 reads")


def hbm_xcd(device: int = 0, slice_mib: int = 256, passes: int = 4, blocks_per_cu: int = 4,
            seed: int = 0x4B3D, scale: Scale = FULL) -> Dict[str, Any]:
    """HBM reads per XCD.  Each XCD streams its own ``slice_mib`` slice (8 of them, far past the L2s and the
    MALL) with its own workgroups, every word checked: first all XCDs together (aggregate read TB/s), then
    each XCD alone (``alone_tbs``: that XCD's own path to the memory stacks).  All XCDs together saturate
    HBM, so the aggregate hides one slow XCD; alone, every XCD of a healthy MI355X reads at 1.28-1.33 TB/s
    (spread < 3 %, profiles/hbm_xcd_explore_mi355x.json).  Judged: the aggregate against the HBM-read
    reference, the slowest XCD alone against the per-XCD reference, and an XCD below
    ``XCD_ALONE_MIN_RATIO`` of the median XCD is degraded even when above the floor."""
    L = lib()
    nslots = L.diag_mfma_burn_slots()
    tbs, errs = ctypes.c_double(), ctypes.c_ulonglong()
    m = (ctypes.c_ulonglong * (3 * nslots))()
    alone = (ctypes.c_double * 8)()
    t0 = time.perf_counter()
    _check(L.diag_hbm_xcd(device, slice_mib << 20, passes, blocks_per_cu, seed, ctypes.byref(tbs),
                          ctypes.byref(errs), m, alone))
    where = cu_map_summary({"hbm_xcd": list(m)})
    # under contention the XCDs' shares of HBM are not even (measured 1.02-1.29x between runs): reported only
    where = {k: v for k, v in where.items() if k in ("cus", "xcds", "bad_cus")}
    per = {x: alone[x] for x in range(8) if alone[x] > 0}
    res: Dict[str, Any] = {"read_tbs": round(tbs.value, 3), "errors": errs.value,
                           "alone_tbs": {str(x): round(v, 3) for x, v in per.items()}, "map": where}
    rates = {"read_tbs": tbs.value}
    exp = {"read_tbs": REFERENCE_RATES["hbm_xcd"]["read_tbs"] * scale.memory}
    notes = []
    if per:
        slow = min(per, key=per.get)
        med = sorted(per.values())[len(per) // 2]
        res["slowest_xcd"], res["slowest_xcd_rel"] = slow, round(per[slow] / med, 3) if med > 0 else None
        rates["slowest_xcd_tbs"] = per[slow]
        exp["slowest_xcd_tbs"] = min(REFERENCE_RATES["hbm_xcd"]["alone_tbs"], exp["read_tbs"])
        if med > 0 and per[slow] < XCD_ALONE_MIN_RATIO * med:
            notes.append(f"xcd{slow} reads HBM at {per[slow]:.2f} TB/s alone, {per[slow] / med:.2f}x the median XCD")
    wrong = f"{errs.value} wrong words on " + ", ".join(where.get("bad_cus", [])[:4]) if errs.value else ""
    res["wall_s"] = round(time.perf_counter() - t0, 3)
    if notes:
        res["lag"] = notes
    return _rated(res, rates, exp, "TB/s", not errs.value, wrong)


def host_link(device: int = 0, mib: int = 256, iters: int = 5, scale: Scale = FULL) -> Dict[str, Any]:
    """Pinned host <-> device bandwidth over the GPU's PCIe link (GB/s each way).  A Gen4 or x8 link
    lands at about half the Gen5 x16 reference and fails."""
    h2d, d2h = ctypes.c_double(), ctypes.c_double()
    t0 = time.perf_counter()
    _check(lib().diag_host_link(device, mib << 20, iters, ctypes.byref(h2d), ctypes.byref(d2h)))
    res = {"h2d_gbps": round(h2d.value, 1), "d2h_gbps": round(d2h.value, 1),
           "wall_s": round(time.perf_counter() - t0, 3)}
    exp = {k: v * scale.compute for k, v in REFERENCE_RATES["host_link"].items()}
    return _rated(res, {"h2d_gbps": h2d.value, "d2h_gbps": d2h.value}, exp, "GB/s")


def poll_selftest(device: int = 0, launches: int = 1000, deadline_ms: float = 20.0) -> Dict[str, Any]:
    """The polled deadline the xGMI pair copies wait with, shown on one GPU: ``launches`` queued 1 GiB writes
    waited for with a ``deadline_ms`` deadline (``timed_out``: the deadline came first), then drained."""
    t, w, d = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
    _check(lib().diag_poll_selftest(device, launches, deadline_ms, ctypes.byref(t), ctypes.byref(w), ctypes.byref(d)))
    return {"timed_out": bool(t.value), "waited_ms": round(w.value, 3), "drained_ms": round(d.value, 3)}


P2P_HUNG = -4  # diag_p2p_copy_t: the copies (or their verification) missed the deadline


def p2p_copy(src: int, dst: int, mib: int = 256, iters: int = 5, timeout_s: Optional[float] = None) -> Dict[str, Any]:
    """One ordered GPU pair: copy bandwidth over xGMI (GB/s) and pattern errors on arrival.

    With ``timeout_s`` the native side polls for completion and gives up at the deadline: the pair comes back
    ``{"hung": True, ...}`` (its buffers stay allocated, as an in-flight copy may still write them) rather than
    blocking the caller on a link that stopped making progress."""
    gbps, errs, peer = ctypes.c_double(), ctypes.c_ulonglong(), ctypes.c_int()
    ms = 0.0 if not timeout_s else max(1.0, 1000.0 * timeout_s)
    rc = lib().diag_p2p_copy_t(src, dst, mib << 20, iters, ms, ctypes.byref(gbps), ctypes.byref(errs),
                               ctypes.byref(peer))
    if rc == P2P_HUNG:
        return {"src": src, "dst": dst, "gbps": 0.0, "errors": 0, "peer": bool(peer.value), "hung": True,
                "detail": lib().diag_last_error().decode(errors="replace")}
    _check(rc)
    return {"src": src, "dst": dst, "gbps": round(gbps.value, 1), "errors": errs.value, "peer": bool(peer.value)}


def link_gbs(width: Any = None, speed_gbps: Any = None) -> float:
    """One direction of one xGMI link in GB/s from its trained lanes and per-lane rate (amd-smi), the MI355X's x16 at
    38 Gb/s for whichever is unknown."""
    from ..models.health import XGMI_LINK_GBPS, XGMI_LINK_WIDTH
    w = width if isinstance(width, int) and not isinstance(width, bool) and width > 0 else XGMI_LINK_WIDTH
    sp = speed_gbps if isinstance(speed_gbps, (int, float)) and not isinstance(speed_gbps, bool) and speed_gbps > 0 \
        else XGMI_LINK_GBPS
    return w * sp / 8.0


def p2p_fan(src: int, dsts: List[int], mib: int = 256, iters: int = 5,
            timeout_s: Optional[float] = None) -> Dict[str, Any]:
    """``src`` copying to every one of ``dsts`` at once (all its links loaded together): per destination the GB/s it
    saw, pattern errors and peer access, and the source's total.  ``{"hung": True, ...}`` at the deadline."""
    n = len(dsts)
    arr = (ctypes.c_int * n)(*dsts)
    gbps, errs, peer = (ctypes.c_double * n)(), (ctypes.c_ulonglong * n)(), (ctypes.c_int * n)()
    total = ctypes.c_double()
    ms = 0.0 if not timeout_s else max(1.0, 1000.0 * timeout_s)
    rc = lib().diag_p2p_fan_t(src, arr, n, mib << 20, iters, ms, gbps, errs, peer, ctypes.byref(total))
    if rc == P2P_HUNG:
        return {"src": src, "hung": True, "detail": lib().diag_last_error().decode(errors="replace"), "to": []}
    _check(rc)
    return {"src": src, "total_gbps": round(total.value, 1),
            "to": [{"dst": d, "gbps": round(gbps[i], 1), "errors": errs[i], "peer": bool(peer[i])}
                   for i, d in enumerate(dsts)]}


def p2p_matrix(devices: Optional[list] = None, mib: int = 256, iters: int = 5,
               timeout_s: Optional[float] = None, link: Optional[float] = None, fan: bool = True) -> Dict[str, Any]:
    """Every ordered pair of ``devices`` (default: all): the node's xGMI fabric, link by link, then (``fan``) every
    source to all its peers at once.

    Pass: every pair has direct peer access, delivers its bytes intact, and runs at no less than
    ``P2P_MIN_FRACTION_OF_MEDIAN`` of the median pair (relative: one slow link among good ones) and no less than
    ``P2P_MIN_FRACTION_OF_LINK`` of ``link`` GB/s (absolute: a hive whose links are all slow alike; ``link`` from the
    training amd-smi reports, :func:`link_gbs`); under the fan every destination delivers intact at no less than
    ``P2P_MIN_FRACTION_OF_MEDIAN`` of the fan's median destination and ``P2P_FAN_MIN_FRACTION_OF_LINK`` of ``link``.

    ``timeout_s`` bounds the whole matrix, both passes: each copy gets what is left of it, and the first that hangs
    ends the matrix (its devices are in an unknown state, with copies possibly still queued behind it), as does a
    deadline that passes between copies; both fail the test and name the pair or the source.
    """
    devs = list(range(device_count())) if devices is None else list(devices)
    t0 = time.perf_counter()
    if len(devs) < 2:
        return {"pass": True, "skipped": f"{len(devs)} GPU(s): no pairs", "pairs": [], "detail": ""}
    link = float(link) if link else link_gbs()
    floor = P2P_MIN_FRACTION_OF_LINK * link
    order = [(a, b) for a in devs for b in devs if a != b]
    pairs: List[Dict[str, Any]] = []
    stopped = ""

    def left() -> Optional[float]:
        return None if not timeout_s else timeout_s - (time.perf_counter() - t0)
    for a, b in order:
        rest = left()
        if rest is not None and rest <= 0:
            stopped = f"deadline of {timeout_s:g} s passed after {len(pairs)}/{len(order)} pairs"
            break
        p = p2p_copy(a, b, mib, iters) if rest is None else p2p_copy(a, b, mib, iters, timeout_s=rest)
        if p.get("hung"):
            stopped = f"{a}->{b} hung: {p['detail']}"
            break
        pairs.append(p)
    rates = sorted(p["gbps"] for p in pairs) or [0.0]
    median = rates[len(rates) // 2]
    slow = [p for p in pairs if p["gbps"] < P2P_MIN_FRACTION_OF_MEDIAN * median]
    under = [p for p in pairs if p["gbps"] < floor and p not in slow]
    bad = [p for p in pairs if p["errors"]]
    nopeer = [p for p in pairs if not p["peer"]]
    problems = (([stopped] if stopped else [])
                + [f"{p['src']}->{p['dst']} {p['gbps']} GB/s" for p in slow]
                + [f"{p['src']}->{p['dst']} {p['gbps']} GB/s under {floor:.0f} GB/s "
                   f"({P2P_MIN_FRACTION_OF_LINK:.0%} of a {link:.0f} GB/s link)" for p in under]
                + [f"{p['src']}->{p['dst']} {p['errors']} bad words" for p in bad]
                + [f"{p['src']}->{p['dst']} no peer access" for p in nopeer])
    out: Dict[str, Any] = {"pairs": pairs, "median_gbps": median, "min_gbps": rates[0], "link_gbps": round(link, 1),
                           "floor_gbps": round(floor, 1)}
    if fan and not stopped:
        fans: List[Dict[str, Any]] = []
        for a in devs:
            rest = left()
            if rest is not None and rest <= 0:
                stopped = f"deadline of {timeout_s:g} s passed after {len(fans)}/{len(devs)} fan sources"
                break
            peers = [b for b in devs if b != a]
            f = p2p_fan(a, peers, mib, iters) if rest is None else p2p_fan(a, peers, mib, iters, timeout_s=rest)
            if f.get("hung"):
                stopped = f"fan from {a} hung: {f['detail']}"
                break
            fans.append(f)
        dests = [dict(t, src=f["src"]) for f in fans for t in f["to"]]
        frates = sorted(t["gbps"] for t in dests) or [0.0]
        fmed = frates[len(frates) // 2]
        ffloor = P2P_FAN_MIN_FRACTION_OF_LINK * link
        fslow = [t for t in dests if t["gbps"] < P2P_MIN_FRACTION_OF_MEDIAN * fmed or t["gbps"] < ffloor]
        fbad = [t for t in dests if t["errors"]]
        if stopped:
            problems.insert(0, stopped)
        problems += ([f"fan {t['src']}->{t['dst']} {t['gbps']} GB/s with every link of {t['src']} busy" for t in fslow]
                     + [f"fan {t['src']}->{t['dst']} {t['errors']} bad words" for t in fbad])
        out["fan"] = {"sources": len(fans), "median_gbps": fmed, "min_gbps": frates[0],
                      "floor_gbps": round(ffloor, 1),
                      "total_gbps": {str(f["src"]): f["total_gbps"] for f in fans}, "to": dests}
    out.update({"pass": not problems, "wall_s": round(time.perf_counter() - t0, 3), "detail": "; ".join(problems[:8])})
    if stopped:
        out["stopped"] = stopped
    return out


LEVELS = {
    0: (),
    1: ("gemm_quick", "gemm_fp8_quick", "hbm_quick", "hbm_xcd", "mfma", "lds", "l2"),
    2: ("gemm", "gemm_fp8", "hbm", "hbm_xcd", "memtest", "mfma", "lds", "l2", "host_link"),
}


def device_scale(device: int = 0, memory_partition: Optional[str] = None,
                 power_fraction: Optional[float] = None) -> Scale:
    """The :class:`Scale` of HIP ``device`` (CU count and memory from HIP; ``memory_partition`` and the power
    cap's share of its default from amd-smi when the caller has them)."""
    info = device_info(device)
    return Scale.of(info.get("cus"), info.get("mem_bytes"), memory_partition, power_fraction)


def _one(test: str, device: int, scale: Scale) -> Dict[str, Any]:
    if test == "gemm_quick":
        return gemm(device, size=4096, warmup=2, iters=10, samples=1024, scale=scale)
    if test == "gemm_fp8_quick":
        return gemm_fp8(device, size=4096, warmup=2, iters=10, samples=1024, scale=scale)
    if test == "gemm_fp8":
        return gemm_fp8(device, scale=scale)
    if test == "hbm_quick":
        return hbm(device, gib=2.0, iters=5, scale=scale)
    if test == "gemm":
        return gemm(device, scale=scale)
    if test == "hbm":
        return hbm(device, scale=scale)
    if test == "memtest":
        return memtest(device)
    if test == "mfma":
        return mfma_burn(device, scale=scale)
    if test == "host_link":
        return host_link(device, scale=scale)
    if test == "lds":
        return lds_test(device)
    if test == "l2":
        return l2_bandwidth(device, scale=scale)
    if test == "hbm_xcd":
        return hbm_xcd(device, scale=scale)
    raise ValueError(f"unknown diagnostic {test!r}")


def _slow_only(res: Dict[str, Any]) -> bool:
    """Below the degraded line on rate alone, or one XCD lagging the others (numerics fine): worth a
    second measurement."""
    lagging = bool(_lag_notes(res.get("map") or {}, "")) or (res.get("slowest_xcd_rel") or 1.0) < XCD_ALONE_MIN_RATIO
    return (res.get("degraded") or not res.get("pass")) \
        and (res.get("fraction", 1.0) < DEGRADED_FRACTION or lagging) and not res.get("numerics") \
        and not any(w in res.get("detail", "") for w in ("wrong results", "err ", "checksums"))


def _goodness(res: Dict[str, Any]) -> tuple:
    """Order two measurements of one test: passing, then not degraded, then the better rate."""
    where = res.get("map") or {}
    return (bool(res.get("pass")), not res.get("degraded"), res.get("fraction", 0.0),
            -max(where.get("slowest_rel") or 0.0, where.get("slowest_cu_rel") or 0.0),
            res.get("slowest_xcd_rel") or 0.0)


def _acquire_shared(device: int, deadline: Optional[float]) -> Optional[str]:
    """Take the host-resource lock for ``device``; None when taken, else why not (the holder and for how long).
    Waits until ``deadline`` (monotonic; default SHARED_WAIT_S from now): one GPU hung inside its host-link
    test must not hold every other GPU's diagnostics past their watchdog and get them all reported hung."""
    wait = SHARED_WAIT_S if deadline is None else max(0.0, deadline - time.monotonic())
    if _HOST_SHARED.acquire(timeout=wait):
        _HOST_HOLDER.update(device=device, since=time.monotonic())
        if _HOST_CELL is not None:
            _HOST_CELL[0], _HOST_CELL[1] = float(device if _HOST_LABEL is None else _HOST_LABEL), time.monotonic()
        return None
    holder = dict(_HOST_HOLDER)
    if _HOST_CELL is not None and _HOST_CELL[0] >= 0:
        holder = {"device": int(_HOST_CELL[0]), "since": _HOST_CELL[1]}
    age = time.monotonic() - holder.get("since", time.monotonic())
    return f"host link held by gpu{holder.get('device', '?')} for {age:.0f} s"


def _release_shared() -> None:
    _HOST_HOLDER.clear()
    if _HOST_CELL is not None:
        _HOST_CELL[0] = -1.0
    _HOST_SHARED.release()


def use_host_lock(lock: Any, cell: Any, label: Optional[int] = None) -> None:
    """Take turns at the SHARED_TESTS with other *processes*: ``lock`` a ``multiprocessing`` lock and ``cell`` a
    shared ``array('d', 2)`` of (holding device, since) that every per-device diagnostic process of one agent cycle
    was given (agent/isolation.py); ``label`` = the node's ordinal of this process's one visible GPU."""
    global _HOST_SHARED, _HOST_CELL, _HOST_LABEL
    _HOST_SHARED, _HOST_CELL, _HOST_LABEL = lock, cell, label


def run(level: int = 1, device: int = 0, scale: Optional[Scale] = None,
        memory_partition: Optional[str] = None, power_fraction: Optional[float] = None,
        deadline: Optional[float] = None) -> Dict[str, Dict[str, Any]]:
    """Run the diagnostics of ``level`` on ``device`` (1 = ~1 s quick check, 2 = deep).

    ``scale`` defaults to the device's own share of a full MI355X (:func:`device_scale`).  A rate that
    lands below the degraded line is measured once more and the better of the two is reported.  Tests of
    host resources (SHARED_TESTS) hold a process-wide lock, so concurrent per-GPU runs take turns there; a device
    that cannot get its turn before ``deadline`` (monotonic) reports that test ``skipped``, naming the holder."""
    out: Dict[str, Dict[str, Any]] = {}
    tests = LEVELS.get(level, ())
    if tests and scale is None:
        try:
            scale = device_scale(device, memory_partition, power_fraction)
        except NativeUnavailable:
            raise
        except Exception:
            scale = FULL
    scale = scale or FULL
    for test in tests:
        name = test.replace("_quick", "")
        shared = name in SHARED_TESTS
        if shared:
            why = _acquire_shared(device, deadline)
            if why is not None:  # not this GPU's finding: the report says whose turn it still is
                out[name] = {"pass": True, "skipped": why, "detail": ""}
                continue
        try:
            res = _one(test, device, scale)
            for _ in range(REMEASURE):
                if not _slow_only(res):
                    break
                again = _one(test, device, scale)
                again["retried"] = True
                if _goodness(again) > _goodness(res):
                    res = again
                else:
                    res["retried"] = True
            if scale is not FULL and (scale.compute < 1.0 or scale.memory < 1.0):
                res["scale"] = scale.to_dict()
            out[name] = res
        except NativeUnavailable:
            raise
        except Exception as e:  # a failing diagnostic is a verdict, not a crash
            out[name] = {"pass": False, "detail": str(e)[:200]}
        finally:
            if shared:
                _release_shared()
    return out


def _summary(test: str, r: Dict[str, Any]) -> str:
    """One line of numbers for a test result (render_text)."""
    if test in ("gemm", "gemm_fp8"):
        return f"{r.get('tflops', 0):.0f} TFLOP/s" + (f" ({r['fraction']:.0%} of reference)" if "fraction" in r else "")
    if test == "hbm":
        return f"copy {r.get('copy_tbs', 0):.2f} / read {r.get('read_tbs', 0):.2f} / write {r.get('write_tbs', 0):.2f} TB/s"
    if test == "mfma":
        m = r.get("map") or {}
        kinds = " · ".join(f"{k} {v.get('tflops', 0):.0f}" for k, v in (r.get("kinds") or {}).items())
        return f"{kinds} TFLOP/s; {m.get('cus', '?')} CUs, XCD spread {m.get('slowest_rel', 1.0):.3f}"
    if test == "lds":
        return f"{r.get('cus', '?')} CUs x {r.get('bytes_per_cu', 0) // 1024} KiB, {r.get('errors', 0)} bad words"
    if test == "l2":
        m = r.get("map") or {}
        return f"{r.get('read_tbs', 0):.1f} TB/s, XCD spread {m.get('slowest_rel', 1.0):.3f}, {r.get('errors', 0)} bad words"
    if test == "memtest":
        return f"{r.get('gib', 0):g} GiB, {r.get('errors', 0)} errors"
    if test == "hbm_xcd":
        alone = r.get("alone_tbs") or {}
        span = f"{min(alone.values()):.2f}-{max(alone.values()):.2f} TB/s per XCD alone" if alone else "no XCD map"
        return f"{r.get('read_tbs', 0):.2f} TB/s all XCDs, {span}, {r.get('errors', 0)} bad words"
    if test == "host_link":
        return f"h2d {r.get('h2d_gbps', 0):.1f} / d2h {r.get('d2h_gbps', 0):.1f} GB/s"
    if test == "p2p":
        if r.get("skipped"):
            return f"skipped ({r['skipped']})"
        fan = r.get("fan") if isinstance(r.get("fan"), dict) else {}
        tail = (f"; fan median {fan.get('median_gbps', 0)} / min {fan.get('min_gbps', 0)} GB/s over {fan.get('sources', 0)}"
                " sources" if fan else "")
        return (f"median {r.get('median_gbps', 0)} / min {r.get('min_gbps', 0)} GB/s over {len(r.get('pairs') or [])} "
                f"pairs (floor {r.get('floor_gbps', '?')}){tail}")
    if test == "rccl":
        rows = r.get("rows") or []
        ops = len({x.get("op") for x in rows})
        if r.get("best_busbw_gbps") is None:
            return f"{r.get('world', '?')} GPU: {ops} collectives' data verified, no bandwidth to judge"
        return f"best busbw {r.get('best_busbw_gbps')} GB/s over {r.get('world', '?')} GPUs, {ops} collectives verified"
    return ""


def render_text(out: Dict[str, Any]) -> str:
    """``mi355x-diag --format text``: one block per GPU, one line per test (PASS / DEGRADED / FAIL, the
    numbers, and the detail of anything not passing), then the node-level fabric and the result."""
    lines = []
    for d, dev in out.get("devices", {}).items():
        info = dev.get("info") or {}
        mem = info.get("mem_bytes")
        head = [f"GPU {d}", info.get("bdf", ""), info.get("name", ""), info.get("arch", "").split(":")[0],
                f"{info.get('cus', '?')} CUs", f"{mem / (1 << 30):.0f} GiB" if isinstance(mem, int) else ""]
        lines.append("  ".join(x for x in head if x))
        for test, r in (dev.get("tests") or {}).items():
            if r.get("skipped"):
                lines.append(f"  {test:<10} {'SKIPPED':<9} {r['skipped']}")
                continue
            state = "FAIL" if not r.get("pass") else ("DEGRADED" if r.get("degraded") else "pass")
            peers = r.get("peers") if isinstance(r.get("peers"), dict) else {}
            ratios = [v for v in (peers.get("ratio") or {}).values() if isinstance(v, (int, float))]
            vs = f"  (x{min(ratios):.2f} vs the other {peers.get('gpus', 0) - 1} GPUs)" if ratios else ""
            lines.append(f"  {test:<10} {state:<9} {_summary(test, r)}{vs}")
            if state != "pass" and r.get("detail"):
                lines.append(f"  {'':<10} {'':<9} {r['detail']}")
    for test, r in (out.get("fabric") or {}).items():
        state = "FAIL" if not r.get("pass") else "pass"
        lines.append(f"fabric {test:<5} {state:<9} {_summary(test, r)}" + (f"  {r['detail']}" if r.get("detail") else ""))
    for w in (out.get("node") or {}).get("warnings") or []:
        lines.append(f"node   DEGRADED  {w}")
    lines.append(f"result: {'PASS' if out.get('pass') else 'FAIL'}")
    return "\n".join(lines) + "\n"


def run_devices(level: int, devices: List[int], parallel: int = 8) -> Dict[int, Dict[str, Dict[str, Any]]]:
    """:func:`run` on every device, at most ``parallel`` at once (one host thread per GPU, as the node agent
    runs them; host-resource tests still take turns under their lock).  A device whose run raised reports it
    as a failed ``run`` test instead of losing the other devices' results."""
    out: Dict[int, Dict[str, Dict[str, Any]]] = {}
    missing: List[NativeUnavailable] = []  # no library at all: raised in the caller's thread, not per device

    def one(d: int) -> None:
        try:
            out[d] = run(level, d)
        except NativeUnavailable as e:
            missing.append(e)
        except Exception as e:  # a broken device: a failed test, not a lost report
            out[d] = {"run": {"pass": False, "detail": f"{type(e).__name__}: {e}"[:200]}}
    if parallel <= 1 or len(devices) <= 1:
        for d in devices:
            one(d)
    else:
        queue = list(devices)
        while queue:
            batch, queue = queue[:parallel], queue[parallel:]
            threads = [threading.Thread(target=one, args=(d,), name=f"diag-gpu{d}", daemon=True) for d in batch]
            for t in threads:
                t.start()
            for t in threads:
                t.join()
    if missing:
        raise missing[0]
    return {d: out[d] for d in devices}


# share of a node-level deadline the xGMI pair matrix may use before the RCCL suite (an 8-GPU matrix is 56 pairs of
# 6 x 256 MiB copies plus a verify pass each, then 8 fans of 7 such copies at once: seconds at xGMI rates, far inside
# 0.45 x the agent's 300 s default)
P2P_SHARE = 0.45


def fabric_tests(devices: List[int], p2p: bool = True, rccl: bool = True,
                 timeout_s: Optional[float] = None, link: Optional[float] = None) -> Dict[str, Any]:
    """The node-level tests of level 2: the xGMI pair matrix (within ``P2P_SHARE`` of ``timeout_s``) and the RCCL
    collectives (within what is left up to 90 %, aborted at that deadline); without a timeout both wait as long
    as they take.  A test that raises is reported as failed; only a missing diag library propagates."""
    import time as _time
    out: Dict[str, Any] = {}
    t0 = _time.monotonic()
    if p2p:
        try:
            out["p2p"] = p2p_matrix(devices, timeout_s=P2P_SHARE * timeout_s if timeout_s else None, link=link)
        except NativeUnavailable:
            raise
        except Exception as e:  # a pair that errors out is a failed fabric, not a lost report
            out["p2p"] = {"pass": False, "detail": f"{type(e).__name__}: {e}"[:200]}
    if rccl:
        try:
            from . import fabric  # with one GPU: RCCL's data path and the result checks, no bandwidth verdict
            left = None if not timeout_s else max(0.001, 0.9 * timeout_s - (_time.monotonic() - t0))
            out["rccl"] = fabric.collective_suite(devices, timeout_s=left) if left else fabric.collective_suite(devices)
        except Exception as e:  # no RCCL library, or its init failed: the suite failed
            out["rccl"] = {"pass": False, "detail": f"{type(e).__name__}: {e}"[:200]}
    return out


def burn_in(level: int, devices: List[int], minutes: float, parallel: int = 8,
            clock: Any = None, progress: Any = None) -> Dict[str, Any]:
    """Acceptance burn-in: the per-device suite of ``level`` on every device, round after round, for
    ``minutes``.  Passes only if every round of every device passed; reports each rate per device as
    min / median / max over the rounds (a GPU that drifts or throttles under sustained load shows as a wide
    spread or a late failure), how many rounds each test passed only as degraded, and the first failing
    rounds."""
    import statistics
    import time as _time
    clock = clock or _time.monotonic
    t0 = clock()
    rounds = 0
    series: Dict[int, Dict[str, List[float]]] = {d: {} for d in devices}
    failures: List[Dict[str, Any]] = []
    failed_rounds = 0
    degraded: Dict[int, Dict[str, int]] = {d: {} for d in devices}  # rounds a test passed only as degraded
    from ..models.peers import judge_node
    node_rounds: Dict[str, int] = {}  # rounds with a node-wide shortfall, per test.metric
    while True:
        res = run_devices(level, devices, parallel)
        for f in judge_node(res):  # each round's GPUs against each other, as the agent judges them
            key = f"{f['test']}.{f['metric']}"
            node_rounds[key] = node_rounds.get(key, 0) + 1
        rounds += 1
        bad: List[str] = []
        for d, tests in res.items():
            for test, r in tests.items():
                if not isinstance(r, dict):
                    continue
                for key in ("tflops", "copy_tbs", "read_tbs", "write_tbs", "h2d_gbps", "d2h_gbps", "fraction",
                            "max_rel_err", "max_err_over_mag", "checksum_err"):  # rates, and numerics margins
                    if isinstance(r.get(key), (int, float)) and not isinstance(r.get(key), bool):
                        series[d].setdefault(f"{test}.{key}", []).append(float(r[key]))
                for kind, row in ((r.get("kinds") or {}) if isinstance(r.get("kinds"), dict) else {}).items():
                    series[d].setdefault(f"{test}.{kind}.tflops", []).append(float(row.get("tflops", 0)))
                if r.get("pass") and r.get("degraded"):
                    degraded[d][test] = degraded[d].get(test, 0) + 1
                if r.get("pass") is False:
                    bad.append(f"gpu{d}:{test}")
                    if len(failures) < 20:
                        failures.append({"round": rounds, "t_s": round(clock() - t0, 1), "device": d, "test": test,
                                         "detail": r.get("detail", "")})
        failed_rounds += 1 if bad else 0
        if progress is not None:  # one line per round (operators watching a long burn-in, CI log liveness)
            progress(f"burn-in round {rounds} at {clock() - t0:.0f} s: " + ("FAIL " + " ".join(bad) if bad else "pass"))
        if clock() - t0 >= 60.0 * minutes:
            break
    def r3(x: float) -> float:  # 3 decimals for rates, 3 significant digits for the tiny error figures
        return round(x, 3) if abs(x) >= 1e-3 or x == 0 else float(f"{x:.3g}")
    summary = {d: {k: {"min": r3(min(v)), "median": r3(statistics.median(v)), "max": r3(max(v))}
                   for k, v in m.items()} for d, m in series.items()}
    return {"minutes": minutes, "rounds": rounds, "failed_rounds": failed_rounds, "wall_s": round(clock() - t0, 1),
            "pass": failed_rounds == 0, "failures": failures, "devices": summary,
            "degraded_rounds": {d: v for d, v in degraded.items() if v}, "node_degraded_rounds": node_rounds}


def main(argv=None) -> int:
    """``mi355x-diag [--level N] [--device D] [--parallel P] [--timeout S] [--duration MIN] [--format json|text]``:
    run the active diagnostics (every device at once, as the node agent does), print one JSON document (or a
    text summary); ``--duration`` turns it into an acceptance burn-in of that many minutes."""
    import argparse
    import json
    ap = argparse.ArgumentParser(prog="mi355x-diag", description="MI355X active diagnostics (HIP, gfx950)")
    ap.add_argument("--level", type=int, default=1, choices=(1, 2))
    ap.add_argument("--device", type=int, action="append", help="GPU index (repeatable; default: all)")
    ap.add_argument("--parallel", type=int, default=8, help="devices tested at once (default 8; 1 = one by one)")
    ap.add_argument("--no-p2p", dest="p2p", action="store_false", help="skip the level-2 xGMI pair matrix")
    ap.add_argument("--no-rccl", dest="rccl", action="store_false",
                    help="skip the level-2 RCCL collectives (ops/fabric.py)")
    ap.add_argument("--timeout", type=float, default=0.0,
                    help="level 2: bound the node-level tests (s); a hung xGMI pair or collective is reported failed")
    ap.add_argument("--duration", type=float, default=0.0,
                    help="burn-in: repeat the per-device suite for this many minutes (0 = one run)")
    ap.add_argument("--format", choices=("json", "text"), default="json")
    args = ap.parse_args(argv)
    devices = args.device if args.device else list(range(device_count()))
    if not devices:  # no GPU is not a passing GPU (driver not loaded, devices not mounted into the pod)
        msg = "no HIP devices visible (amdgpu driver loaded? /dev/kfd and /dev/dri mounted?)"
        print(f"result: FAIL ({msg})" if args.format == "text" else json.dumps({"devices": {}, "pass": False,
                                                                                "error": msg}, indent=1))
        return 1
    if args.duration > 0:
        import sys as _sys
        b = burn_in(args.level, devices, args.duration, max(1, args.parallel),
                    progress=lambda line: print(line, file=_sys.stderr, flush=True))
        if args.level >= 2 and (args.p2p or args.rccl):  # the node-level tests once, after the rounds
            b["fabric"] = fabric_tests(devices, args.p2p, args.rccl, args.timeout or None)
            b["pass"] = b["pass"] and all(r.get("pass") for r in b["fabric"].values())
        if args.format == "text":
            lines = [f"burn-in: {b['rounds']} rounds in {b['wall_s']} s on {len(devices)} GPU(s)"]
            for d, m in b["devices"].items():
                for k in sorted(m):
                    if k.endswith(".fraction"):
                        continue
                    v = m[k]
                    lines.append(f"  GPU {d} {k:<28} min {v['min']:<10g} median {v['median']:<10g} max {v['max']:g}")
            for d, tests in b["degraded_rounds"].items():
                lines.append(f"  GPU {d} degraded (below {DEGRADED_FRACTION:.0%} of the reference after re-measuring) in "
                             + ", ".join(f"{t} {n}/{b['rounds']} rounds" for t, n in sorted(tests.items())))
            lines += [f"  FAIL round {f['round']} GPU {f['device']} {f['test']}: {f['detail']}" for f in b["failures"]]
            for test, r in (b.get("fabric") or {}).items():
                lines.append(f"fabric {test:<5} {'pass' if r.get('pass') else 'FAIL':<9} {_summary(test, r)}"
                             + (f"  {r['detail']}" if r.get("detail") else ""))
            lines.append(f"result: {'PASS' if b['pass'] else 'FAIL'}")
            print("\n".join(lines))
        else:
            print(json.dumps(b, indent=1))
        return 0 if b["pass"] else 1
    results = run_devices(args.level, devices, max(1, args.parallel))
    from ..models.peers import finding_text, judge_node
    findings = judge_node(results)  # GPUs measured together: each against the others (lone: the references)
    out: Dict[str, Any] = {"devices": {d: {"info": device_info(d), "tests": results[d]} for d in devices}}
    if findings:
        out["node"] = {"findings": findings, "warnings": [finding_text(f) for f in findings]}
    ok = all(t.get("pass") for d in out["devices"].values() for t in d["tests"].values())
    if args.level >= 2 and (args.p2p or args.rccl):
        out["fabric"] = fabric_tests(devices, args.p2p, args.rccl, args.timeout or None)
        ok = ok and all(r.get("pass") for r in out["fabric"].values())
    out["pass"] = ok
    print(render_text(out) if args.format == "text" else json.dumps(out, indent=1), end="" if args.format == "text" else "\n")
    return 0 if out["pass"] else 1


if __name__ == "__main__":
    raise SystemExit(main())
