"""Active MI355X diagnostics: ctypes front-end of ``libmi355x_diag.so`` (``csrc/diag/diag.hip``).

Each test returns a dict that the node agent folds into its probe report
under ``gpus[i].diag.<test>`` and that :func:`models.health.evaluate_gpu`
turns into a failure when ``pass`` is false.

Thresholds are deliberately conservative fractions of what a healthy MI355X
delivers (numbers in ``profiles/``): they flag a GPU that is broken or badly
throttled, not one that is a few percent off.

The library is *required* on a GPU box: a missing build raises
:class:`~k8s_gpu_node_checker_amd.ops.native.NativeUnavailable` instead of
silently skipping the diagnostic.
"""

from __future__ import annotations

import ctypes
import time
from typing import Any, Dict, Optional

from .native import NativeUnavailable, load_cdll

# Pass thresholds vs a healthy MI355X (measured: profiles/gemm_explore_mi355x.json,
# profiles/hbm_explore_mi355x.json): GEMM 4096^3 ~1200 / 8192^3 ~1370 TFLOP/s bf16, HBM copy ~6.6 TB/s,
# read ~7.0 TB/s.  Device-to-device DVFS spread is ~10 %; these flag broken or badly throttled parts.
GEMM_MIN_TFLOPS = 600.0       # bf16 MFMA GEMM (4096^3 quick / 8192^3 deep)
GEMM_MAX_REL_ERR = 2e-3       # vs fp32 reference; bf16 inputs are exact in fp32, so ~1e-5 is typical
GEMM_FP8_MIN_TFLOPS = 1200.0  # MX-fp8 GEMM (measured 2100 @4096^3, 2590 @8192^3, profiles/gemm_fp8_mi355x.jsonl)
GEMM_FP8_MAX_ERR = 4e-5       # |C - ref| / sum|a*b|: the MX MFMA's own accumulation error is <= 1.6e-5
HBM_MIN_COPY_TBS = 4.0        # 16-byte copy (read + write bytes counted)
HBM_MIN_READ_TBS = 4.5
MEMTEST_MAX_ERRORS = 0
# Matrix-core burn-in (register-resident MFMA loops, random {-1,0,1} operands; measured
# profiles/mfma_lab_mi355x.jsonl: bf16 1687, fp8 1803, MX-fp8 4027, MX-fp4 7171 TFLOP/s dense)
MFMA_KINDS = ("bf16", "fp8", "mxfp8", "mxfp4")
MFMA_MIN_TFLOPS = {"bf16": 1000.0, "fp8": 1000.0, "mxfp8": 2400.0, "mxfp4": 4300.0}
P2P_MIN_FRACTION_OF_MEDIAN = 0.5  # a GPU pair slower than half the node's median pair: suspect link
HOST_LINK_MIN_GBPS = 28.0     # PCIe Gen5 x16 host link, pinned copies: measured 56.8 / 56.7 GB/s h2d / d2h
                              # (profiles/diag_mi355x.json); a Gen4 or x8 link lands at about half

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
        L.diag_device_count.restype = ctypes.c_int
        L.diag_device_arch.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.diag_gemm_bf16_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.diag_gemm_bf16.argtypes = [ctypes.c_int] * 7 + [ctypes.POINTER(ctypes.c_double)] * 3
        L.diag_gemm_fp8.argtypes = [ctypes.c_int] * 7 + [ctypes.POINTER(ctypes.c_double)] * 3
        L.diag_gemm_fp4_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.diag_gemm_fp8_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.diag_hbm_bandwidth.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int] + \
            [ctypes.POINTER(ctypes.c_double)] * 3
        L.diag_memtest.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong),
                                   ctypes.POINTER(ctypes.c_double)]
        L.diag_mfma_burn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_ulonglong)]
        L.diag_host_link.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double)]
        L.diag_p2p_copy.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_ulonglong),
                                    ctypes.POINTER(ctypes.c_int)]
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


GEMM_VARIANTS = {"auto": 0, "v1": 1, "v2": 2, "v3": 3}


def set_gemm_variant(variant: str = "auto") -> None:
    """Select the GEMM kernel: ``auto`` (v3 for 256-multiples that fill the chip, else v1),
    ``v1`` 128x128 register-staged, ``v2`` 256x256 LDS-DMA, ``v3`` 256x256 staggered LDS-DMA.
    v2/v3 need M, N multiples of 256."""
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


def gemm(device: int = 0, size: int = 8192, warmup: int = 3, iters: int = 20, samples: int = 4096) -> Dict[str, Any]:
    tf, err, ms = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    t0 = time.perf_counter()
    _check(lib().diag_gemm_bf16(device, size, size, size, warmup, iters, samples, ctypes.byref(tf),
                                ctypes.byref(err), ctypes.byref(ms)))
    ok = tf.value >= GEMM_MIN_TFLOPS and err.value <= GEMM_MAX_REL_ERR
    return {"pass": ok, "tflops": round(tf.value, 1), "max_rel_err": err.value, "ms_per_gemm": round(ms.value, 4),
            "shape": [size, size, size], "wall_s": round(time.perf_counter() - t0, 3),
            "detail": "" if ok else f"{tf.value:.0f} TFLOP/s, rel err {err.value:.2e}"}


def gemm_fp8(device: int = 0, size: int = 8192, warmup: int = 3, iters: int = 20,
             samples: int = 4096) -> Dict[str, Any]:
    """MX-fp8 GEMM burn-in: rate and sampled fp64-reference error (normalised by sum|a*b|)."""
    tf, err, ms = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    t0 = time.perf_counter()
    _check(lib().diag_gemm_fp8(device, size, size, size, warmup, iters, samples, ctypes.byref(tf),
                               ctypes.byref(err), ctypes.byref(ms)))
    ok = tf.value >= GEMM_FP8_MIN_TFLOPS and err.value <= GEMM_FP8_MAX_ERR
    return {"pass": ok, "tflops": round(tf.value, 1), "max_err_over_mag": err.value, "ms_per_gemm": round(ms.value, 4),
            "shape": [size, size, size], "wall_s": round(time.perf_counter() - t0, 3),
            "detail": "" if ok else f"{tf.value:.0f} TFLOP/s, err {err.value:.2e}"}


def hbm(device: int = 0, gib: float = 4.0, iters: int = 10) -> Dict[str, Any]:
    c, r, w = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    t0 = time.perf_counter()
    _check(lib().diag_hbm_bandwidth(device, int(gib * (1 << 30)), iters, ctypes.byref(c), ctypes.byref(r),
                                    ctypes.byref(w)))
    ok = c.value >= HBM_MIN_COPY_TBS and r.value >= HBM_MIN_READ_TBS
    return {"pass": ok, "copy_tbs": round(c.value, 3), "read_tbs": round(r.value, 3), "write_tbs": round(w.value, 3),
            "gib": gib, "wall_s": round(time.perf_counter() - t0, 3),
            "detail": "" if ok else f"copy {c.value:.2f} TB/s, read {r.value:.2f} TB/s"}


def memtest(device: int = 0, gib: float = 8.0, passes: int = 1, seed: int = 0x5EED) -> Dict[str, Any]:
    errs, first, gbps = ctypes.c_ulonglong(), ctypes.c_ulonglong(), ctypes.c_double()
    t0 = time.perf_counter()
    _check(lib().diag_memtest(device, int(gib * (1 << 30)), seed, passes, ctypes.byref(errs), ctypes.byref(first),
                              ctypes.byref(gbps)))
    ok = errs.value <= MEMTEST_MAX_ERRORS
    res: Dict[str, Any] = {"pass": ok, "errors": errs.value, "gib": gib, "passes": passes,
                           "gbps": round(gbps.value, 1), "wall_s": round(time.perf_counter() - t0, 3),
                           "detail": "" if ok else f"{errs.value} bad 16-byte words"}
    if errs.value:
        res["first_bad_byte"] = first.value
    return res


def mfma_burn(device: int = 0, kinds=MFMA_KINDS, iters: int = 2000, reps: int = 5) -> Dict[str, Any]:
    """Every matrix-core precision of the MI355X: dense TFLOP/s and exact-result errors per kind."""
    t0 = time.perf_counter()
    rows: Dict[str, Any] = {}
    problems = []
    for kind in kinds:
        tf, errs = ctypes.c_double(), ctypes.c_ulonglong()
        _check(lib().diag_mfma_burn(device, MFMA_KINDS.index(kind), iters, reps, ctypes.byref(tf), ctypes.byref(errs)))
        rows[kind] = {"tflops": round(tf.value, 1), "errors": errs.value}
        if errs.value:
            problems.append(f"{kind}: {errs.value} wrong results")
        if tf.value < MFMA_MIN_TFLOPS[kind]:
            problems.append(f"{kind}: {tf.value:.0f} TFLOP/s")
    return {"pass": not problems, "kinds": rows, "wall_s": round(time.perf_counter() - t0, 3),
            "detail": "; ".join(problems)}


def host_link(device: int = 0, mib: int = 256, iters: int = 5) -> Dict[str, Any]:
    """Pinned host <-> device bandwidth over the GPU's PCIe link (GB/s each way)."""
    h2d, d2h = ctypes.c_double(), ctypes.c_double()
    t0 = time.perf_counter()
    _check(lib().diag_host_link(device, mib << 20, iters, ctypes.byref(h2d), ctypes.byref(d2h)))
    ok = h2d.value >= HOST_LINK_MIN_GBPS and d2h.value >= HOST_LINK_MIN_GBPS
    return {"pass": ok, "h2d_gbps": round(h2d.value, 1), "d2h_gbps": round(d2h.value, 1),
            "wall_s": round(time.perf_counter() - t0, 3),
            "detail": "" if ok else f"h2d {h2d.value:.1f} GB/s, d2h {d2h.value:.1f} GB/s"}


def p2p_copy(src: int, dst: int, mib: int = 256, iters: int = 5) -> Dict[str, Any]:
    """One ordered GPU pair: copy bandwidth over xGMI (GB/s) and pattern errors on arrival."""
    gbps, errs, peer = ctypes.c_double(), ctypes.c_ulonglong(), ctypes.c_int()
    _check(lib().diag_p2p_copy(src, dst, mib << 20, iters, ctypes.byref(gbps), ctypes.byref(errs),
                               ctypes.byref(peer)))
    return {"src": src, "dst": dst, "gbps": round(gbps.value, 1), "errors": errs.value, "peer": bool(peer.value)}


def p2p_matrix(devices: Optional[list] = None, mib: int = 256, iters: int = 5) -> Dict[str, Any]:
    """Every ordered pair of ``devices`` (default: all): the node's xGMI fabric, link by link.

    Pass: every pair has direct peer access, delivers its bytes intact, and runs at no less than
    ``P2P_MIN_FRACTION_OF_MEDIAN`` of the median pair (relative, so it holds for any hive size,
    partition mode or firmware; an absolute floor would need per-platform numbers).
    """
    devs = list(range(device_count())) if devices is None else list(devices)
    t0 = time.perf_counter()
    if len(devs) < 2:
        return {"pass": True, "skipped": f"{len(devs)} GPU(s): no pairs", "pairs": [], "detail": ""}
    pairs = [p2p_copy(a, b, mib, iters) for a in devs for b in devs if a != b]
    rates = sorted(p["gbps"] for p in pairs)
    median = rates[len(rates) // 2]
    slow = [p for p in pairs if p["gbps"] < P2P_MIN_FRACTION_OF_MEDIAN * median]
    bad = [p for p in pairs if p["errors"]]
    nopeer = [p for p in pairs if not p["peer"]]
    problems = ([f"{p['src']}->{p['dst']} {p['gbps']} GB/s" for p in slow]
                + [f"{p['src']}->{p['dst']} {p['errors']} bad words" for p in bad]
                + [f"{p['src']}->{p['dst']} no peer access" for p in nopeer])
    return {"pass": not problems, "pairs": pairs, "median_gbps": median, "min_gbps": rates[0],
            "wall_s": round(time.perf_counter() - t0, 3), "detail": "; ".join(problems[:8])}


LEVELS = {
    0: (),
    1: ("gemm_quick", "gemm_fp8_quick", "hbm_quick", "mfma"),
    2: ("gemm", "gemm_fp8", "hbm", "memtest", "mfma", "host_link"),
}


def run(level: int = 1, device: int = 0) -> Dict[str, Dict[str, Any]]:
    """Run the diagnostics of ``level`` on ``device`` (1 = ~1 s quick check, 2 = deep)."""
    out: Dict[str, Dict[str, Any]] = {}
    for test in LEVELS.get(level, ()):
        try:
            if test == "gemm_quick":
                out["gemm"] = gemm(device, size=4096, warmup=2, iters=10, samples=1024)
            elif test == "gemm_fp8_quick":
                out["gemm_fp8"] = gemm_fp8(device, size=4096, warmup=2, iters=10, samples=1024)
            elif test == "gemm_fp8":
                out["gemm_fp8"] = gemm_fp8(device)
            elif test == "hbm_quick":
                out["hbm"] = hbm(device, gib=2.0, iters=5)
            elif test == "gemm":
                out["gemm"] = gemm(device)
            elif test == "hbm":
                out["hbm"] = hbm(device)
            elif test == "memtest":
                out["memtest"] = memtest(device)
            elif test == "mfma":
                out["mfma"] = mfma_burn(device)
            elif test == "host_link":
                out["host_link"] = host_link(device)
        except NativeUnavailable:
            raise
        except Exception as e:  # a failing diagnostic is a verdict, not a crash
            out[test.replace("_quick", "")] = {"pass": False, "detail": str(e)[:200]}
    return out


def main(argv=None) -> int:
    """``mi355x-diag [--level N] [--device D]``: run the active diagnostics, print one JSON document."""
    import argparse
    import json
    ap = argparse.ArgumentParser(prog="mi355x-diag", description="MI355X active diagnostics (HIP, gfx950)")
    ap.add_argument("--level", type=int, default=1, choices=(1, 2))
    ap.add_argument("--device", type=int, action="append", help="GPU index (repeatable; default: all)")
    ap.add_argument("--no-p2p", dest="p2p", action="store_false", help="skip the level-2 xGMI pair matrix")
    ap.add_argument("--no-rccl", dest="rccl", action="store_false",
                    help="skip the level-2 RCCL collectives (ops/fabric.py)")
    args = ap.parse_args(argv)
    devices = args.device if args.device else list(range(device_count()))
    out: Dict[str, Any] = {"devices": {d: {"info": device_info(d), "tests": run(args.level, d)} for d in devices}}
    ok = all(t.get("pass") for d in out["devices"].values() for t in d["tests"].values())
    if args.level >= 2 and args.p2p:
        out["fabric"] = {"p2p": p2p_matrix(devices)}
        ok = ok and out["fabric"]["p2p"]["pass"]
    if args.level >= 2 and args.rccl:
        from . import fabric  # with one GPU: RCCL's data path and the result checks, no bandwidth verdict
        out.setdefault("fabric", {})["rccl"] = fabric.collective_suite(devices)
        ok = ok and out["fabric"]["rccl"]["pass"]
    out["pass"] = ok
    print(json.dumps(out, indent=1))
    return 0 if out["pass"] else 1


if __name__ == "__main__":
    raise SystemExit(main())
