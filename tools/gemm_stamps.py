#!/usr/bin/env python3
"""Where the v3 GEMM's K-loop spends its cycles, slot by slot: in-kernel ``s_memtime`` stamps.

Builds ``csrc/diag/diag.hip`` with ``-DDIAG_GEMM_STAMPS`` into ``tools/_stamps/`` (``--build``, on the CPU
side), then on the GPU runs one 8192^3 bf16 GEMM per restaging schedule and reads the stamps of the middle
K-tile: for wave 0 (group 0) and wave 4 (group 1, one barrier behind) of the first 8 workgroups, each phase's
load slot (restaging + fragment reads + barrier wait), MFMA issue, and the wait at the barrier closing the
MFMA slot -- the barrier wait is time the other group's load slot took beyond this group's MFMAs.

    python tools/gemm_stamps.py --build            # CPU: hipcc the stamp build
    python tools/gemm_stamps.py --schedules 0,1    # GPU: one JSON line per schedule
    python tools/gemm_stamps.py --no-store-ab      # GPU: shipped kernels vs the build that skips the C write
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT_DIR = os.path.join(REPO, "tools", "_stamps")
SO = os.path.join(OUT_DIR, "libmi355x_diag_stamps.so")
SO_NOSTORE = os.path.join(OUT_DIR, "libmi355x_diag_nostore.so")


def build() -> None:
    os.makedirs(OUT_DIR, exist_ok=True)
    src = os.path.join(REPO, "k8s_gpu_node_checker_amd", "csrc", "diag", "diag.hip")
    base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
            "-Wno-unused-result"]
    subprocess.run(base + ["-DDIAG_GEMM_STAMPS", src, "-o", SO], check=True)
    # ablation: the same kernels with the C write skipped at run time (the epilogue's LDS staging still runs)
    subprocess.run(base + ["-DDIAG_GEMM_NO_STORE", src, "-o", SO_NOSTORE], check=True)
    print(SO, SO_NOSTORE)


def no_store_ab(rounds: int = 7) -> None:
    """Time the shipped kernels against the no-store ablation (same process, interleaved): how much of the
    run the C write costs."""
    import torch
    libs = {"shipped": ctypes.CDLL(os.path.join(REPO, "k8s_gpu_node_checker_amd", "_native", "libmi355x_diag.so")),
            "no_store": ctypes.CDLL(SO_NOSTORE)}
    for L in libs.values():
        for f in ("diag_gemm_bf16_launch", "diag_gemm_fp8_launch"):
            getattr(L, f).argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
        L.diag_set_gemm_variant.argtypes = [ctypes.c_int]
        L.diag_set_gemm_variant(3)
    st = torch.cuda.current_stream().cuda_stream
    for n in (4096, 8192):
        g = torch.Generator(device="cuda").manual_seed(n)
        a = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
        b = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
        c = torch.empty(n, n, device="cuda")
        for name, dt, fn in (("bf16", torch.bfloat16, "diag_gemm_bf16_launch"),
                             ("mxfp8", torch.float8_e4m3fn, "diag_gemm_fp8_launch")):
            x, y = a.to(dt), b.to(dt)
            tf = {k: [] for k in libs}
            for _ in range(rounds):
                for k, L in libs.items():
                    launch = getattr(L, fn)
                    for _ in range(3):
                        launch(x.data_ptr(), y.data_ptr(), c.data_ptr(), n, n, n, st)
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    it = 30 if n <= 4096 else 10
                    s.record()
                    for _ in range(it):
                        launch(x.data_ptr(), y.data_ptr(), c.data_ptr(), n, n, n, st)
                    e.record()
                    torch.cuda.synchronize()
                    tf[k].append(2.0 * n ** 3 / (s.elapsed_time(e) / it) / 1e9)
            med = {k: round(statistics.median(v), 1) for k, v in tf.items()}
            print(json.dumps({"dtype": name, "size": n, "median_tflops": med,
                              "c_write_share": round(1 - med["shipped"] / med["no_store"], 3)}), flush=True)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--schedules", default="0,1")
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "mxfp8"))
    ap.add_argument("--no-store-ab", action="store_true", help="time the shipped kernels against the no-store build")
    args = ap.parse_args()
    if args.build:
        build()
        return 0
    if args.no_store_ab:
        no_store_ab()
        return 0
    import torch
    L = ctypes.CDLL(SO)
    L.diag_last_error.restype = ctypes.c_char_p
    for f in ("diag_set_gemm_variant", "diag_set_gemm_schedule", "diag_set_gemm_epilogue"):
        getattr(L, f).argtypes = [ctypes.c_int]
    launch = L.diag_gemm_bf16_launch if args.dtype == "bf16" else L.diag_gemm_fp8_launch
    launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                       ctypes.c_void_p]
    L.diag_gemm_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    n = args.size
    g = torch.Generator(device="cuda").manual_seed(7)
    a = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
    b = torch.rand(n, n, device="cuda", generator=g) * 2 - 1
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float8_e4m3fn
    x, y = a.to(dt), b.to(dt)
    c = torch.empty(n, n, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    L.diag_set_gemm_variant(3)
    for sched in (int(s) for s in args.schedules.split(",")):
        L.diag_set_gemm_schedule(sched)
        for _ in range(20):  # warm clocks, then the stamped launch is the last one
            if launch(x.data_ptr(), y.data_ptr(), c.data_ptr(), n, n, n, st) != 0:
                print(L.diag_last_error().decode(), file=sys.stderr)
                return 1
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (8 * 2 * 4 * 4))()
        if L.diag_gemm_stamps(buf) != 0:
            print(L.diag_last_error().decode(), file=sys.stderr)
            return 1
        v = list(buf)

        def at(blk, grp, ph, q):
            return v[((blk * 2 + grp) * 4 + ph) * 4 + q]
        rows = {}
        for grp in (0, 1):
            for ph in range(4):
                load = [at(bk, grp, ph, 1) - at(bk, grp, ph, 0) for bk in range(8)]
                issue = [at(bk, grp, ph, 2) - at(bk, grp, ph, 1) for bk in range(8)]
                wait = [at(bk, grp, ph, 3) - at(bk, grp, ph, 2) for bk in range(8)]
                rows[f"g{grp}p{ph}"] = {"load_slot": statistics.median(load), "mfma_issue": statistics.median(issue),
                                        "barrier_wait": statistics.median(wait)}
        tile = [at(bk, 0, 3, 3) - at(bk, 0, 0, 0) for bk in range(8)]
        print(json.dumps({"dtype": args.dtype, "size": n, "schedule": sched, "k_tile_cycles": statistics.median(tile),
                          "slots": rows}), flush=True)
    L.diag_set_gemm_schedule(1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
