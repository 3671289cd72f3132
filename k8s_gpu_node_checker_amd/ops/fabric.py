"""Node-level xGMI fabric check with RCCL in one process: ctypes front-end of ``libmi355x_fabric.so``
(``csrc/fabric/fabric.hip``).

The node agent cannot rely on ``torchrun`` (one process per GPU, ``parallel/collectives.py``) inside a
DaemonSet, so its level-2 diagnostics drive every local MI355X from one process through
``ncclCommInitAll``: all-reduce, reduce-scatter, all-gather and all-to-all at each message size, every
received element checked on its GPU, bus bandwidth in the nccl-tests convention.  The verdict is the
one ``parallel/collectives.py`` applies (:func:`~k8s_gpu_node_checker_amd.parallel.collectives.verdict`):
correct data everywhere, and on a full 8-GPU hive a >= 256 MiB all-reduce busbw of at least
``MIN_BUSBW_GBPS``.

The communicators are non-blocking: with ``timeout_s`` every wait polls against one deadline for the whole
suite, and a collective that has not completed by then is aborted (``ncclCommAbort``) and reported as a failed,
``aborted`` suite -- the node agent's watchdog then sees a verdict, not a thread stuck in the driver.

The library is required: a missing build raises ``NativeUnavailable``.

    python -m k8s_gpu_node_checker_amd.ops.fabric [--device 0 --device 1 ...] [--sizes 64M,256M]
"""

from __future__ import annotations

import ctypes
import time
from typing import Any, Dict, List, Optional, Sequence

from ..parallel.collectives import MIN_BUSBW_GBPS, OPS, parse_size, verdict
from .native import load_cdll

DEFAULT_SIZES = (64 << 20, 256 << 20)

_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        L = load_cdll("libmi355x_fabric.so", required=True)
        assert L is not None
        L.fabric_last_error.restype = ctypes.c_char_p
        L.fabric_rccl_version.restype = ctypes.c_int
        L.fabric_open.restype = ctypes.c_void_p
        L.fabric_open.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_double]
        L.fabric_run.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_double), ctypes.c_double]
        L.fabric_close.argtypes = [ctypes.c_void_p]
        L.fabric_aborted.argtypes = [ctypes.c_void_p]
        L.fabric_aborted.restype = ctypes.c_int
        _lib = L
    return _lib


def _error() -> str:
    return lib().fabric_last_error().decode(errors="replace")


ABORTED = -4  # fabric_run / fabric_open: the deadline passed and the communicators were aborted


def collective_suite(devices: Sequence[int], sizes: Sequence[int] = DEFAULT_SIZES, ops: Sequence[str] = OPS,
                     iters: int = 10, warmup: int = 3, min_busbw: float = MIN_BUSBW_GBPS,
                     timeout_s: Optional[float] = None) -> Dict[str, Any]:
    """Every op at every size over ``devices``; rows like ``parallel.collectives.collective_bench``.  With
    ``timeout_s`` the whole suite (communicator setup included) has that long; past it the communicators are
    aborted and the result is a failure with ``aborted: True``."""
    devs = list(devices)
    t0 = time.perf_counter()
    deadline = None if not timeout_s or timeout_s <= 0 else time.monotonic() + timeout_s

    def left_ms() -> float:  # 0 = no deadline; a spent one still gets 1 ms (the call aborts at once)
        return 0.0 if deadline is None else max(1.0, (deadline - time.monotonic()) * 1e3)
    arr = (ctypes.c_int * len(devs))(*devs)
    ctx = lib().fabric_open(arr, len(devs), left_ms())
    if not ctx:
        err = _error()
        return {"pass": False, "world": len(devs), "rows": [], "aborted": "ncclCommAbort" in err,
                "detail": f"RCCL init: {err}"[:200]}
    rows: List[Dict[str, Any]] = []
    try:
        out = (ctypes.c_double * 4)()
        for op in ops:
            for nbytes in sizes:
                rc = lib().fabric_run(ctx, OPS.index(op), nbytes, iters, warmup, out, left_ms())
                if rc != 0:
                    # aborted: the deadline passed, or a communicator's async error aborted them all -- either way
                    # the context leaked its buffers, so the agent must not re-run the suite (fabric_abandoned)
                    aborted = rc == ABORTED or bool(lib().fabric_aborted(ctx))
                    return {"pass": False, "world": len(devs), "rows": rows, "aborted": aborted,
                            "detail": f"{op} {nbytes} B: {_error()}"[:200],
                            "wall_s": round(time.perf_counter() - t0, 3)}
                rows.append({"op": op, "bytes": nbytes, "ms": round(out[0], 4), "algbw_gbps": round(out[1], 2),
                             "busbw_gbps": round(out[2], 2) if len(devs) > 1 else None,
                             "errors": int(out[3]), "correct": out[3] == 0})
    finally:
        lib().fabric_close(ctx)
    res = {**verdict(rows, len(devs), min_busbw), "rows": rows, "rccl": rccl_version(),
           "wall_s": round(time.perf_counter() - t0, 3)}
    return res


def rccl_version() -> str:
    v = int(lib().fabric_rccl_version())
    return f"{v // 10000}.{v // 100 % 100}.{v % 100}" if v > 0 else "unknown"


def main(argv: Optional[List[str]] = None) -> int:
    import argparse
    import json

    from . import diag
    ap = argparse.ArgumentParser(prog="mi355x-fabric", description="xGMI fabric check: RCCL collectives, one process")
    ap.add_argument("--device", type=int, action="append", help="GPU index (repeatable; default: all)")
    ap.add_argument("--sizes", default="64M,256M")
    ap.add_argument("--ops", default=",".join(OPS))
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args(argv)
    devices = args.device if args.device else list(range(diag.device_count()))
    res = collective_suite(devices, [parse_size(s) for s in args.sizes.split(",")], args.ops.split(","),
                           args.iters, args.warmup)
    print(json.dumps(res, indent=1))
    return 0 if res["pass"] else 1


if __name__ == "__main__":
    raise SystemExit(main())
