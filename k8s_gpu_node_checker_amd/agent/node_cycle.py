"""One node-level agent cycle over several local GPUs, as a standalone process: the multi-device paths of the
node agent on real hardware.

``bench.py`` runs it (untimed, rank 0, in a child process with a time limit) whenever it has more than one
GPU: the agent's per-device diagnostic threads on every GPU at once (``--diag-parallel``, the thread-local GEMM
knobs, the per-device dynamic-LDS attribute, the host-link lock), then the node-level xGMI pair matrix and the
in-process RCCL suite under its deadline.  Prints one JSON line.

    python -m k8s_gpu_node_checker_amd.agent.node_cycle --devices 0,1,2,3,4,5,6,7 --level 1 --timeout 150
"""

from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from typing import Any, Dict, List, Optional


def run(devices: List[int], level: int = 1, timeout_s: float = 150.0, parallel: int = 8,
        fabric: bool = True) -> Dict[str, Any]:
    """The cycle; returns the summary (never raises for a failed test: failures are in the result)."""
    from ..ops import diag
    from .agent import Agent
    t0 = time.monotonic()
    out: Dict[str, Any] = {"devices": devices, "level": level, "parallel": parallel}
    live = [0]
    peak = [0]
    lock = threading.Lock()
    real_run = diag.run

    def counted(lvl: int, d: int, **kw: Any) -> Dict[str, Any]:
        with lock:
            live[0] += 1
            peak[0] = max(peak[0], live[0])
        try:
            return real_run(lvl, d, **kw)
        finally:
            with lock:
                live[0] -= 1
    diag.run = counted  # type: ignore[assignment]
    try:
        ag = Agent("node-cycle", source="auto", diag_level=level, devices=list(devices), diag_when="always",
                   diag_timeout=timeout_s, diag_parallel=parallel)
        rep = ag.probe_once()
    finally:
        diag.run = real_run  # type: ignore[assignment]
    per: Dict[str, Any] = {}
    for d in devices:
        res = ag._diag_cache.get(d)
        if res is None:
            per[str(d)] = {"skipped": ag._diag_skipped.get(d, "no result")}
            continue
        per[str(d)] = {"pass": all(r.get("pass") is not False for r in res.values() if isinstance(r, dict)),
                       "failed": sorted(k for k, r in res.items() if isinstance(r, dict) and r.get("pass") is False),
                       "degraded": sorted(k for k, r in res.items() if isinstance(r, dict) and r.get("degraded")),
                       "gemm_tflops": (res.get("gemm") or {}).get("tflops"),
                       "hbm_read_tbs": (res.get("hbm") or {}).get("read_tbs"),
                       # every rate test as a share of its single-GPU reference: with all GPUs of the node running
                       # the suite at once, this is the measurement the lone-GPU calibration lacks
                       "fractions": {k: r["fraction"] for k, r in res.items()
                                     if isinstance(r, dict) and isinstance(r.get("fraction"), (int, float))}}
    out["per_device"] = per
    out["peak_threads"] = peak[0]
    out["diag_wall_s"] = round(time.monotonic() - t0, 2)
    out["probe_gpus"] = len(rep.get("gpus") or [])
    out["verdict"] = rep.get("state")
    if fabric and len(devices) >= 2:
        t1 = time.monotonic()
        out["fabric"] = Agent._fabric_suite(list(devices), timeout_s)
        out["fabric_wall_s"] = round(time.monotonic() - t1, 2)
    out["wall_s"] = round(time.monotonic() - t0, 2)
    return out


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="mi355x-node-cycle", description=__doc__.splitlines()[0])
    ap.add_argument("--devices", required=True, help="comma list of HIP ordinals")
    ap.add_argument("--level", type=int, default=1, choices=(1, 2))
    ap.add_argument("--timeout", type=float, default=150.0, help="per-device watchdog and RCCL deadline (s)")
    ap.add_argument("--parallel", type=int, default=8)
    ap.add_argument("--no-fabric", dest="fabric", action="store_false")
    args = ap.parse_args(argv)
    devices = [int(x) for x in args.devices.split(",") if x.strip()]
    res = run(devices, args.level, args.timeout, args.parallel, args.fabric)
    print(json.dumps(res, separators=(",", ":"), default=str), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
