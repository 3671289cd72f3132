#!/usr/bin/env python3
"""Soak the level-2 diagnostics on one GPU for a fixed wall time: every test, every round, with its
verdict and rates, plus min/median/max per metric.  A burn-in tool that faults, hangs or drifts under
sustained load is worse than none; this is the evidence that it does not.

    python tools/soak.py --minutes 5 --out gpurun_out/soak.json [--rccl]

``--rccl`` adds the in-process RCCL collectives (``ops/fabric.py``: communicator set up and torn down
every round, as the agent does hourly) and tracks host RSS and amd-smi VRAM in use across the run, so
a per-round leak shows as drift.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402

METRICS = (("gemm", "tflops"), ("gemm_fp8", "tflops"), ("hbm", "copy_tbs"), ("hbm", "read_tbs"),
           ("hbm", "write_tbs"), ("memtest", "errors"), ("host_link", "h2d_gbps"), ("host_link", "d2h_gbps"),
           ("l2", "read_tbs"), ("l2", "errors"), ("lds", "errors"), ("hbm_xcd", "read_tbs"), ("hbm_xcd", "errors"),
           ("hbm_xcd", "slowest_xcd_rel"))


def _rss_mb() -> float:
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return round(int(line.split()[1]) / 1024, 1)
    return 0.0


def _vram_used_mb(device: int):
    from k8s_gpu_node_checker_amd.ops import amdsmi_probe
    gpus = amdsmi_probe.probe_native("soak").get("gpus") or []
    return gpus[device].get("vram_used_mb") if device < len(gpus) else None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=5.0)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/soak.json")
    ap.add_argument("--level", type=int, default=2, choices=(1, 2), help="diagnostics level (1: 4096^3 quick)")
    ap.add_argument("--rccl", action="store_true", help="also run the RCCL collectives every round")
    args = ap.parse_args()
    deadline = time.monotonic() + args.minutes * 60
    rounds, failures = [], []
    series: dict = {}
    t0 = time.time()
    while time.monotonic() < deadline:
        res = diag.run(args.level, args.device)
        rnd_extra: dict = {}
        if args.rccl:
            from k8s_gpu_node_checker_amd.ops import fabric
            fab = fabric.collective_suite([args.device], sizes=[64 << 20], iters=3, warmup=1)
            res["rccl"] = {"pass": fab["pass"], "detail": fab.get("detail", "")}
            for row in fab["rows"]:
                series.setdefault(f"rccl.{row['op']}.algbw_gbps", []).append(row["algbw_gbps"])
            series.setdefault("host.rss_mb", []).append(_rss_mb())
            vram = _vram_used_mb(args.device)
            if isinstance(vram, (int, float)):
                series.setdefault("gpu.vram_used_mb", []).append(vram)
                rnd_extra["vram_mb"] = vram
            rnd_extra["rss_mb"] = series["host.rss_mb"][-1]
        rnd = {"t": round(time.time() - t0, 1), "pass": all(r.get("pass") for r in res.values()), **rnd_extra}
        for test, key in METRICS:
            v = (res.get(test) or {}).get(key)
            if isinstance(v, (int, float)):
                series.setdefault(f"{test}.{key}", []).append(v)
        for test in ("mfma", "l2"):  # where on the chip: the XCD / CU lag of the per-CU maps
            m = (res.get(test) or {}).get("map") or {}
            for key in ("slowest_rel", "slowest_cu_rel"):
                if isinstance(m.get(key), (int, float)):
                    series.setdefault(f"{test}.map.{key}", []).append(m[key])
        degraded = sorted(k for k, v in res.items() if v.get("degraded"))
        if degraded:
            rnd_extra["degraded"] = degraded
            for k in degraded:
                series.setdefault(f"degraded.{k}", []).append(1)
        for kind, row in ((res.get("mfma") or {}).get("kinds") or {}).items():
            series.setdefault(f"mfma.{kind}.tflops", []).append(row["tflops"])
            series.setdefault(f"mfma.{kind}.errors", []).append(row["errors"])
        if not rnd["pass"]:
            failures.append({"t": rnd["t"], "failed": {k: v for k, v in res.items() if not v.get("pass")}})
        rounds.append(rnd)
        print(json.dumps({"round": len(rounds), **rnd}), flush=True)
    summary = {k: {"min": min(v), "median": statistics.median(v), "max": max(v), "n": len(v)}
               for k, v in series.items()}
    out = {"device": diag.device_info(args.device), "level": args.level, "minutes": args.minutes, "rounds": len(rounds),
           "all_pass": not failures, "failures": failures[:20], "summary": summary}
    if args.rccl:
        rss, vram = series.get("host.rss_mb") or [None], series.get("gpu.vram_used_mb") or [None]
        out["leak_check"] = {"rss_mb_first_round": rss[0], "rss_mb_last_round": rss[-1],
                             "vram_used_mb_first_round": vram[0], "vram_used_mb_last_round": vram[-1],
                             "vram_used_mb_every_10th_round": vram[::10], "rss_mb_every_10th_round": rss[::10]}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"rounds": len(rounds), "all_pass": not failures}))
    return 0 if not failures else 1


if __name__ == "__main__":
    raise SystemExit(main())
