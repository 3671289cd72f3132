#!/usr/bin/env python3
"""Probe telemetry on a real MI355X: native and Python-binding probes, idle and right after a
level-2 diagnostic burst, and the throttle windows the agent derives from consecutive samples.

    python tools/telemetry_check.py --out gpurun_out/telemetry.json
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.agent.agent import Agent  # noqa: E402
from k8s_gpu_node_checker_amd.models.health import evaluate_report  # noqa: E402
from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag  # noqa: E402

TELEMETRY = ("power_w", "power_cap_w", "power_cap_default_w", "hbm_temp_c", "hotspot_c", "gfxclk_mhz",
             "vram_used_mb", "processes", "throttle_acc", "throttle")


def pick(rep):
    return [{k: g.get(k) for k in ("index", "bdf") + TELEMETRY if k in g} for g in rep.get("gpus") or []]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/telemetry.json")
    ap.add_argument("--burst-s", type=float, default=6.0)
    args = ap.parse_args()
    out = {}
    t = time.perf_counter()
    out["native_idle"] = pick(amdsmi_probe.probe_native("n"))
    out["native_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    try:
        t = time.perf_counter()
        out["python_idle"] = pick(amdsmi_probe.probe_python("n"))
        out["python_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    except Exception as e:  # the binding may be missing on a host; the native probe is what ships
        out["python_idle"] = f"{type(e).__name__}: {e}"
    agent = Agent("n", source="native")
    agent.probe_once()
    # load: back-to-back level-2 diagnostics on GPU 0 (GEMMs, MFMA burn, HBM) for --burst-s
    end = time.monotonic() + args.burst_s
    rounds = 0
    while time.monotonic() < end:
        diag.run(2, 0)
        rounds += 1
    rep = agent.probe_once()
    out["after_burst"] = pick(rep)
    out["burst_rounds"] = rounds
    time.sleep(2.0)
    rep = agent.probe_once()
    out["idle_after"] = pick(rep)
    v = evaluate_report(rep, 0)
    out["verdict"] = v.to_dict()
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out)[:3000])
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
