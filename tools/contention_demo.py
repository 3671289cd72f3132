#!/usr/bin/env python3
"""Do the level-1 thresholds catch a GPU that delivers only part of its rate?  Runs the level-1 suite on an
idle MI355X, then again while a second process keeps the same GPU busy with bf16 GEMMs (time-sliced, so
every diagnostic gets a fraction of the chip, like a GPU stuck at a low clock or power cap), and prints
each test's verdict and fraction of its reference.  The agent never does this on purpose (--diag-when
idle); here the contention stands in for a slow part.

    python tools/contention_demo.py --out gpurun_out/contention_demo.json
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

HOG = r"""
import sys, time, torch
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
print("hog ready", flush=True)
end = time.time() + float(sys.argv[1])
while time.time() < end:
    for _ in range(20):
        c = a @ b
    torch.cuda.synchronize()
"""


def summarize(res):
    return {t: {"pass": r.get("pass"), "degraded": r.get("degraded"), "fraction": r.get("fraction"),
                "detail": (r.get("detail") or "")[:160]} for t, r in res.items()}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/contention_demo.json")
    ap.add_argument("--hog-seconds", type=float, default=40.0)
    args = ap.parse_args()
    from k8s_gpu_node_checker_amd.ops import diag
    idle = diag.run(1, 0)
    hog = subprocess.Popen([sys.executable, "-c", HOG, str(args.hog_seconds)], stdout=subprocess.PIPE, text=True)
    try:
        line = hog.stdout.readline()
        assert "hog ready" in line, line
        time.sleep(2.0)
        busy = diag.run(1, 0)
    finally:
        hog.terminate()
        try:
            hog.wait(30)
        except subprocess.TimeoutExpired:
            hog.kill()
            hog.wait()
    from k8s_gpu_node_checker_amd.models import health as H
    out = {"idle": summarize(idle), "contended": summarize(busy)}
    for k, res in (("idle", idle), ("contended", busy)):
        rep = {"schema": H.SCHEMA, "node": "n", "ts": time.time(), "gpus": [{"index": 0, "gfx": H.GFX_TARGET,
                                                                                "diag": res}]}
        v = H.evaluate_report(rep, 0, H.HealthExpectations(xgmi_links=0, require_product=False), rep["ts"])
        out[k + "_diag_verdict"] = {"reasons": v.reasons, "warnings": v.warnings}
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
