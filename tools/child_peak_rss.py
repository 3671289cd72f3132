#!/usr/bin/env python3
"""Peak host memory of one diagnostic suite run in a child process, as the agent's isolated children run it:
``mi355x-diag --level N --device 0`` (no xGMI, no RCCL) in a fresh interpreter, its peak RSS from ``wait4``.  One JSON
line per level: peak MiB, wall time, every test passing.

    python tools/child_peak_rss.py --levels 1,2
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--levels", default="1,2")
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args()
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    for level in (int(x) for x in args.levels.split(",")):
        t0 = time.monotonic()
        p = subprocess.Popen([sys.executable, "-m", "k8s_gpu_node_checker_amd.ops.diag", "--level", str(level),
                              "--device", str(args.device), "--no-p2p", "--no-rccl", "--format", "json"],
                             stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env)
        out = p.stdout.read() if p.stdout else b""
        _, status, ru = os.wait4(p.pid, 0)
        p.returncode = os.waitstatus_to_exitcode(status)
        try:
            tests = json.loads(out)["devices"][str(args.device)]["tests"]
            passed = all(t.get("pass") is not False for t in tests.values() if isinstance(t, dict))
        except (ValueError, KeyError):
            passed = None
        print(json.dumps({"level": level, "peak_rss_mib": round(ru.ru_maxrss / 1024, 1),
                          "wall_s": round(time.monotonic() - t0, 2), "exit": p.returncode, "all_pass": passed}),
              flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
