"""Whole-process wall clock of one CLI run (median of R), ours vs the reference script with test stand-ins.

SURVEY §6 measured the reference at 152 ms (N=1) .. 223 ms (N=1000) this way (excluding the real
`kubernetes` import, which the stand-in avoids, so the reference numbers here are a lower bound).
"""
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from k8s_gpu_node_checker_amd.testing import fixtures  # noqa: E402
from k8s_gpu_node_checker_amd.testing.mock_apiserver import MockApiServer, write_kubeconfig  # noqa: E402

REF = "/root/reference/check-gpu-node.py"
STUBS = os.path.join(REPO, "tests", "refstub")


def wall(cmd, env, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        p = subprocess.run(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        ts.append(time.perf_counter() - t)
        assert p.returncode in (0, 2, 3), cmd
    return statistics.median(ts) * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    out = []
    for n, kind in ((1, "amd"), (8, "amd"), (1000, "mixed")):
        with MockApiServer(fixtures.cluster(n, kind)) as srv:
            kc = write_kubeconfig(f"/tmp/coldstart-kc-{n}.yaml", srv.url)
            base = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH", "SLACK_WEBHOOK_URL")}
            row = {"nodes": n,
                   "ours_ms": round(wall([sys.executable, os.path.join(REPO, "check-gpu-node.py"), "--kubeconfig", kc,
                                          "--json"], base, reps), 1)}
            if os.path.exists(REF):
                row["reference_stub_ms"] = round(wall([sys.executable, REF, "--kubeconfig", kc, "--json"],
                                                      dict(base, PYTHONPATH=STUBS), reps), 1)
            out.append(row)
            print(json.dumps(row), flush=True)
    floor = wall([sys.executable, "-c", "pass"], dict(os.environ), reps)
    print(json.dumps({"python_floor_ms": round(floor, 1)}))


if __name__ == "__main__":
    main()
