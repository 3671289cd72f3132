#!/usr/bin/env python3
"""Interleaved same-machine A/B of the checker code of earlier rounds against the current tree.

VERDICT r3 asked whether the driver's 1-node headline moving from 0.552 ms (r01, ``BENCH_r01.json``, head
b0cd0d8) to 0.693 ms (r03, ``BENCH_r03.json``, head ddb9efe) is code or box.  This runs each version's *own*
``bench.py`` (so each reads the cluster the way it did when the driver measured it) on one machine, version
after version in rotation, so drift of the machine lands on every version alike:

    python tools/ab_rounds.py --prepare            # git archive b0cd0d8 / ddb9efe into .ab/, build fast paths
    python tools/ab_rounds.py --nodes 1 8 1000 --repeats 7 --out profiles/ab_rounds.json

``--prepare`` extracts only what a bench run loads (package, bench.py) and builds each version's g++ fast path
and amd-smi probe (no HIP: ``--diag-level 0``, the check path is host-only).  Each run is one child process:
``bench.py --steps S --warmup W --nodes N --diag-level 0``; the per-version result is the median (and min) of
its runs' ``ms_per_step``, plus p50 latency.  The driver's own command is ``--steps 20 --warmup 5``; 200 steps
are run too because 20 are few enough for one slow step to move the mean.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AB = os.path.join(REPO, ".ab")
VERSIONS = {"r01": "b0cd0d86efe0", "r03": "ddb9efea6717"}


def prepare() -> None:
    os.makedirs(AB, exist_ok=True)
    for tag, sha in VERSIONS.items():
        dst = os.path.join(AB, tag)
        if not os.path.isdir(dst):
            os.makedirs(dst)
            arch = subprocess.run(["git", "-C", REPO, "archive", sha, "k8s_gpu_node_checker_amd", "bench.py",
                                   "check-gpu-node.py"], capture_output=True, check=True).stdout
            subprocess.run(["tar", "-x", "-C", dst], input=arch, check=True)
        subprocess.run([sys.executable, "-m", "k8s_gpu_node_checker_amd.build", "--only", "fastpath,probe"], cwd=dst,
                       check=True)
        print(f"{tag}: {sha} in {os.path.relpath(dst, REPO)}", flush=True)


def one(tree: str, nodes: int, steps: int, warmup: int) -> dict:
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH",)}
    cmd = [sys.executable, os.path.join(tree, "bench.py"), "--steps", str(steps), "--warmup", str(warmup),
           "--nodes", str(nodes), "--diag-level", "0"]
    p = subprocess.run(cmd, capture_output=True, text=True, cwd=tree, env=env, timeout=600)
    line = next((x for x in reversed(p.stdout.splitlines()) if x.startswith("{")), None)
    if p.returncode != 0 or line is None:
        raise RuntimeError(f"{tree} nodes={nodes}: rc {p.returncode}\n{p.stderr[-2000:]}")
    d = json.loads(line)
    return {"ms": d["ms_per_step"], "p50": (d.get("latency_ms") or {}).get("p50"), "check_ok": d.get("check_ok"),
            "backend": d.get("backend")}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--prepare", action="store_true")
    ap.add_argument("--nodes", type=int, nargs="+", default=[1, 8, 1000])
    ap.add_argument("--repeats", type=int, default=7)
    ap.add_argument("--schedules", default="20:5,200:20", help="steps:warmup pairs (default: the driver's 20:5, 200:20)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    if args.prepare:
        prepare()
        return 0
    trees = {tag: os.path.join(AB, tag) for tag in VERSIONS}
    trees["r04"] = REPO
    for tag, tree in trees.items():
        if not os.path.exists(os.path.join(tree, "bench.py")):
            raise SystemExit(f"{tag}: {tree} missing (run --prepare)")
    sched = [tuple(int(x) for x in s.split(":")) for s in args.schedules.split(",")]
    runs = {}
    t0 = time.time()
    for rep in range(args.repeats):
        for n in args.nodes:
            for steps, warmup in sched:
                # rotate the order every repeat: no version always runs first (cold caches) or last
                order = list(trees)
                k = rep % len(order)
                for tag in order[k:] + order[:k]:
                    if n == 1000 and steps > 100:
                        steps, warmup = 100, 10  # 1000-node checks are ~10 ms: 100 steps are plenty
                    r = one(trees[tag], n, steps, warmup)
                    runs.setdefault(f"{n}:{steps}", {}).setdefault(tag, []).append(r)
                    print(f"rep {rep} nodes {n} steps {steps} {tag}: {r['ms']:.4f} ms (p50 {r['p50']})", flush=True)
    summary = {}
    for key, per in runs.items():
        summary[key] = {tag: {"median_ms": round(statistics.median(x["ms"] for x in rs), 4),
                              "min_ms": round(min(x["ms"] for x in rs), 4),
                              "median_p50_ms": round(statistics.median(x["p50"] for x in rs if x["p50"] is not None), 4),
                              "runs": len(rs), "all_ok": all(x["check_ok"] for x in rs),
                              "backend": sorted({x["backend"] for x in rs})}
                        for tag, rs in per.items()}
    doc = {"what": "interleaved same-machine A/B of each round's own bench.py (--diag-level 0, host check path)",
           "versions": dict(VERSIONS, r04="working tree"), "repeats": args.repeats, "wall_s": round(time.time() - t0, 1),
           "host": os.uname().nodename, "cpus": os.cpu_count(), "summary": summary, "runs": runs}
    text = json.dumps(doc, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    print(json.dumps(summary, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
