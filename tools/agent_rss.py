"""Host memory of the node agent by stage, on a real MI355X: what the DaemonSet memory limit is sized from.

Stages (RSS and peak RSS from /proc/self/status after each):
  python + agent import -> native amd-smi probe -> HIP runtime on the device (first device call) ->
  level-1 diagnostics -> level-2 diagnostics (pinned host buffer of the host-link test) -> RCCL suite.
The increment of the first HIP device call is the per-device cost (context, code objects loaded for that
device); on a box with one GPU that is the only per-device number measurable, so the budget for N devices
extrapolates it (agent.memory_budget_mib).

    python tools/agent_rss.py --out gpurun_out/agent_rss.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def mem() -> dict:
    """RSS and peak, split into anonymous memory (allocations: what grows per device and per test) and
    file-backed pages (shared libraries: loaded once per process whatever the device count)."""
    out = {}
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith(("VmRSS:", "VmHWM:", "RssAnon:", "RssFile:", "RssShmem:")):
                out[line.split(":")[0]] = int(line.split()[1]) // 1024
    return {"rss_mib": out.get("VmRSS"), "peak_mib": out.get("VmHWM"), "anon_mib": out.get("RssAnon"),
            "file_mib": out.get("RssFile"), "shmem_mib": out.get("RssShmem")}


def top_mappings(n: int = 12) -> list:
    """The largest resident mappings (/proc/self/smaps), by backing file or [anon]/[heap]."""
    sizes: dict = {}
    name = "?"
    with open("/proc/self/smaps") as f:
        for line in f:
            head = line.split()
            if head and "-" in head[0] and len(head) >= 5 and not line.startswith(("Rss", "Size")):
                name = head[5] if len(head) >= 6 else "[anon]"
                name = os.path.basename(name) if name.startswith("/") else name
            elif line.startswith("Rss:"):
                sizes[name] = sizes.get(name, 0) + int(line.split()[1])
    return [{"mapping": k, "rss_mib": round(v / 1024, 1)} for k, v in sorted(sizes.items(), key=lambda kv: -kv[1])[:n]]


def breakdown(out_path: str) -> int:
    """Anonymous/peak RSS after every level-1/2 test, then after each RCCL step (open, every op x size),
    blocking ncclCommInitAll path vs the agent's non-blocking one is not distinguishable from Python; the
    steps show where host memory goes."""
    import ctypes
    from k8s_gpu_node_checker_amd.ops import diag, fabric
    rows = [dict(step="start", **mem())]
    diag.device_info(0)
    rows.append(dict(step="hip init", **mem()))
    for test in diag.LEVELS[2]:
        try:
            diag._one(test, 0, diag.FULL)
            ok = True
        except Exception as e:  # noqa: BLE001
            ok = repr(e)[:100]
        rows.append(dict(step=f"diag {test}", ok=ok, **mem()))
    n = diag.device_count()
    L = fabric.lib()
    arr = (ctypes.c_int * n)(*range(n))
    ctx = L.fabric_open(arr, n, 60000.0)
    rows.append(dict(step="fabric_open (non-blocking)", ok=bool(ctx), **mem()))
    out = (ctypes.c_double * 4)()
    for op in fabric.OPS:
        for size in (64 << 20, 256 << 20):
            rc = L.fabric_run(ctx, fabric.OPS.index(op), size, 10, 3, out, 60000.0)
            rows.append(dict(step=f"{op} {size >> 20}M", rc=rc, **mem()))
    L.fabric_close(ctx)
    rows.append(dict(step="fabric_close", **mem()))
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    with open(out_path, "w") as f:
        json.dump({"rows": rows, "top_mappings_end": top_mappings()}, f, indent=1)
    for r in rows:
        print(json.dumps(r))
    return 0


def first_launch(out_path: str) -> int:
    """Is the host memory a GEMM adds a one-time cost of the first launch (runtime, code objects) or does it
    grow with the problem size?  Small calls of every kernel family first, then the large ones."""
    from k8s_gpu_node_checker_amd.ops import diag
    rows = [dict(step="start", **mem())]
    diag.device_info(0)
    rows.append(dict(step="hip init", **mem()))
    steps = [("hbm 0.25 GiB", lambda: diag.hbm(0, gib=0.25, iters=2)),
             ("gemm 256", lambda: diag.gemm(0, size=256, warmup=1, iters=2, samples=64)),
             ("gemm 1024", lambda: diag.gemm(0, size=1024, warmup=1, iters=2, samples=64)),
             ("gemm 4096", lambda: diag.gemm(0, size=4096, warmup=1, iters=2, samples=256)),
             ("gemm 8192", lambda: diag.gemm(0, size=8192, warmup=1, iters=2, samples=256)),
             ("gemm 8192 again", lambda: diag.gemm(0, size=8192, warmup=1, iters=2, samples=256)),
             ("gemm_fp8 256", lambda: diag.gemm_fp8(0, size=256, warmup=1, iters=2, samples=64)),
             ("gemm_fp8 8192", lambda: diag.gemm_fp8(0, size=8192, warmup=1, iters=2, samples=256)),
             ("mfma", lambda: diag.mfma_burn(0, iters=200, reps=1))]
    for name, fn in steps:
        try:
            fn()
            ok = True
        except Exception as e:  # noqa: BLE001
            ok = repr(e)[:120]
        rows.append(dict(step=name, ok=ok, **mem()))
    with open(out_path, "w") as f:
        json.dump({"rows": rows, "top_mappings_end": top_mappings()}, f, indent=1)
    for r in rows:
        print(json.dumps(r))
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/agent_rss.json")
    ap.add_argument("--level", type=int, default=2)
    ap.add_argument("--first-launch", action="store_true",
                    help="RSS across small-then-large calls of each kernel family (one-time vs size-dependent)")
    ap.add_argument("--breakdown", action="store_true",
                    help="RSS after each diagnostic test and each RCCL step instead of the stage summary")
    args = ap.parse_args()
    if args.breakdown:
        return breakdown(args.out)
    if args.first_launch:
        return first_launch(args.out)
    stages = [("python", mem())]
    from k8s_gpu_node_checker_amd.agent import agent as A  # noqa: F401
    from k8s_gpu_node_checker_amd.ops import amdsmi_probe, diag, fabric
    stages.append(("import agent", mem()))
    t = time.perf_counter()
    rep = amdsmi_probe.probe("rss", "native", None)
    stages.append(("amd-smi probe", dict(mem(), gpus=len(rep.get("gpus") or []), ms=round((time.perf_counter() - t) * 1e3))))
    n = diag.device_count()
    info = diag.device_info(0)
    stages.append(("HIP device 0 initialised", dict(mem(), hip_devices=n, cus=info["cus"])))
    tops = {}
    for level in range(1, args.level + 1):
        t = time.perf_counter()
        res = diag.run(level, 0)
        tops[level] = top_mappings()
        stages.append((f"diag level {level}", dict(mem(), all_pass=all(r.get("pass") for r in res.values()),
                                                    s=round(time.perf_counter() - t, 2))))
    r = fabric.collective_suite(list(range(n)), sizes=[64 << 20, 256 << 20], timeout_s=120)
    stages.append(("RCCL suite", dict(mem(), rccl_pass=r["pass"])))
    by = {k: v for k, v in stages}
    by_stage_top = top_mappings()
    out = {"stages": [dict(stage=k, **v) for k, v in stages], "top_mappings_after_level1": tops.get(1),
           # HIP runtime + the device's context and code objects (loaded at the first kernel) + test buffers
           "per_device_hip_mib": by["diag level 1"]["rss_mib"] - by["amd-smi probe"]["rss_mib"],
           "peak_mib": stages[-1][1]["peak_mib"], "top_mappings_end": by_stage_top}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
