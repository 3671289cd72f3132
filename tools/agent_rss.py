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


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/agent_rss.json")
    ap.add_argument("--level", type=int, default=2)
    args = ap.parse_args()
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
