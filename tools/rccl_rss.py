"""Peak host memory of the in-process RCCL suite (libmi355x_fabric.so) under RCCL environment settings.

The node agent's level-2 fabric test opens one communicator per local GPU in the agent's own process, so
whatever RCCL allocates on the host counts against the DaemonSet's memory limit.  Each variant runs in a
fresh child process (fabric_open, one all-reduce of 64 MiB, fabric_close) and reports RSS and peak RSS
(VmHWM) after each step.

    python tools/rccl_rss.py --out gpurun_out/rccl_rss.json
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

VARIANTS = {
    "default": {},
    "no_msccl": {"RCCL_MSCCL_ENABLE": "0", "RCCL_MSCCLPP_ENABLE": "0"},
    "runtime_connect": {"NCCL_RUNTIME_CONNECT": "1"},
    "no_msccl+runtime_connect": {"RCCL_MSCCL_ENABLE": "0", "RCCL_MSCCLPP_ENABLE": "0", "NCCL_RUNTIME_CONNECT": "1"},
    "nchannels_4": {"NCCL_MAX_NCHANNELS": "4"},
    "comgr_cache_off": {"AMD_COMGR_CACHE": "0"},
    "comgr_cache_tmp": {"AMD_COMGR_CACHE_DIR": "/tmp/comgr-cache-rss"},
}

CHILD = r"""
import ctypes, json, os, sys
sys.path.insert(0, %(repo)r)
def mem():
    out = {}
    for line in open("/proc/self/status"):
        if line.startswith(("VmRSS:", "VmHWM:", "RssAnon:")):
            out[line.split(":")[0]] = int(line.split()[1]) // 1024
    return out
from k8s_gpu_node_checker_amd.ops import diag, fabric
rows = [("start", mem())]
n = diag.device_count()
rows.append(("hip init", mem()))
L = fabric.lib()
arr = (ctypes.c_int * n)(*range(n))
ctx = L.fabric_open(arr, n, 60000.0)
rows.append(("fabric_open", mem()))
out = (ctypes.c_double * 4)()
rc = L.fabric_run(ctx, 0, 64 << 20, 3, 1, out, 60000.0)
rows.append(("all_reduce 64M rc=%%d" %% rc, mem()))
L.fabric_close(ctx)
rows.append(("fabric_close", mem()))
print("ROWS " + json.dumps(rows))
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/rccl_rss.json")
    ap.add_argument("--only", default="")
    ap.add_argument("--sequence", default="", help="comma list of variants run in this order (repeats allowed): "
                    "the first RCCL start on a fresh box may differ from later ones (on-disk caches)")
    args = ap.parse_args()
    res = {}
    order = args.sequence.split(",") if args.sequence else [v for v in VARIANTS
                                                          if not args.only or v in args.only.split(",")]
    for i, name in enumerate(order):
        env = VARIANTS[name]
        name = f"{i}:{name}"
        e = dict(os.environ, **env)
        p = subprocess.run([sys.executable, "-c", CHILD % {"repo": REPO}], capture_output=True, text=True, env=e,
                           timeout=120)
        line = next((x for x in p.stdout.splitlines() if x.startswith("ROWS ")), None)
        res[name] = {"env": env, "rc": p.returncode, "rows": json.loads(line[5:]) if line else None,
                     "stderr": p.stderr[-400:] if p.returncode else ""}
        print(name, json.dumps(res[name]["rows"]), flush=True)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
