#!/usr/bin/env python3
"""The diagnostics' host-link test (``ops/diag.host_link``: pinned buffers, hipMemcpyAsync each way) against
PyTorch's pinned copies (``dev.copy_(host, non_blocking=True)`` and back) of the same size, interleaved rounds:
whether the 57 GB/s reference is what the vendor stack reaches over the GPU's PCIe Gen5 x16 link.

    python tools/hostlink_vs_torch.py --mib 256 --rounds 7
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / 1e3 / iters


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    nbytes = args.mib << 20
    host = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    rows = {k: [] for k in ("diag_h2d", "diag_d2h", "torch_h2d", "torch_d2h")}
    for _ in range(args.rounds):
        r = diag.host_link(0, mib=args.mib, iters=args.iters)
        rows["diag_h2d"].append(r["h2d_gbps"])
        rows["diag_d2h"].append(r["d2h_gbps"])
        rows["torch_h2d"].append(nbytes / timed(lambda: dev.copy_(host, non_blocking=True), args.iters) / 1e9)
        rows["torch_d2h"].append(nbytes / timed(lambda: host.copy_(dev, non_blocking=True), args.iters) / 1e9)
        print(json.dumps({k: round(v[-1], 2) for k, v in rows.items()}), flush=True)
    med = {k: round(statistics.median(v), 2) for k, v in rows.items()}
    print(json.dumps({"mib": args.mib, "rounds": args.rounds, "median_gbps": med,
                      "diag_over_torch": {m: round(med[f"diag_{m}"] / med[f"torch_{m}"], 3) for m in ("h2d", "d2h")}}),
          flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
