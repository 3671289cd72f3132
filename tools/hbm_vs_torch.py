#!/usr/bin/env python3
"""The diagnostics' HBM streams (``ops/diag.hbm``: one 16-B element per thread, full-buffer grid, nontemporal
copy/read) against PyTorch's own kernels on the same GPU and buffer size, in interleaved rounds: copy
(``dst.copy_(src)``, bytes read + written), read (``src.sum()``, bytes read) and write (``dst.fill_``).  Tells
whether the diagnostic's rates -- its references -- sit at what the vendor stack reaches.

    python tools/hbm_vs_torch.py --gib 4 --rounds 7
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
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    n = int(args.gib * (1 << 30)) // 4
    src = torch.rand(n, device="cuda")
    dst = torch.empty_like(src)
    nbytes = n * 4
    rows = {k: [] for k in ("diag_copy", "diag_read", "diag_write", "torch_copy", "torch_read", "torch_write")}
    for _ in range(args.rounds):
        r = diag.hbm(0, gib=args.gib, iters=args.iters)
        rows["diag_copy"].append(r["copy_tbs"])
        rows["diag_read"].append(r["read_tbs"])
        rows["diag_write"].append(r["write_tbs"])
        rows["torch_copy"].append(2 * nbytes / timed(lambda: dst.copy_(src), args.iters) / 1e12)
        rows["torch_read"].append(nbytes / timed(lambda: src.sum(), args.iters) / 1e12)
        rows["torch_write"].append(nbytes / timed(lambda: dst.fill_(1.0), args.iters) / 1e12)
        print(json.dumps({k: round(v[-1], 3) for k, v in rows.items()}), flush=True)
    med = {k: round(statistics.median(v), 3) for k, v in rows.items()}
    print(json.dumps({"gib": args.gib, "rounds": args.rounds, "median_tbs": med,
                      "diag_over_torch": {m: round(med[f"diag_{m}"] / med[f"torch_{m}"], 3)
                                          for m in ("copy", "read", "write")}}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
