"""xGMI / RCCL collective diagnostic: all-reduce bus bandwidth across a node's MI355X GPUs.

The passive probe only sees that every xGMI link reports "Up"; this measures
what the fabric actually delivers.  One process per GPU, ``torch.distributed``
with backend ``"nccl"`` (= RCCL on ROCm) over the 7 point-to-point xGMI links
of each MI355X.  For each message size it times ``iters`` all-reduces and
reports

* ``algbw = bytes / t`` and ``busbw = algbw * 2 (n-1) / n`` (ring-equivalent
  bytes each GPU moves, the nccl-tests convention), and
* a correctness check: every rank contributes ``rank + 1``; the result must be
  ``n (n + 1) / 2`` everywhere (a broken link or a bad GPU corrupts it).

Run on a node (the agent's level-3 check, or by hand)::

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m k8s_gpu_node_checker_amd.parallel.collectives --sizes 64M,256M,1G

Size choice for xGMI: ring all-reduce is per-link bound, so the bandwidth
plateau needs messages of hundreds of MB per GPU; 288 GB of HBM per GPU makes
1-4 GB buffers cheap.  On CPU (``gloo``) the same code runs as a unit test.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import Any, Dict, List, Optional, Sequence

# Minimum bus bandwidth (GB/s) to call an 8-GPU MI355X hive healthy at >= 256 MB messages.
# Conservative: a single downed/slow link drags every ring well below this.
MIN_BUSBW_GBPS = 100.0


def parse_size(s: str) -> int:
    s = s.strip().upper()
    mult = 1
    for suf, m in (("K", 1 << 10), ("M", 1 << 20), ("G", 1 << 30)):
        if s.endswith(suf):
            s, mult = s[:-1], m
            break
    return int(float(s) * mult)


def allreduce_bench(sizes: Sequence[int], iters: int = 20, warmup: int = 5, device: Optional[Any] = None,
                    group: Any = None) -> List[Dict[str, Any]]:
    """Time all-reduce at each byte size on the current process group; returns per-size rows (rank-local)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = device if device is not None else torch.device("cpu")
    rows = []
    for nbytes in sizes:
        n = max(1, nbytes // 4)
        x = torch.full((n,), float(rank + 1), dtype=torch.float32, device=dev)
        expect = world * (world + 1) / 2
        for _ in range(warmup):
            dist.all_reduce(x, group=group)
            x.fill_(float(rank + 1))
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x, group=group)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / iters
        # after `iters` in-place reductions the value is expect * world**(iters-1); check the last one only
        x.fill_(float(rank + 1))
        dist.all_reduce(x, group=group)
        ok = bool(torch.all(x == expect).item())
        algbw = n * 4 / dt / 1e9
        rows.append({"bytes": n * 4, "ms": round(dt * 1e3, 4), "algbw_gbps": round(algbw, 2),
                     "busbw_gbps": round(algbw * 2 * (world - 1) / world, 2) if world > 1 else None,
                     "correct": ok})
    return rows


def verdict(rows: List[Dict[str, Any]], world: int, min_busbw: float = MIN_BUSBW_GBPS) -> Dict[str, Any]:
    big = [r for r in rows if r["bytes"] >= 256 << 20 and r["busbw_gbps"] is not None]
    best = max((r["busbw_gbps"] for r in big), default=None)
    correct = all(r["correct"] for r in rows)
    ok = correct and (best is None or world < 8 or best >= min_busbw)
    detail = "" if ok else ("all-reduce result mismatch" if not correct else f"busbw {best} GB/s < {min_busbw}")
    return {"pass": ok, "world": world, "best_busbw_gbps": best, "detail": detail}


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="RCCL/xGMI all-reduce bus-bandwidth diagnostic")
    ap.add_argument("--sizes", default="1M,16M,64M,256M,1G")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--backend", default=None, help="nccl (RCCL, default with GPUs) or gloo")
    ap.add_argument("--min-busbw", type=float, default=MIN_BUSBW_GBPS)
    args = ap.parse_args(argv)
    import torch
    import torch.distributed as dist

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available() and args.backend != "gloo"
    backend = args.backend or ("nccl" if cuda else "gloo")
    if cuda:
        torch.cuda.set_device(local_rank)
    dist.init_process_group(backend)
    dev = torch.device(f"cuda:{local_rank}") if cuda else torch.device("cpu")
    rows = allreduce_bench([parse_size(s) for s in args.sizes.split(",")], args.iters, args.warmup, dev)
    world = dist.get_world_size()
    if dist.get_rank() == 0:
        print(json.dumps({"backend": backend, "rows": rows, **verdict(rows, world, args.min_busbw)}), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
