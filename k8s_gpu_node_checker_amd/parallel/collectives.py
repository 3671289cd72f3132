"""xGMI / RCCL collective diagnostic: bus bandwidth of every collective across a node's MI355X GPUs.

The passive probe only sees that every xGMI link reports "Up"; this measures
what the fabric actually delivers.  One process per GPU, ``torch.distributed``
with backend ``"nccl"`` (= RCCL on ROCm) over the 7 point-to-point xGMI links
of each MI355X.  The four collectives data/tensor/sequence/expert parallelism
lean on take different RCCL algorithms (rings for all-reduce / reduce-scatter /
all-gather, direct peer exchanges for all-to-all), so each is checked.  For each
op and message size it times ``iters`` calls and reports

* ``algbw = bytes / t`` and ``busbw`` in the nccl-tests convention:
  ``algbw * 2 (n-1) / n`` for all-reduce, ``algbw * (n-1) / n`` for the others
  (``bytes`` = the larger of the per-rank input and output), and
* a correctness check with rank-coded data: all-reduce of ``rank + 1`` must be
  ``n (n + 1) / 2``; reduce-scatter likewise per chunk; all-gather chunk ``i``
  must be ``i + 1``; all-to-all chunk ``i`` received by rank ``r`` must be
  ``i * n + r`` (a broken link, a wrong route or a bad GPU corrupts it).

Run on a node by hand (the node agent's level-2 diagnostics run the same four ops from one
process through ``libmi355x_fabric.so``, ``ops/fabric.py``)::

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m k8s_gpu_node_checker_amd.parallel.collectives --sizes 64M,256M,1G [--ops all_reduce,all_to_all]

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


OPS = ("all_reduce", "reduce_scatter", "all_gather", "all_to_all")


def _op_buffers(op: str, nbytes: int, world: int, rank: int, dev: Any):
    """(call, check) for one op: ``call()`` runs it once, ``check()`` re-seeds, runs and verifies."""
    import torch
    import torch.distributed as dist

    chunk = max(1, nbytes // 4 // world)
    n = chunk * world
    if op == "all_reduce":
        x = torch.full((n,), float(rank + 1), dtype=torch.float32, device=dev)

        def call(group=None):
            dist.all_reduce(x, group=group)

        def check(group=None):
            x.fill_(float(rank + 1))
            call(group)
            return bool(torch.all(x == world * (world + 1) / 2).item())
    elif op == "reduce_scatter":
        x = torch.full((n,), float(rank + 1), dtype=torch.float32, device=dev)
        y = torch.empty((chunk,), dtype=torch.float32, device=dev)

        def call(group=None):
            dist.reduce_scatter_tensor(y, x, group=group)

        def check(group=None):
            y.fill_(-1.0)
            call(group)
            return bool(torch.all(y == world * (world + 1) / 2).item())
    elif op == "all_gather":
        x = torch.full((chunk,), float(rank + 1), dtype=torch.float32, device=dev)
        y = torch.empty((n,), dtype=torch.float32, device=dev)
        want = torch.arange(1, world + 1, dtype=torch.float32, device=dev).repeat_interleave(chunk)

        def call(group=None):
            dist.all_gather_into_tensor(y, x, group=group)

        def check(group=None):
            y.fill_(-1.0)
            call(group)
            return bool(torch.equal(y, want))
    elif op == "all_to_all":
        # chunk j of rank r's input goes to rank j; value r * world + j identifies (source, destination)
        x = (rank * world + torch.arange(world, dtype=torch.float32, device=dev)).repeat_interleave(chunk)
        y = torch.empty((n,), dtype=torch.float32, device=dev)
        want = (torch.arange(world, dtype=torch.float32, device=dev) * world + rank).repeat_interleave(chunk)

        def call(group=None):
            dist.all_to_all_single(y, x, group=group)

        def check(group=None):
            y.fill_(-1.0)
            call(group)
            return bool(torch.equal(y, want))
    else:
        raise ValueError(f"unknown collective {op!r}")
    return n * 4, call, check


def collective_bench(sizes: Sequence[int], ops: Sequence[str] = OPS, iters: int = 20, warmup: int = 5,
                     device: Optional[Any] = None, group: Any = None) -> List[Dict[str, Any]]:
    """Time each collective at each byte size on the current process group; rank-local rows."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = device if device is not None else torch.device("cpu")
    rows = []
    for op in ops:
        factor = 2 * (world - 1) / world if op == "all_reduce" else (world - 1) / world
        for nbytes in sizes:
            nb, call, check = _op_buffers(op, nbytes, world, rank, dev)
            for _ in range(warmup):
                call(group)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            dist.barrier(group=group)
            t0 = time.perf_counter()
            for _ in range(iters):
                call(group)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            dt = (time.perf_counter() - t0) / iters
            ok = check(group)
            algbw = nb / dt / 1e9
            rows.append({"op": op, "bytes": nb, "ms": round(dt * 1e3, 4), "algbw_gbps": round(algbw, 2),
                         "busbw_gbps": round(algbw * factor, 2) if world > 1 else None, "correct": ok})
    return rows


def allreduce_bench(sizes: Sequence[int], iters: int = 20, warmup: int = 5, device: Optional[Any] = None,
                    group: Any = None) -> List[Dict[str, Any]]:
    """All-reduce rows only (the historical entry point)."""
    return collective_bench(sizes, ("all_reduce",), iters, warmup, device, group)


def verdict(rows: List[Dict[str, Any]], world: int, min_busbw: float = MIN_BUSBW_GBPS) -> Dict[str, Any]:
    """Pass: every op returned the right data, and on a full 8-GPU hive the best >= 256 MiB all-reduce
    busbw clears ``min_busbw`` (the other ops are reported, not thresholded)."""
    big = [r for r in rows if r["bytes"] >= 256 << 20 and r["busbw_gbps"] is not None
           and r.get("op", "all_reduce") == "all_reduce"]
    best = max((r["busbw_gbps"] for r in big), default=None)
    wrong = sorted({r.get("op", "all_reduce") for r in rows if not r["correct"]})
    ok = not wrong and (best is None or world < 8 or best >= min_busbw)
    detail = "" if ok else (f"result mismatch: {', '.join(wrong)}" if wrong else f"busbw {best} GB/s < {min_busbw}")
    per_op = {}
    for r in rows:
        op = r.get("op", "all_reduce")
        if r["busbw_gbps"] is not None:
            per_op[op] = max(per_op.get(op, 0.0), r["busbw_gbps"])
    return {"pass": ok, "world": world, "best_busbw_gbps": best, "best_busbw_by_op": per_op, "detail": detail}


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="RCCL/xGMI all-reduce bus-bandwidth diagnostic")
    ap.add_argument("--sizes", default="1M,16M,64M,256M,1G")
    ap.add_argument("--ops", default=",".join(OPS), help="comma list of " + ", ".join(OPS))
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
    if backend == "nccl" and cuda:
        dist.init_process_group(backend, device_id=torch.device(f"cuda:{local_rank}"))
    else:
        dist.init_process_group(backend)
    dev = torch.device(f"cuda:{local_rank}") if cuda else torch.device("cpu")
    rows = collective_bench([parse_size(s) for s in args.sizes.split(",")], args.ops.split(","), args.iters,
                            args.warmup, dev)
    world = dist.get_world_size()
    if dist.get_rank() == 0:
        print(json.dumps({"backend": backend, "rows": rows, **verdict(rows, world, args.min_busbw)}), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
