"""Concurrent launches of the diagnostic GEMMs from several threads on one GPU, each on its own stream, repeated: every
output must equal the single-threaded one bit for bit (bf16 and fp8, the v4 and v3 kernels).  A stress check for the
per-device once-only LDS attribute and for anything shared between concurrent launches.

    python tools/gemm_concurrency_stress.py --threads 4 --rounds 20
"""
import argparse
import json
import os
import sys
import threading

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--size", type=int, default=4096)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n = args.size
    g = torch.Generator(device=dev).manual_seed(5)
    a = torch.randn(n, n, device=dev, generator=g)
    b = torch.randn(n, n, device=dev, generator=g)
    cases = {"bf16": (a.to(torch.bfloat16), b.to(torch.bfloat16), diag.gemm_launch),
             "fp8": (a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn), diag.gemm_fp8_launch)}
    bad = 0
    for variant in ("v4", "v3"):
        for name, (x, y, launch) in cases.items():
            ref = torch.empty(n, n, device=dev)
            with diag.gemm_config(variant=variant):
                launch(x.data_ptr(), y.data_ptr(), ref.data_ptr(), n, n, n, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            mism, errs = [0], []

            def worker():
                try:
                    torch.cuda.set_device(dev)
                    s = torch.cuda.Stream(device=dev)
                    c = torch.full((n, n), float("nan"), device=dev)
                    s.wait_stream(torch.cuda.current_stream(dev))
                    with diag.gemm_config(variant=variant):
                        for _ in range(args.rounds):
                            with torch.cuda.stream(s):
                                launch(x.data_ptr(), y.data_ptr(), c.data_ptr(), n, n, n, s.cuda_stream)
                            s.synchronize()
                            if not torch.equal(c, ref):
                                mism[0] += 1
                            c.fill_(float("nan"))
                            s.wait_stream(torch.cuda.current_stream(dev))
                except Exception as e:  # noqa: BLE001
                    errs.append(repr(e))

            ts = [threading.Thread(target=worker) for _ in range(args.threads)]
            for t in ts:
                t.start()
            for t in ts:
                t.join(300)
            bad += mism[0] + len(errs)
            print(json.dumps({"variant": variant, "dtype": name, "threads": args.threads, "rounds": args.rounds,
                              "mismatches": mism[0], "errors": errs}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
