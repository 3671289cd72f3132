#!/usr/bin/env python3
"""Library reference point for the diag GEMM: torch.matmul bf16 (hipBLASLt) at the diag's shapes.

Same operand layout as the diag kernel (A row-major, B given as Bt, fp32-accumulated bf16
inputs); timed with HIP events over a warm loop.  One JSON line per shape.
"""

import json

import torch


def main() -> None:
    for n in (4096, 8192):
        a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
        bt = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
        for _ in range(5):
            c = a @ bt.t()
        torch.cuda.synchronize()
        iters = 50 if n == 4096 else 20
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            c = a @ bt.t()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / iters
        print(json.dumps({"kernel": "torch.matmul(bf16 out, hipBLASLt)", "size": n, "ms": round(ms, 4),
                          "tflops": round(2 * n ** 3 / (ms * 1e-3) / 1e12, 1)}), flush=True)
        del c


if __name__ == "__main__":
    main()
