"""Numerics sweep of the bf16 GEMM variants over K-tile counts and grid shapes: max relative error of fp32 C against
torch (fp32 accumulate) and whether C equals v3's bit for bit.  One JSON line per (shape, variant).

    python tools/gemm_v4_check.py [--variants v3,v4,v4t]

fp8 (OCP E4M3, the unscaled MFMA) is checked the same way against an fp64 reference, error normalised by sum|a*b|.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k8s_gpu_node_checker_amd.ops import diag  # noqa: E402

SHAPES = [(256, 256, 64), (256, 256, 128), (256, 256, 192), (256, 256, 256), (256, 256, 320), (512, 256, 192),
          (768, 512, 320), (1024, 768, 4096), (2048, 2048, 2048), (4096, 4096, 4096), (4096, 4096, 4160)]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="v3,v4,v4t")
    args = ap.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    bad = 0
    for m, n, k in SHAPES:
        if k % 128 == 0:  # fp8: K a multiple of 128
            g = torch.Generator(device="cuda").manual_seed(m + 5 * n + 3 * k)
            x = torch.randn(m, k, device="cuda", generator=g).to(torch.float8_e4m3fn)
            y = torch.randn(n, k, device="cuda", generator=g).to(torch.float8_e4m3fn)
            ref = x.double() @ y.double().t()
            mag = (x.double().abs() @ y.double().abs().t()).clamp_min(1e-30)
            base = None
            for v in args.variants.split(","):
                c = torch.full((m, n), float("nan"), device="cuda")
                with diag.gemm_config(variant=v):
                    diag.gemm_fp8_launch(x.data_ptr(), y.data_ptr(), c.data_ptr(), m, n, k, st)
                torch.cuda.synchronize()
                err = ((c.double() - ref).abs() / mag).max().item()
                same = None if base is None else bool(torch.equal(c, base))
                base = c if base is None else base
                ok = err < diag.GEMM_FP8_MAX_ERR
                bad += not ok
                print(json.dumps({"dtype": "fp8", "shape": [m, n, k], "variant": v, "max_err_over_mag": err, "ok": ok,
                                  "equals_first": same}), flush=True)
        g = torch.Generator(device="cuda").manual_seed(m + 3 * n + 7 * k)
        a = torch.randn(m, k, device="cuda", generator=g).to(torch.bfloat16)
        bt = torch.randn(n, k, device="cuda", generator=g).to(torch.bfloat16)
        ref = a.float() @ bt.float().t()
        base = None
        for v in args.variants.split(","):
            c = torch.full((m, n), float("nan"), device="cuda")
            with diag.gemm_config(variant=v):
                diag.gemm_launch(a.data_ptr(), bt.data_ptr(), c.data_ptr(), m, n, k, st)
            torch.cuda.synchronize()
            rel = ((c - ref).abs() / ref.abs().clamp_min(1.0)).max().item()
            same = None if base is None else bool(torch.equal(c, base))
            base = c if base is None else base
            ok = rel < 1e-4 * max(1, k / 512)
            bad += not ok
            print(json.dumps({"dtype": "bf16", "shape": [m, n, k], "variant": v, "max_rel_err": rel, "ok": ok,
                              "equals_first": same}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
