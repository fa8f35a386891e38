"""gemm_ln (GEMM + residual + full-row LayerNorm) vs gemm + layernorm on the MiT-b2 B = 256 stage-3 / stage-4
shapes, f16.  GPU box: python tools/gemm_ln_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from svk import ops  # noqa: E402
from pk_cfg_sweep import timeit  # noqa: E402


def main():
    dev, dt = torch.device("cuda:0"), torch.float16
    ops.GEMM_LN = True
    for M, N, K, what in ((50176, 320, 320, "s3 proj + norm2"), (50176, 320, 80, "s3 shared MLP + norm1"),
                          (12544, 512, 512, "s4 proj + norm2"), (12544, 512, 128, "s4 shared MLP + norm1")):
        a = torch.randn(M, K, device=dev).to(dt)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(dt)
        b, g, bt = torch.randn(N, device=dev), torch.ones(N, device=dev), torch.zeros(N, device=dev)
        r = torch.randn(M, N, device=dev).to(dt)
        pk = ops.gemm_ln_pack(w)
        f = lambda: ops.gemm_ln(a, pk, N, b, r, g, bt, 1e-6)
        u = lambda: ops.layernorm(ops.gemm(a, w, b, residual=r), g, bt, 1e-6)
        tf, tu = timeit(f, 30), timeit(u, 30)
        x16 = ops.gemm(a, w, b, residual=r)
        tg = timeit(lambda: ops.gemm(a, w, b, residual=r), 30)
        d = (f()[1].float() - u().float()).abs().max().item()
        print(f"{what:24s} ({M}, {N}, {K}): gemm_ln {tf * 1e3:6.1f} us | gemm + layernorm {tu * 1e3:6.1f} us "
              f"(gemm {tg * 1e3:.1f}) | max|d h| {d:.2e}", flush=True)
        del x16


if __name__ == "__main__":
    main()
