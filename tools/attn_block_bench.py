"""Fused stage-1 attention half of a Block (svk_attn_block) vs the unfused chain (q GEMM, sequence-
reduced attention, proj GEMM + residual, LayerNorm) at B = 256 (stage 1 and stage 2 shapes).  Usage (GPU box): python tools/attn_block_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    for N, C in ((3136, 64), (784, 128)):
        run(N, C)


def run(N, C):
    dev, dt, B, Nk, heads = torch.device("cuda:0"), torch.float16, 256, 49, C // 64
    r = lambda *s: torch.randn(*s, device=dev).to(dt)
    hn, x, kv = r(B, N, C), r(B, N, C), r(B, Nk, 2 * C)
    wq, wp = r(C, C) * 0.125, r(C, C) * 0.125
    bq, bp, g2, b2 = (torch.randn(C, device=dev) for _ in range(4))
    fused = lambda: ops.attn_block(hn, x, kv, wq, bq, wp, bp, g2, b2, 1e-6, 0.125)
    q = ops.gemm(hn, wq, bq)
    o = ops.attention(q, kv[:, :, :C], kv[:, :, C:], heads, 0.125)
    y = ops.gemm(o, wp, bp, residual=x)
    parts = {"q": lambda: ops.gemm(hn, wq, bq),
             "attn": lambda: ops.attention(q, kv[:, :, :C], kv[:, :, C:], heads, 0.125),
             "proj": lambda: ops.gemm(o, wp, bp, residual=x),
             "ln2": lambda: ops.layernorm(y, g2, b2, 1e-6)}
    if C == 64:
        from svk import _lib
        for rep in range(3):
            for sel, what in ((6, "4 waves x 256 queries"), (4, "8 waves x 512 queries"), (0, "8 waves x 256 queries")):
                _lib.load().svk_tune(b"attn_cfg", sel)
                print(f"C=64 {what}: fused {timeit(fused):7.1f} us")
        _lib.load().svk_tune(b"attn_cfg", -1)
    tf = timeit(fused)
    tp = {k: timeit(f) for k, f in parts.items()}
    print(f"C={C}: fused {tf:7.1f} us | unfused {sum(tp.values()):7.1f} us = " + " + ".join(f"{k} {v:.1f}" for k, v in tp.items()))
    print(f"fused: {4 * B * N * C * 2 / (tf * 1e-6) / 1e12:.2f} TB/s over h, x in and y, h2 out")


if __name__ == "__main__":
    main()
