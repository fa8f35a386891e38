"""Resident-K/V attention forward (16-bit) at the extraction step's stage-3 / 4 shapes, B = 256: per shape the
median of 3 x 20 launches.  Usage: python tools/attn_fwd_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from svk import ops  # noqa: E402
from pk_cfg_sweep import timeit  # noqa: E402

SHAPES = [(196, 196, 5, "s3 flow cross-attn"), (196, 49, 5, "s3 self-attn (SR 49)"), (49, 49, 8, "s4 self / cross")]


def main():
    dev, dt, B, hd = torch.device("cuda:0"), torch.float16, 256, 64
    for Nq, Nk, heads, what in SHAPES:
        C = heads * hd
        q = torch.randn(B, Nq, C, device=dev).to(dt)
        kv = torch.randn(B, Nk, 2 * C, device=dev).to(dt)
        k, v = kv[:, :, :C], kv[:, :, C:]
        t = sorted(timeit(lambda: ops.attention(q, k, v, heads, hd ** -0.5), 20) for _ in range(3))[1]
        gb = (2 * q.numel() + 2 * B * Nk * C) * 2 / 1e9
        print(f"{what:24s} B={B} Nq={Nq} Nk={Nk} heads={heads}: {t * 1e3:7.1f} us  {gb / (t * 1e-3) / 1e3:4.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
