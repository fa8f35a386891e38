"""Runs only the stage-1 whole-MixFFN kernel (svk_mixffn_rw, B = 256, 56 x 56, C = 64, f16) a few times, for
rocprofv3 counter passes and timing.  GPU box: python tools/mixffn_prof.py"""
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
    B, H, W, C = 256, 56, 56, 64
    xn = torch.randn(B, H, W, C, device=dev).to(dt)
    x = torch.randn(B, H, W, C, device=dev).to(dt)
    w1 = (torch.randn(4 * C, C, device=dev) * C ** -0.5).to(dt)
    w2 = (torch.randn(C, 4 * C, device=dev) * (4 * C) ** -0.5).to(dt)
    b1, b2 = torch.randn(4 * C, device=dev) * 0.1, torch.randn(C, device=dev) * 0.1
    taps, db = torch.randn(9, 4 * C, device=dev) * 0.3, torch.randn(4 * C, device=dev) * 0.1
    f = lambda: ops.mixffn_rw(xn, x, w1, b1, taps, db, w2, b2)
    if os.environ.get("ITERS"):
        for _ in range(int(os.environ["ITERS"])):
            f()
        torch.cuda.synchronize()
        return
    print(f"mixffn_rw B={B}: {timeit(f, 20) * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
