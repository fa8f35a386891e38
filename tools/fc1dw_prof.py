"""Times the stage-2 MixFFN front half (svk_mixffn_fc1_dwconv at B = 256, 28 x 28, C = 128, f16: fc1dw_rw /
fc1dw_rwd by SVK_RW_VAR).  GPU box: python tools/fc1dw_prof.py"""
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
    B, H, W, C = 256, 28, 28, 128
    xn = torch.randn(B, H, W, C, device=dev).to(dt)
    w1 = (torch.randn(4 * C, C, device=dev) * C ** -0.5).to(dt)
    b1 = torch.randn(4 * C, device=dev) * 0.1
    taps, db = torch.randn(9, 4 * C, device=dev) * 0.3, torch.randn(4 * C, device=dev) * 0.1
    f = lambda: ops.mixffn_fc1_dwconv(xn, w1, b1, taps, db, act="gelu")
    f()
    print(f"{ops._last_kernel()} B={B}: {timeit(f, 20) * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
