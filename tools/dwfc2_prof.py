"""Runs only the fused stage-3 dw_fc2 kernel (B = 256, 14 x 14, 1280 -> 320, f16) a few times, for rocprofv3
counter passes.  GPU box: rocprofv3 --pmc ... -- python tools/dwfc2_prof.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, W, K, N, dt = 256, 14, 1280, 320, torch.float16
    h = torch.randn(B, W, W, K, device=dev).to(dt)
    taps = torch.randn(9, K, device=dev) * 0.3
    db = torch.randn(K, device=dev) * 0.1
    w2 = (torch.randn(N, K, device=dev) * K ** -0.5).to(dt)
    b2 = torch.randn(N, device=dev)
    r = torch.randn(B, W * W, N, device=dev).to(dt)
    for _ in range(int(os.environ.get("ITERS", "5"))):
        ops.mixffn_dw_fc2(h, taps, db, w2, b2, residual=r)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
