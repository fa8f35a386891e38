"""FETCH_SIZE / WRITE_SIZE calibration for the depthwise conv: the stage-3 map
(B = 256, 14 x 14, 1280 channels, f16) through dwconv3x3_strip, next to a known-byte stream of the same map
(svk's own 16-byte-per-lane elementwise cast f16 -> f16 via ops.cast, read 128 MB + write 128 MB) and torch's
copy.  Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes); tools/pmc_traffic.py
style per-kernel averages give bytes per launch to compare with the algorithmic 2 x 128 MB.
GPU box: python tools/dw_calib.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, W, K = 256, 14, 1280
    h = torch.randn(B, W, W, K, device=dev).half()
    taps = torch.randn(9, K, device=dev) * 0.3
    db = torch.randn(K, device=dev) * 0.1
    out = torch.empty_like(h)
    for _ in range(3):
        ops.dwconv3x3(h, taps, db, act="gelu")
        out.copy_(h)
    torch.cuda.synchronize()
    print("bytes per map", h.numel() * 2, flush=True)


if __name__ == "__main__":
    main()
