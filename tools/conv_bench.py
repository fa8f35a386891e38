"""Implicit-GEMM conv shapes of the extraction step (B = 256, f16) under each gemm_pk tile config.
GPU box: python tools/conv_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from svk import ops  # noqa: E402
from pk_cfg_sweep import timeit  # noqa: E402

SHAPES = [  # (H, W, Cin, Cout, k, stride, pad, what)
    (57, 57, 48, 64, 2, 1, 0, "stem s2d rgb (7x7 s4)"), (57, 57, 32, 64, 2, 1, 0, "stem s2d flow"),
    (56, 56, 64, 128, 3, 2, 1, "patch embed 2"), (28, 28, 128, 320, 3, 2, 1, "patch embed 3"),
    (14, 14, 320, 512, 3, 2, 1, "patch embed 4"), (56, 56, 64, 64, 8, 8, 0, "sr s1 (k8)"),
    (28, 28, 128, 128, 4, 4, 0, "sr s2 (k4)"), (14, 14, 320, 320, 2, 2, 0, "sr s3 (k2)"),
]


def main():
    dev = torch.device("cuda:0")
    B = 256
    for H, W, Cin, Cout, k, s, p, what in SHAPES:
        x = torch.randn(B, H, W, Cin, device=dev).half()
        w = (torch.randn(Cout, k * k * Cin, device=dev) * (k * k * Cin) ** -0.5).half()
        b = torch.randn(Cout, device=dev)
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        M = B * OH * OW
        row = []
        for cfg in (-1, 10, 20, 30, 0):
            ops.tune("pk_cfg", cfg)
            ops.conv2d_nhwc(x, w, k, s, p, bias=b)
            kn = ops._last_kernel()
            ms = timeit(lambda: ops.conv2d_nhwc(x, w, k, s, p, bias=b), 20)
            row.append(f"{cfg}:{ms * 1e3:6.1f}us")
        ops.tune("pk_cfg", -1)
        byt = (x.numel() + M * Cout) * 2
        print(f"{what:22s} M={M} N={Cout} K={k * k * Cin}  " + " ".join(row) +
              f"  | HBM floor {byt / 6.0e12 * 1e6:.1f} us  ({kn[:40]})", flush=True)


if __name__ == "__main__":
    main()
