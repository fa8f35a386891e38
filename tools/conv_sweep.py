"""Implicit-GEMM conv tile sweep on the MiT-b2 (B = 256) patch-embed / flow-encoder shapes, f16: every pk_cfg
variant interleaved in one process.  GPU box: python tools/conv_sweep.py [--reps 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from svk import ops, _lib  # noqa: E402
from pk_cfg_sweep import timeit  # noqa: E402

SHAPES = [  # (B, H, W, Cin, Cout, k, stride, pad, what)
    (256, 28, 28, 128, 320, 3, 2, 1, "s3 patch embed / flow conv3"),
    (256, 56, 56, 64, 128, 3, 2, 1, "s2 patch embed / flow conv2"),
    (256, 14, 14, 320, 512, 3, 2, 1, "s4 patch embed / flow conv4"),
]
CFGS = [(-1, "auto"), (0, "128x128"), (10, "128x64"), (20, "64x128"), (30, "64x64"), (40, "128x160")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dt, dev = torch.float16, torch.device("cuda:0")
    lib = _lib.load()
    for B, H, W, Cin, Cout, k, s, pad, what in SHAPES:
        x = torch.randn(B, H, W, Cin, device=dev).to(dt)
        w = (torch.randn(Cout, k * k * Cin, device=dev) * (k * k * Cin) ** -0.5).to(dt)
        b = torch.randn(Cout, device=dev)
        ref, row = None, []
        for cfg, name in CFGS:
            lib.svk_tune(b"pk_cfg", cfg)
            y = ops.conv2d_nhwc(x, w, k, s, pad, bias=b)
            kname = ops._last_kernel()
            if ref is None:
                ref = y.clone()
            d = (y.float() - ref.float()).abs().max().item()
            t = timeit(lambda: ops.conv2d_nhwc(x, w, k, s, pad, bias=b), args.reps)
            row.append(f"{name} {t * 1e3:6.1f}us{'' if d < 1e-2 else f' MISMATCH {d:.2e}'}")
            del kname
        lib.svk_tune(b"pk_cfg", -1)
        print(f"{what:30s} " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
