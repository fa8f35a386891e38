"""MixFFN front half (fc1 -> dwconv3x3 -> GELU) fused vs unfused on the four MiT-b2 stage shapes.

Inference: f16, B = 256, G only.  Training forward: bf16, B = 88, G + the pre-activation map.
Usage: python tools/fc1dw_bench.py [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402

STAGES = [(56, 64), (28, 128), (14, 320), (7, 512)]


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for dt, B, train in ((torch.float16, 256, False), (torch.bfloat16, 88, True)):
        for H, C in STAGES:
            hid = 4 * C
            xn = torch.randn(B, H, H, C, device=dev).to(dt)
            w1 = (torch.randn(hid, C, device=dev) * C ** -0.5).to(dt)
            b1 = torch.randn(hid, device=dev) * 0.1
            taps = torch.randn(9, hid, device=dev) * 0.3
            db = torch.randn(hid, device=dev) * 0.1
            pre = torch.empty(B, H, H, hid, device=dev, dtype=dt) if train else None

            def fused():
                return ops.mixffn_fc1_dwconv(xn, w1, b1, taps, db, act="gelu", pre_out=pre)

            def unfused():
                h = ops.gemm(xn.view(B, H * H, C), w1, b1).view(B, H, H, hid)
                return ops.dwconv3x3(h, taps, db, act="gelu", pre_out=pre)

            tf, tu = timed(fused, a.reps), timed(unfused, a.reps)
            d = float((fused().float() - unfused().float()).abs().max())
            print(f"{'train bf16' if train else 'infer f16 '} B={B:3d} {H}x{H}x{C:<3d} fused {tf:8.1f} us  "
                  f"unfused {tu:8.1f} us  ratio {tu / tf:5.2f}  maxdiff {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
