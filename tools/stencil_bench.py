"""Micro-benchmark of the memory-bound stencil kernels on the MiT-b2 (B=256) shapes.
Usage (GPU box): SVK_DW_R=7 python tools/stencil_bench.py"""
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
    return s.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda:0")
    B = 256
    tot = 0.0
    for H, C, n in ((56, 256, 3), (28, 512, 4), (14, 1280, 6), (7, 2048, 3)):
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        taps = torch.randn(9, C, device=dev)
        bias = torch.randn(C, device=dev)
        ms = timeit(lambda: ops.dwconv3x3(x, taps, bias, act="gelu"))
        m0 = timeit(lambda: ops.dwconv3x3(x, taps, bias))
        y = torch.empty_like(x)
        mc = timeit(lambda: y.copy_(x))
        nb = 2 * x.numel() * 2
        tot += ms * n
        print(f"dwconv H={H:3d} C={C:5d}  {ms * 1e3:8.1f} us  {nb / ms / 1e6:8.1f} GB/s   no-act {m0 * 1e3:8.1f} us"
              f"   torch copy {mc * 1e3:8.1f} us {nb / mc / 1e6:8.1f} GB/s", flush=True)
    print(f"dwconv total per extraction step (16 launches): {tot * 1e3:.1f} us", flush=True)
    x = torch.randn(B, 3, 224, 224, device=dev)
    for name, fn in (("nchw_to_nhwc", lambda: ops.nchw_to_nhwc(x, torch.bfloat16, 8)),
                     ("gauss5x5", lambda: ops.gauss5x5_reflect(x, torch.bfloat16, 8))):
        try:
            ms = timeit(fn)
        except (AttributeError, TypeError) as e:
            print(name, "skipped", e)
            continue
        nb = x.numel() * 4 + B * 224 * 224 * 8 * 2
        print(f"{name:14s} {ms * 1e3:8.1f} us  {nb / ms / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
