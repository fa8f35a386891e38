"""Depthwise 3x3: the all-rows-up-front strip kernel vs the rolling 8-channel window (svk_tune dw_lds 0 / 3)
on the MiT-b2 extraction (f16, B = 256, + GELU) and training (bf16, B = 88, forward with pre-activation and
the flipped-tap backward) shapes.  Outputs must be identical.  Usage: python tools/dw_roll_bench.py"""
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
    return s.elapsed_time(e) * 1e3 / reps


def main():
    dev = torch.device("cuda:0")
    for dt, B, act, pre in ((torch.float16, 256, "gelu", False), (torch.bfloat16, 88, "gelu", True),
                            (torch.bfloat16, 88, None, False)):
        for H, C in ((56, 256), (28, 512), (14, 1280), (7, 2048)):
            x = torch.randn(B, H, H, C, device=dev).to(dt)
            taps = torch.randn(9, C, device=dev) * 0.3
            bias = torch.randn(C, device=dev) * 0.1
            p = torch.empty_like(x) if pre else None
            res = {}
            for knob in (0, 3):
                ops.tune("dw_lds", knob)
                fn = (lambda: ops.dwconv3x3(x, taps, bias, act=act, pre_out=p)) if act else \
                     (lambda: ops.dwconv3x3(x, taps, bias))
                t = timeit(fn)
                res[knob] = (t, fn().clone(), None if p is None else p.clone())
            ops.tune("dw_lds", -1)
            same = torch.equal(res[0][1], res[3][1]) and (p is None or torch.equal(res[0][2], res[3][2]))
            nb = x.numel() * x.element_size() * (3 if pre else 2)
            print(f"{str(dt)[6:]:8s} B={B:3d} {H:2d}x{H:2d}x{C:<4d} act={act} pre={pre}:  strip {res[0][0]:7.1f} us "
                  f"({nb / res[0][0] / 1e3:6.0f} GB/s)  roll8 {res[3][0]:7.1f} us ({nb / res[3][0] / 1e3:6.0f} GB/s)  "
                  f"identical={same}", flush=True)
            assert same


if __name__ == "__main__":
    main()
