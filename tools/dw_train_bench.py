"""Depthwise 3x3 (the train step's data gradient: flipped taps, zero bias, no activation; bf16, B = 88) per
dw_lds knob variant (0 strip, 1 LDS halo tile, 2 rolling window), interleaved passes, median, with the HBM roofline
(one read + one write of the map).  Usage: python tools/dw_train_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from svk import ops, _lib  # noqa: E402
from pk_cfg_sweep import timeit  # noqa: E402

SHAPES = [(56, 256), (28, 512), (14, 1280), (7, 2048)]
VARIANTS = [(0, "strip"), (1, "lds"), (2, "roll4")]
ACT = os.environ.get("DW_ACT", "")   # "gelu": the training forward's form (GELU + pre-activation store)


def main():
    dev, B = torch.device("cuda:0"), 88
    lib = _lib.load()
    for H, C in SHAPES:
        x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
        taps = torch.randn(9, C, device=dev)
        zero = torch.zeros(C, device=dev)
        pre = torch.empty_like(x)
        times, ref, err = {v: [] for v, _ in VARIANTS}, None, {}

        def run(v):
            lib.svk_tune(b"dw_lds", v)
            if ACT:
                return ops.dwconv3x3(x, taps, zero, act=ACT, pre_out=pre)
            return ops.dwconv3x3(x, taps, zero)
        for v, _ in VARIANTS:
            y = run(v).float()
            ref = y if ref is None else ref
            err[v] = float((y - ref).abs().max())
        for _ in range(3):
            for v, _ in VARIANTS:
                times[v].append(timeit(lambda: run(v), 20))
        lib.svk_tune(b"dw_lds", -1)
        gb = (3 if ACT else 2) * x.numel() * 2 / 1e9
        print(f"[{B},{H},{H},{C}] " + " | ".join(
            f"{nm} {sorted(times[v])[1] * 1e3:6.1f}us {gb / (sorted(times[v])[1] * 1e-3) / 1e3:4.2f}TB/s d={err[v]:.0e}"
            for v, nm in VARIANTS), flush=True)


if __name__ == "__main__":
    main()
