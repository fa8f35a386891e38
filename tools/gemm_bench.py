"""Micro-benchmark of the svk GEMM / implicit-GEMM conv on the MiT-b2 (B=256) shapes.
Usage (GPU box): python tools/gemm_bench.py [--dtype bf16] [--reps 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402

# (M, N, K, residual) for B = 256 frames
SHAPES = [
    (802816, 256, 64, False), (802816, 64, 256, True), (802816, 64, 64, True), (802816, 16, 16, False),
    (200704, 512, 128, False), (200704, 128, 512, True), (200704, 128, 128, True),
    (50176, 1280, 320, False), (50176, 320, 1280, True), (50176, 320, 320, True),
    (12544, 2048, 512, False), (12544, 512, 2048, True), (12544, 2048, 1024, False), (12544, 512, 512, True),
    (4096, 4096, 4096, False),
]
CONVS = [  # (B, H, W, Cin, Cout, k, s, p)
    (256, 224, 224, 3, 64, 7, 4, 3), (256, 56, 56, 64, 64, 8, 8, 0), (256, 56, 56, 64, 128, 3, 2, 1),
    (256, 14, 14, 320, 320, 2, 2, 0), (256, 14, 14, 320, 512, 3, 2, 1),
]


def timeit(fn, reps):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-lib", action="store_true", help="skip the hipBLASLt comparison")
    ap.add_argument("--no-conv", action="store_true")
    args = ap.parse_args()
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    dev = torch.device("cuda:0")
    es = torch.tensor([], dtype=dt).element_size()
    for M, N, K, res in SHAPES:
        a = torch.randn(M, K, device=dev).to(dt)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(dt)
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev).to(dt) if res else None
        out = torch.empty(M, N, device=dev, dtype=dt)
        ms = timeit(lambda: ops.gemm(a, w, b, residual=r, out=out), args.reps)
        nb = (M * K + N * K + M * N * (2 if res else 1)) * es
        # hipBLASLt (torch.nn.functional.linear, bias fused, no residual) on the same shape: the
        # library ceiling for a plain GEMM, for comparison only
        bt = b.to(dt)
        ml = timeit(lambda: torch.nn.functional.linear(a, w, bt), args.reps) if not args.no_lib else float("nan")
        print(f"gemm M={M:7d} N={N:5d} K={K:5d} res={int(res)}  {ms * 1e3:9.1f} us  "
              f"{2 * M * N * K / ms / 1e9:8.1f} TF/s  {nb / ms / 1e6:8.1f} GB/s   hipblaslt {ml * 1e3:9.1f} us "
              f"{2 * M * N * K / ml / 1e9:8.1f} TF/s", flush=True)
        del a, w, r, out
    for B, H, W, Cin, Cout, k, s, p in ([] if args.no_conv else CONVS):
        x = torch.randn(B, H, W, Cin, device=dev).to(dt)
        wp = torch.randn(Cout, k * k * Cin, device=dev).to(dt)
        b = torch.randn(Cout, device=dev)
        OH = (H + 2 * p - k) // s + 1
        M, K = B * OH * OH, k * k * Cin
        ms = timeit(lambda: ops.conv2d_nhwc(x, wp, k, s, p, bias=b), args.reps)
        nb = (x.numel() + Cout * K + M * Cout) * es
        print(f"conv M={M:7d} N={Cout:5d} K={K:5d} k{k}s{s}   {ms * 1e3:9.1f} us  "
              f"{2 * M * Cout * K / ms / 1e9:8.1f} TF/s  {nb / ms / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
