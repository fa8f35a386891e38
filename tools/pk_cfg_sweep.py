"""Persistent-GEMM tile sweep on the MFMA-heavy MiT-b2 (B = 256) shapes, f16: every pk_cfg variant
interleaved in one process.  Usage (GPU box): python tools/pk_cfg_sweep.py [--reps 30]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops, _lib  # noqa: E402

SHAPES = [  # (M, N, K, residual, what)
    (50176, 320, 1280, True, "s3 fc2"), (50176, 1280, 320, False, "s3 fc1"), (50176, 320, 320, True, "s3 q/proj"),
    (12544, 640, 320, False, "s3 kv"), (12544, 2048, 512, False, "s4 fc1"), (12544, 512, 2048, True, "s4 fc2"),
    (12544, 512, 512, True, "s4 q/proj"), (12544, 1024, 512, False, "s4 kv"), (12544, 2048, 1024, False, "head"),
    (200704, 512, 128, False, "s2 fc1"), (200704, 128, 512, True, "s2 fc2"), (200704, 128, 128, True, "s2 q/proj"),
    (802816, 64, 64, True, "s1 q/proj"), (50176, 320, 80, True, "s3 prompt"), (50176, 80, 80, False, "s3 plight"),
    (12544, 1536, 512, False, "s4 qkv"),
]
CFGS = [(-1, "auto"), (10, "128x64"), (20, "64x128"), (30, "64x64"), (40, "128x160"), (60, "128x128e"), (70, "ppRF"), (71, "ppPair"), (90, "wt256"), (91, "wt160"), (92, "wt128"), (93, "wt192")]


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
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--no-sk", action="store_true", help="skip the stream-K variant")
    ap.add_argument("--cfgs", default="", help="comma-separated pk_cfg values to run (default: all)")
    args = ap.parse_args()
    cfgs = [c for c in CFGS if not (args.no_sk and c[0] == 72)]
    if args.cfgs:
        want = [int(v) for v in args.cfgs.split(",")]
        cfgs = [c for c in CFGS if c[0] in want]
    dt, dev = torch.float16, torch.device("cuda:0")
    lib = _lib.load()
    for M, N, K, res, what in SHAPES:
        a = torch.randn(M, K, device=dev).to(dt)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(dt)
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev).to(dt) if res else None
        out = torch.empty(M, N, device=dev, dtype=dt)
        ref = None
        row = []
        for cfg, name in cfgs:
            lib.svk_tune(b"pk_cfg", cfg)
            y = ops.gemm(a, w, b, residual=r, out=out).clone()
            kname = ops._last_kernel()
            if ref is None:
                ref = y
            err = float((y.float() - ref.float()).abs().max())
            ms = timeit(lambda: ops.gemm(a, w, b, residual=r, out=out), args.reps)
            gbs = 2 * (M * K + N * K + M * N * (2 if res else 1)) / ms / 1e6
            row.append(f"{name} {ms * 1e3:7.1f}us {2 * M * N * K / ms / 1e9:6.0f}TF {gbs:5.0f}GB/s d={err:.1e}"
                       + ("" if cfg < 70 or kname.startswith(("gemm_pp", "gemm_wt"))
                             else " (fallback)"))
        lib.svk_tune(b"pk_cfg", -1)
        ms = timeit(lambda: torch.matmul(a, w.t(), out=out), args.reps)   # hipBLASLt, no epilogue (yardstick)
        row.append(f"torch {ms * 1e3:7.1f}us {2 * M * N * K / ms / 1e9:6.0f}TF")
        print(f"{what:10s} ({M},{N},{K}) " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
