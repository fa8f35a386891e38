"""Persistent-GEMM tile sweep on the MFMA-heavy MiT-b2 (B = 256) shapes, f16: every pk_cfg variant
interleaved in one process.  Round 6 (a first-column cold-clock effect made `auto` and
`128x128e` — the same kernel — read 71 vs 64 us): each variant is timed in --rounds round-robin passes over
all variants and the median pass is reported.  Usage (GPU box): python tools/pk_cfg_sweep.py [--reps 20]"""
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
CFGS = [(-1, "auto"), (10, "128x64"), (20, "64x128"), (30, "64x64"), (40, "128x160"), (60, "128x128e"), (70, "ppRF"),
        (71, "ppPair"), (80, "128x128w8"), (82, "128x256w8"), (84, "128x128w8s3"), (85, "w8s5"), (86, "w8s4"),
        (87, "128x256s3"), (88, "192x128"), (90, "wt256"), (91, "wt160"),
        (92, "wt128"), (93, "wt192"), (100, "torch")]


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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--cfgs", default="", help="comma-separated pk_cfg values to run (default: all; 100 = torch)")
    ap.add_argument("--shapes", default="", help="comma-separated shape names (default: all)")
    args = ap.parse_args()
    cfgs = list(CFGS)
    if args.cfgs:
        want = [int(v) for v in args.cfgs.split(",")]
        cfgs = [c for c in CFGS if c[0] in want]
    dt, dev = torch.float16, torch.device("cuda:0")
    lib = _lib.load()
    shapes = [sh for sh in SHAPES if not args.shapes or sh[4] in args.shapes.split(",")]
    for M, N, K, res, what in shapes:
        a = torch.randn(M, K, device=dev).to(dt)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(dt)
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev).to(dt) if res else None
        out = torch.empty(M, N, device=dev, dtype=dt)
        ref, info, times = None, {}, {c: [] for c, _ in cfgs}

        def run(cfg):
            if cfg == 100:                                  # hipBLASLt, no epilogue (yardstick only)
                return torch.matmul(a, w.t(), out=out)
            lib.svk_tune(b"pk_cfg", cfg)
            return ops.gemm(a, w, b, residual=r, out=out)
        for cfg, name in cfgs:
            y = run(cfg).clone()
            kname = "torch" if cfg == 100 else ops._last_kernel()
            if ref is None and cfg != 100:
                ref = y
            err = float((y.float() - ref.float()).abs().max()) if cfg != 100 else 0.0
            info[cfg] = (err, cfg < 70 or cfg >= 100 or kname.startswith(("gemm_pp", "gemm_wt")) or
                         (cfg >= 80 and cfg < 90 and kname.startswith("gemm_pk")))
        for _ in range(args.rounds):                        # round-robin: every variant sees the same clock drift
            for cfg, _ in cfgs:
                times[cfg].append(timeit(lambda: run(cfg), args.reps))
        lib.svk_tune(b"pk_cfg", -1)
        row = []
        for cfg, name in cfgs:
            ms = sorted(times[cfg])[len(times[cfg]) // 2]
            gbs = 2 * (M * K + N * K + M * N * (2 if res else 1)) / ms / 1e6
            err, ok = info[cfg]
            row.append(f"{name} {ms * 1e3:7.1f}us {2 * M * N * K / ms / 1e9:6.0f}TF {gbs:5.0f}GB/s d={err:.1e}"
                       + ("" if ok else " (fallback)"))
        print(f"{what:10s} ({M},{N},{K}) " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
