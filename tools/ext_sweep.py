"""gemm_pk tile sweep on the train step's extended-epilogue GEMMs (bf16, B = 88: data gradients with the DropPath
row scale and the activation backward from a saved pre-activation) and its few-row plain GEMMs, every pk_cfg interleaved in round-robin
passes, median reported.  Usage (GPU box): python tools/ext_sweep.py [--reps 20] [--rounds 3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from svk import ops, _lib  # noqa: E402
from pk_cfg_sweep import timeit  # noqa: E402

SHAPES = [  # (M, N, K, rows per frame) of svk/train.py's row_scale + dact GEMMs at B = 88 (profiles/r05/train_gemm_shapes.txt)
    (275968, 256, 64, 3136), (68992, 512, 128, 784), (17248, 1280, 320, 196), (17248, 320, 1280, 196),
    (17248, 320, 320, 196), (68992, 128, 128, 784), (275968, 64, 64, 3136), (275968, 64, 256, 3136),
    (68992, 128, 512, 784), (4312, 2048, 512, 49), (4312, 512, 2048, 49), (4312, 512, 512, 49)]
PLAIN = [  # (M, N, K) of the train step's plain-epilogue GEMMs that the policy gives 128 x 128 tiles at B = 88
    (4312, 512, 512), (4312, 2048, 512), (4312, 1280, 320), (4312, 640, 320), (4312, 512, 1024), (4312, 2048, 128),
    (4312, 128, 128), (68992, 128, 512), (17248, 1280, 320), (4312, 2048, 8192), (4312, 8192, 2048)]
CFGS = [(-1, "auto"), (0, "128x128"), (10, "128x64"), (20, "64x128"), (30, "64x64"), (60, "128x128e")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dt, dev = torch.bfloat16, torch.device("cuda:0")
    lib = _lib.load()
    for M, N, K, rpf in SHAPES + [sh + (0,) for sh in PLAIN]:
        a = torch.randn(M, K, device=dev).to(dt)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(dt)
        u = torch.randn(M, N, device=dev).to(dt)
        rs = (torch.rand(M // rpf, device=dev) < 0.9).float() / 0.9 if rpf else None
        out = torch.empty(M, N, device=dev, dtype=dt)
        times, names, ref, err = {c: [] for c, _ in CFGS}, {}, None, {}

        def run(cfg):
            lib.svk_tune(b"pk_cfg", cfg)
            if not rpf:
                return ops.gemm(a, w, None, out=out)
            return ops.gemm(a, w, None, row_scale=rs, rows_per=rpf, dact="gelu", dact_src=u, out=out)
        for cfg, _ in CFGS:
            y = run(cfg).clone()
            names[cfg] = ops._last_kernel()
            ref = y if ref is None else ref
            err[cfg] = float((y.float() - ref.float()).abs().max())
        for _ in range(args.rounds):
            for cfg, _ in CFGS:
                times[cfg].append(timeit(lambda: run(cfg), args.reps))
        lib.svk_tune(b"pk_cfg", -1)
        row = [f"{nm} {sorted(times[c])[len(times[c]) // 2] * 1e3:6.1f}us d={err[c]:.0e}" for c, nm in CFGS]
        print(f"{'ext' if rpf else 'plain'} ({M},{N},{K}) auto={names[-1][:44]} | " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
