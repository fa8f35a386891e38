"""Fused vs unfused MixFFN on the stage-1/2 shapes (B=256).  Usage: python tools/mixffn_bench.py [--only fused]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402


def run(B, H, C, reps, only, dt=torch.float16):
    dev = torch.device("cuda:0")
    xn = torch.randn(B, H, H, C, device=dev).to(dt)
    x = torch.randn(B, H, H, C, device=dev).to(dt)
    w1 = (torch.randn(4 * C, C, device=dev) * C ** -0.5).to(dt)
    b1 = torch.randn(4 * C, device=dev) * 0.1
    taps = torch.randn(9, 4 * C, device=dev) * 0.3
    db = torch.randn(4 * C, device=dev) * 0.1
    w2 = (torch.randn(C, 4 * C, device=dev) * (4 * C) ** -0.5).to(dt)
    b2 = torch.randn(C, device=dev) * 0.1
    tpk = ops.mixffn_pack_taps(taps, db, dt)

    def fused():
        return ops.mixffn_fused(xn, x, w1, b1, tpk, w2, b2)

    def rw():
        return ops.mixffn_rw(xn, x, w1, b1, taps, db, w2, b2)

    def rw_ln():
        return ops.mixffn_rw(xn, x, w1, b1, taps, db, w2, b2, ln=(b2 + 1, b2, 1e-6))

    def fused_ln():
        return ops.mixffn_fused(xn, x, w1, b1, tpk, w2, b2, ln=(b2 + 1, b2, 1e-6))

    def diag(n):       # timing diagnostics of the whole-MixFFN kernel (csrc/mixffn.hip: outputs meaningless);
        # only a -DSVK_DIAG build of libsvk.so reads SVK_FFN_DIAG — the product library ignores it
        def fn():
            os.environ["SVK_FFN_DIAG"] = str(n)
            try:
                return ops.mixffn_fused(xn, x, w1, b1, tpk, w2, b2)
            finally:
                os.environ["SVK_FFN_DIAG"] = "0"
        return fn

    fused_relu = diag(1)        # GELU replaced by a ReLU
    fused_nodw = diag(2)        # dwconv waves idle: the producer waves alone
    fused_noprod = diag(3)      # producer waves idle: the dwconv waves alone

    def fc1dw():
        g = ops.mixffn_fc1_dwconv(xn, w1, b1, taps, db, act="gelu")
        return ops.gemm(g.view(-1, 4 * C), w2, b2, residual=x.view(-1, C))

    def unfused():
        h = ops.gemm(xn.view(-1, C), w1, b1)
        g = ops.dwconv3x3(h.view(B, H, H, 4 * C), taps, db, act="gelu")
        return ops.gemm(g.view(-1, 4 * C), w2, b2, residual=x.view(-1, C))

    for name, fn in (("rw", rw), ("rw_ln", rw_ln), ("fused", fused), ("fused_relu", fused_relu), ("fused_nodw", fused_nodw),
                     ("fused_noprod", fused_noprod), ("fused_ln", fused_ln), ("fc1dw", fc1dw), ("unfused", unfused)):
        if only and name != only:
            continue
        if name.startswith("fused") and not ops.mixffn_supported(H, C):
            continue
        if name.startswith("rw") and not ops.mixffn_rw_supported(dt, H, C):
            continue
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        print(f"B={B} H={H} C={C} {name:8s} {s.elapsed_time(e) / reps * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    run(256, 56, 64, a.reps, a.only)
    run(256, 28, 128, a.reps, a.only)
