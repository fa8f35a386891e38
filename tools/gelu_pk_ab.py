"""Per-kernel times of the GELU-carrying MixFFN kernels at B = 256, f16 (round 6: GELU on packed f32 pairs,
SVK_GELU_PK=1, vs the element-wise form, SVK_GELU_PK=0 — read once per process, so run this twice):
stage-1 mixffn_rwd, stage-2 fc1dw_rw, stage-3 / 4 dw_fc2_mx.  Usage: SVK_GELU_PK=0|1 python tools/gelu_pk_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402


def timed(fn, reps=30):
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
    dev, dt, B = torch.device("cuda:0"), torch.float16, 256
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc)
    res = {}
    # stage 1: whole MixFFN (C = 64, 56 x 56)
    C, W = 64, 56
    xn, x = r(B, W, W, C).to(dt), r(B, W, W, C).to(dt)
    w1, b1 = r(4 * C, C, sc=C ** -0.5).to(dt), r(4 * C, sc=0.1)
    taps, db = r(9, 4 * C, sc=0.3), r(4 * C, sc=0.1)
    w2, b2 = r(C, 4 * C, sc=(4 * C) ** -0.5).to(dt), r(C, sc=0.1)
    f1 = lambda: ops.mixffn_rw(xn, x, w1, b1, taps, db, w2, b2)
    # stage 2: fc1 + dwconv + GELU (C = 128, 28 x 28)
    C2, W2 = 128, 28
    xn2 = r(B, W2, W2, C2).to(dt)
    w12, b12 = r(4 * C2, C2, sc=C2 ** -0.5).to(dt), r(4 * C2, sc=0.1)
    taps2, db2 = r(9, 4 * C2, sc=0.3), r(4 * C2, sc=0.1)
    f2 = lambda: ops.mixffn_fc1_dwconv(xn2, w12, b12, taps2, db2, act="gelu")
    fs = {"mixffn_rwd s1": f1, "fc1dw_rw s2": f2}
    for W3, K3, N3 in ((14, 1280, 320), (7, 2048, 512)):
        h = r(B, W3, W3, K3).to(dt)
        t3, d3 = r(9, K3, sc=0.3), r(K3, sc=0.1)
        w3, b3, r3 = r(N3, K3, sc=K3 ** -0.5).to(dt), r(N3), r(B, W3 * W3, N3).to(dt)
        pk = ops.mixffn_dw_fc2_pack(t3, d3, w3, W3)
        fs[f"dw_fc2_mx {W3}x{W3}"] = (lambda h=h, t3=t3, d3=d3, w3=w3, b3=b3, r3=r3, pk=pk:
                                     ops.mixffn_dw_fc2(h, t3, d3, w3, b3, residual=r3, packed=pk))
    for name, fn in fs.items():
        fn()
        res[name] = (ops._last_kernel(), sorted(timed(fn) for _ in range(3))[1])
    tag = os.environ.get("SVK_GELU_PK", "1")
    print(f"SVK_GELU_PK={tag}: " + " | ".join(f"{n} {t:.1f} us ({k})" for n, (k, t) in res.items()), flush=True)


if __name__ == "__main__":
    main()
