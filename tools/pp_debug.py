"""gemm_pp diagnostics (GPU box): per-shape error maps by 16-row x 16-column block against an f64 reference.
Usage: python tools/pp_debug.py [cfg]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 70
    dev = torch.device("cuda:0")
    ops.tune("pk_cfg", cfg)
    for M, N, K in ((256, 256, 64), (256, 256, 128), (256, 256, 512), (512, 256, 64), (256, 512, 256),
                    (300, 256, 64), (256, 320, 64), (5000, 320, 1280), (12544, 512, 512)):
        g = torch.Generator(device="cpu").manual_seed(1)
        a = torch.randn(M, K, generator=g).to(torch.float16).to(dev)
        w = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.float16).to(dev)
        y = ops.gemm(a, w, None)
        torch.cuda.synchronize()
        ref = (a.double() @ w.double().t())
        bad = ((y.double() - ref).abs() > 2e-2 + 2e-2 * ref.abs())
        nb = int(bad.sum())
        line = f"({M},{N},{K}) {ops._last_kernel()[:40]} bad {nb}/{M * N}"
        if nb:
            rows = bad.any(1).nonzero().flatten()
            cols = bad.any(0).nonzero().flatten()
            rb = sorted(set((rows // 16).tolist()))
            cb = sorted(set((cols // 16).tolist()))
            line += f" rowblocks16 {rb[:24]}{'...' if len(rb) > 24 else ''} colblocks16 {cb[:24]}"
            r0 = int(rows[0])
            c0 = int(bad[r0].nonzero()[0])
            line += f" first ({r0},{c0}) got {float(y[r0, c0]):.4f} ref {float(ref[r0, c0]):.4f}"
            # is the wrong value the product with some other K-tile / row?
        print(line, flush=True)
    ops.tune("pk_cfg", -1)


if __name__ == "__main__":
    main()
