"""Runs one GEMM shape through svk (ops.gemm, default policy) a few times, for rocprofv3 counter passes.
GPU box: SHAPE=M,N,K[,res] python tools/gemm_prof.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402


def main():
    dev, dt = torch.device("cuda:0"), torch.float16
    v = [int(t) for t in os.environ.get("SHAPE", "50176,1280,320,0").split(",")]
    M, N, K = v[:3]
    res = len(v) > 3 and v[3]
    a = torch.randn(M, K, device=dev).to(dt)
    w = (torch.randn(N, K, device=dev) * K ** -0.5).to(dt)
    b = torch.randn(N, device=dev)
    r = torch.randn(M, N, device=dev).to(dt) if res else None
    out = torch.empty(M, N, device=dev, dtype=dt)
    for _ in range(int(os.environ.get("ITERS", "5"))):
        ops.gemm(a, w, b, residual=r, out=out)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
