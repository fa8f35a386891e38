"""One GEMM shape, one kernel configuration, a few launches (for rocprofv3 counter passes).
Usage: python tools/pp_one.py M N K cfg [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402


def main():
    M, N, K, cfg = (int(v) for v in sys.argv[1:5])
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    dev = torch.device("cuda:0")
    a = (torch.rand(M, K, device=dev) * 2 - 1).half()
    w = (torch.rand(N, K, device=dev) * 2 - 1).half()
    out = torch.empty(M, N, device=dev, dtype=torch.half)
    ops.tune("pk_cfg", cfg)
    for _ in range(reps):
        ops.gemm(a, w, None, out=out)
    torch.cuda.synchronize()
    print(ops._last_kernel(), flush=True)


if __name__ == "__main__":
    main()
