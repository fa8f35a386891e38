"""Large square GEMMs (f16, uniform random [-1, 1)): gemm_pp / gemm_pk / hipBLASLt, to separate the kernel's
own throughput from the tile-quantisation and L2 effects of the MiT shapes.  GPU box: python tools/pp_square.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pk_cfg_sweep import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for M, N, K in ((4096, 4096, 4096), (8192, 8192, 8192), (8192, 8192, 1024), (16384, 4096, 1024)):
        a = (torch.rand(M, K, device=dev) * 2 - 1).half()
        w = (torch.rand(N, K, device=dev) * 2 - 1).half()
        out = torch.empty(M, N, device=dev, dtype=torch.half)
        row = []
        for cfg, name in ((60, "128x128e"), (70, "ppRF"), (71, "ppPair")):
            ops.tune("pk_cfg", cfg)
            ops.gemm(a, w, None, out=out)
            kn = ops._last_kernel()
            ms = timeit(lambda: ops.gemm(a, w, None, out=out), 10)
            row.append(f"{name} {ms * 1e3:8.1f}us {2 * M * N * K / ms / 1e9:6.0f}TF{'' if cfg < 70 or kn.startswith('gemm_pp') else ' (fallback)'}")
        ops.tune("pk_cfg", -1)
        ms = timeit(lambda: torch.matmul(a, w.t(), out=out), 10)
        row.append(f"torch {ms * 1e3:8.1f}us {2 * M * N * K / ms / 1e9:6.0f}TF")
        print(f"({M},{N},{K}) " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
