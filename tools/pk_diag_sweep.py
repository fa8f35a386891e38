"""gemm_pk timing ablations on the MiT-b2 shapes (svk_tune("pk_diag"): 1 = drain the stores after every
tile's epilogue, 2 = no C stores), interleaved in one process.  Usage: python tools/pk_diag_sweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pk_cfg_sweep import SHAPES, timeit  # noqa: E402
from svk import ops, _lib  # noqa: E402


def main():
    dt, dev = torch.float16, torch.device("cuda:0")
    lib = _lib.load()
    for M, N, K, res, what in SHAPES:
        a = torch.randn(M, K, device=dev).to(dt)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(dt)
        b = torch.randn(N, device=dev)
        r = torch.randn(M, N, device=dev).to(dt) if res else None
        out = torch.empty(M, N, device=dev, dtype=dt)
        row = []
        for d in (0, 1, 2, 0):
            lib.svk_tune(b"pk_diag", d)
            ms = timeit(lambda: ops.gemm(a, w, b, residual=r, out=out), 30)
            row.append(f"d{d} {ms * 1e3:6.1f}us")
        lib.svk_tune(b"pk_diag", 0)
        ms = timeit(lambda: torch.matmul(a, w.t(), out=out), 30)
        print(f"{what:10s} {str((M, N, K)):18s} " + " | ".join(row) + f" | torch {ms * 1e3:6.1f}us", flush=True)


if __name__ == "__main__":
    main()
