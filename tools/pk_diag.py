"""Diagnose persistent-GEMM mismatches for one (dtype, cfg, shape): where the wrong elements sit
(tile, row/col within the tile) and what they look like (residual / bias missing or stale)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402

dev = torch.device("cuda", 0)
dt = torch.float16
for M, N, K, res, bias, act in ((12544, 512, 512, True, True, "gelu"), (12544, 512, 512, True, True, None),
                                (12544, 512, 512, False, True, "gelu"), (12544, 512, 512, True, False, "gelu"),
                                (12544, 512, 256, True, True, "gelu"), (25088, 512, 512, True, True, "gelu"),
                                (12544, 256, 512, True, True, "gelu")):
    g = torch.Generator(device=dev).manual_seed(7)
    a = torch.randn(M, K, device=dev, generator=g).to(dt)
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
    b = torch.randn(N, device=dev, generator=g) if bias else None
    r = torch.randn(M, N, device=dev, generator=g).to(dt) if res else None
    os.environ["SVK_NO_PK"] = "1"
    ref = ops.gemm(a, w, b, act=act, residual=r).float()
    del os.environ["SVK_NO_PK"]
    ops.tune("pk_cfg", 30)
    got = ops.gemm(a, w, b, act=act, residual=r).float()
    ops.tune("pk_cfg", -1)
    bad = ((got - ref).abs() > 4e-3 * (1 + ref.abs())).nonzero()
    print(f"M{M} N{N} K{K} res={res} bias={bias} act={act}: {len(bad)} bad", flush=True)
    if len(bad) == 0:
        continue
    ntn = N // 64
    tiles = (bad[:, 0] // 64) * ntn + bad[:, 1] // 64
    ut = torch.unique(tiles)
    print("  tiles:", ut[:20].tolist(), "count", len(ut))
    print("  rows in tile:", torch.unique(bad[:, 0] % 64).tolist()[:40])
    print("  cols in tile:", torch.unique(bad[:, 1] % 64).tolist()[:40])
    for (m, n) in bad[:6].tolist():
        rv = float(r[m, n]) if r is not None else 0.0
        bv = float(b[n]) if b is not None else 0.0
        print(f"  ({m},{n}) got {float(got[m, n]):.4f} ref {float(ref[m, n]):.4f} r {rv:.4f} b {bv:.4f}")
