"""Locate persistent-GEMM mismatches for one (dtype, cfg, shape) and identify what the wrong values are:
the register they live in (wave, fragment block, lane group, component of the transposed 16x16x32 MFMA
layout), whether the same elements are wrong on every launch, and which candidate stale value they equal:
the result without the last MFMA's k-slice (an accumulator read before its MFMA finished), without
bias / residual, or the previous tile's value at the same register position."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402

dev = torch.device("cuda", 0)
dt = torch.float16
cfg = int(os.environ.get("PK_CFG", "30"))
BM = BN = 64
WM = WN = 32


def epi(acc, b, act, r):
    v = acc + (b if b is not None else 0)
    if act == "gelu":
        v = torch.nn.functional.gelu(v)
    return v + (r.float() if r is not None else 0)


for M, N, K, res, bias, act in ((12544, 512, 512, True, True, "gelu"), (12544, 512, 512, True, True, None),
                                (12544, 512, 512, False, True, "gelu"), (12544, 512, 512, True, False, "gelu"),
                                (12544, 512, 256, True, True, "gelu"), (12544, 512, 64, True, True, "gelu")):
    g = torch.Generator(device=dev).manual_seed(7)
    a = torch.randn(M, K, device=dev, generator=g).to(dt)
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
    b = torch.randn(N, device=dev, generator=g) if bias else None
    r = torch.randn(M, N, device=dev, generator=g).to(dt) if res else None
    full = a.float() @ w.float().t()
    ref = epi(full, b, act, r)
    ops.tune("pk_cfg", cfg)
    runs = [ops.gemm(a, w, b, act=act, residual=r).float() for _ in range(5)]
    ops.tune("pk_cfg", -1)
    bads = [((x - ref).abs() > 4e-3 * (1 + ref.abs())) for x in runs]
    n = [int(x.sum()) for x in bads]
    print(f"M{M} N{N} K{K} res={res} bias={bias} act={act}: bad per launch {n}", flush=True)
    if not any(n):
        continue
    k = max(range(5), key=lambda i: n[i])
    got, bad = runs[k], bads[k].nonzero()
    same = all(torch.equal(bads[k], x) for x in bads if x.any())
    print(f"  same positions on every failing launch: {same}")
    m64, n64 = bad[:, 0] % BM, bad[:, 1] % BN
    regs = set()
    for mm, nn in zip(m64.tolist(), n64.tolist()):
        wm, i, fr = mm // WM, (mm % WM) // 16, mm % 16
        wn, j, fq, c = nn // WN, (nn % WN) // 16, (nn % 16) // 4, nn % 4
        regs.add((wm, wn, i, j, fq, c))
    print(f"  registers (wm, wn, i, j, lane group fq, component): {sorted(regs)[:12]} ({len(regs)} distinct)")
    print(f"  tiles: {torch.unique((bad[:, 0] // BM) * (N // BN) + bad[:, 1] // BN).tolist()[:16]}")
    part = {s: epi(a[:, :K - s].float() @ w[:, :K - s].float().t(), b, act, r) for s in (32, 64) if s < K}
    for (mm, nn) in bad[:8].tolist():
        gv = float(got[mm, nn])
        cands = {"ref": float(ref[mm, nn])}
        for s, pv in part.items():
            cands[f"no_last_{s}k"] = float(pv[mm, nn])
        cands["no_bias"] = float(epi(full[mm, nn], None, act, r[mm, nn] if r is not None else None))
        if r is not None:
            cands["no_res"] = float(epi(full[mm, nn], b[nn] if b is not None else None, act, None))
        best = min(cands, key=lambda c: abs(cands[c] - gv))
        print(f"  ({mm},{nn}) got {gv:.4f} | " + " ".join(f"{c} {v:.4f}" for c, v in cands.items()) + f" -> closest {best}")
