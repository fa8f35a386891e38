"""Repeat svk_bn_bwd (BN train backward + ReLU, the head's linear_fuse.bn shape [147, 2048] f32) on fixed inputs
and classify every non-reproducible result: which rows / channels moved, and whether the wrong dX equals the
value computed with the channel sums (dbeta = sum dy', dgamma = sum dy'*xhat) still zero, i.e. the apply kernel
having read the gradient buffers before the reduction kernel's atomics reached them."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd"), REPO]
from svk import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n_iter = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    M, C = int(os.environ.get("M", 147)), int(os.environ.get("C", 2048))
    g = torch.Generator().manual_seed(0)
    X = torch.randn(M, C, generator=g).to(dev)
    dY = (torch.randn(M, C, generator=g) * 1e-2).to(dev)
    gamma = (1 + 0.1 * torch.randn(C, generator=g)).to(dev)
    beta = (0.1 * torch.randn(C, generator=g)).to(dev)
    s1, s2 = X.sum(0), (X * X).sum(0)
    flat = torch.zeros(2 * C + 64, device=dev)
    dgam, dbet = flat[:C], flat[C + 16:2 * C + 16]
    ref = None
    # host model of the formula with correct and with zero channel sums
    Xd, dYd = X.double().cpu(), dY.double().cpu()
    mean = s1.double().cpu() / M
    rstd = torch.rsqrt((s2.double().cpu() / M - mean * mean).clamp_min(0) + 1e-5)
    xh = (Xd - mean) * rstd
    d = torch.where(xh * gamma.double().cpu() + beta.double().cpu() <= 0, torch.zeros_like(dYd), dYd)
    sdy, sdyx = d.sum(0), (d * xh).sum(0)
    good = gamma.double().cpu() * rstd / M * (M * d - sdy - xh * sdyx)
    zero = gamma.double().cpu() * rstd / M * (M * d)
    nbad = 0
    for it in range(n_iter):
        flat.zero_()
        dx = ops.bn_bwd(X, dY, s1, s2, gamma, beta, 1e-5, dgam, dbet, relu=True)
        if ref is None:
            ref = dx.clone()
            e = (ref.double().cpu() - good).abs().max().item() / good.abs().max().item()
            print(f"first call vs host formula: rel {e:.3e}", flush=True)
            continue
        diff = (dx - ref).abs()
        if diff.max().item() > 1e-5 * ref.abs().max().item():
            nbad += 1
            bad = diff > 1e-5 * ref.abs().max().item()
            rows = bad.any(1).nonzero().flatten().tolist()
            cols = bad.any(0).nonzero().flatten().tolist()
            dc = dx.double().cpu()
            ez = ((dc - zero).abs()[bad.cpu()]).max().item()
            eg = ((dc - good).abs()[bad.cpu()]).max().item()
            # linear index range of the bad elements (apply kernel: one element per thread, 256 per block)
            li = bad.flatten().nonzero().flatten()
            print(f"iter {it}: {int(bad.sum())} elements in {len(rows)} rows x {len(cols)} channels; "
                  f"linear idx {li.min().item()}..{li.max().item()} (blocks {li.min().item() // 256}..{li.max().item() // 256}); "
                  f"max|dx - zero-sum model| {ez:.3e}, max|dx - correct| {eg:.3e}; dgamma/dbeta "
                  f"{(dgam.sum().item(), dbet.sum().item())}", flush=True)
            if nbad >= 20:
                break
    print(f"{nbad} non-reproducible results in {n_iter} calls")


if __name__ == "__main__":
    main()
