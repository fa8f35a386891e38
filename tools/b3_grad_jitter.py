"""Run-to-run spread of the f32 train-step gradients of mit_b3_evp (tests/test_train_gpu.py::
test_train_step_grads_fp32_vs_oracle): the fp64 oracle once, the GPU step N times on the same inputs; prints the
worst err / scale per run against the oracle and the largest run-to-run difference per tensor.
GPU box: python tools/b3_grad_jitter.py [N] [variant]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd")]
from oracle import inputs as I, params as P, train_evp as TR  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    variant = sys.argv[2] if len(sys.argv) > 2 else "mit_b3_evp"
    from models import mix_transformer_evp as mte
    from svk.train import EVPTrainStep
    cuda = torch.device("cuda:0")
    m = getattr(mte, variant)()
    sd = P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0)
    m.load_state_dict(sd)
    m = m.to(cuda)
    B = 3
    g = torch.Generator().manual_seed(101)
    x, y, fl = I.frames(B, 1), I.segmaps(B, 1), I.flow(B, 1)
    lab, at = torch.randint(0, 7, (B,), generator=g), torch.rand(B, 7, generator=g)
    masks = TR.make_masks(B, variant, seed=5)
    lp, la, grads, stats = TR.loss_and_grads(x, y, fl, lab, at, sd, variant, masks)
    gmax = max(v.abs().max().item() for v in grads.values())
    runs = []
    for k in range(n):
        tr = EVPTrainStep(m, dtype=torch.float32)
        tr.forward_backward(x.to(cuda), y.to(cuda), fl.to(cuda), lab.to(cuda), at.to(cuda), masks=masks)
        torch.cuda.synchronize()
        gr = {nm: tr.params[nm].grad.detach().double().cpu().clone() for nm in grads}
        runs.append(gr)
        worst = []
        for nm, b in grads.items():
            scale = max(b.abs().max().item(), 1e-3 * gmax)
            worst.append(((gr[nm] - b).abs().max().item() / scale, nm))
        worst.sort(reverse=True)
        print(f"run {k}: worst err/scale " + ", ".join(f"{nm} {r:.2e}" for r, nm in worst[:5]), flush=True)
    if n > 1:
        diffs = []
        for nm, b in grads.items():
            scale = max(b.abs().max().item(), 1e-3 * gmax)
            d = max((runs[k][nm] - runs[0][nm]).abs().max().item() for k in range(1, n))
            diffs.append((d / scale, nm))
        diffs.sort(reverse=True)
        print("run-to-run max diff / scale: " + ", ".join(f"{nm} {r:.2e}" for r, nm in diffs[:8]), flush=True)


if __name__ == "__main__":
    main()
