"""Uninitialised-read probe for the f32 train step (tests/test_train_gpu.py::test_train_step_grads_fp32_vs_oracle):
the caching allocator's free memory is filled with NaN before the step is built, so any kernel that reads device
memory nobody wrote (torch.empty buffers only partly written, reads past an operand's end) poisons its output.
Prints the loss and, per gradient tensor, NaN counts and the error against the fp64 oracle.
GPU box: python tools/b3_poison.py [variant] [poison_gb]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd")]
from oracle import inputs as I, params as P, train_evp as TR  # noqa: E402


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else "mit_b3_evp"
    gb = float(sys.argv[2]) if len(sys.argv) > 2 else 24.0
    from models import mix_transformer_evp as mte
    from svk.train import EVPTrainStep
    cuda = torch.device("cuda:0")
    B = 3
    m = getattr(mte, variant)()
    sd = P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0)
    m.load_state_dict(sd)
    g = torch.Generator().manual_seed(101)
    x, y, fl = I.frames(B, 1), I.segmaps(B, 1), I.flow(B, 1)
    lab, at = torch.randint(0, 7, (B,), generator=g), torch.rand(B, 7, generator=g)
    masks = TR.make_masks(B, variant, seed=5)
    lp, la, grads, stats = TR.loss_and_grads(x, y, fl, lab, at, sd, variant, masks)
    # poison: fill (almost) all the memory the caching allocator will hand out with NaN, then free it
    chunks = []
    for _ in range(int(gb)):
        t = torch.empty(1 << 28, device=cuda, dtype=torch.float32)   # 1 GiB
        t.fill_(float("nan"))
        chunks.append(t)
    torch.cuda.synchronize()
    del chunks
    m = m.to(cuda)
    tr = EVPTrainStep(m, dtype=torch.float32)
    loss, logits, ant = tr.forward_backward(x.to(cuda), y.to(cuda), fl.to(cuda), lab.to(cuda), at.to(cuda), masks=masks)
    torch.cuda.synchronize()
    print("loss gpu", loss.tolist(), "oracle", [lp.item(), la.item()], flush=True)
    gmax = max(v.abs().max().item() for v in grads.values())
    rows = []
    for nm, b in grads.items():
        a = tr.params[nm].grad.detach().double().cpu()
        nan = int(torch.isnan(a).sum())
        scale = max(b.abs().max().item(), 1e-3 * gmax)
        err = (torch.nan_to_num(a, nan=0.0) - b).abs().max().item() / scale
        rows.append((nan, err, nm))
    rows.sort(key=lambda r: (-r[0], -r[1]))
    for nan, err, nm in rows[:25]:
        print(f"{nm:60s} nan {nan:8d} err/scale {err:.2e}", flush=True)
    print("tensors with NaN:", sum(1 for r in rows if r[0]), "of", len(rows), flush=True)


if __name__ == "__main__":
    main()
