"""CPU restatement of generate_phase_anticipation.generate_anticipation_gt (oracle / test infrastructure only).

generate_phase_anticipation.py:10-30: walking each phase's presence signal backwards, count = 0 where the
phase is present, otherwise min(horizon, count + 1/1500) (Python float), starting at count = horizon; stored
into a FloatTensor (f32) and divided by horizon (f32 tensor op); :33-34 stacks the phases and permutes to
[T, P].  Pinned by tests/golden/anticipation_golden.npz, produced by the reference function itself
(tests/golden/gen_anticipation.py).
"""
import torch


def anticipation_gt_onephase(code, horizon):
    out = torch.zeros(len(code), dtype=torch.float32)
    count = horizon
    for i in range(len(code) - 1, -1, -1):
        count = 0 if code[i] else min(horizon, count + 1 / 1500)
        out[i] = count
    return out / horizon


def anticipation_gt(phases, horizon):
    return torch.stack([anticipation_gt_onephase(c.tolist(), horizon) for c in phases]).permute(1, 0)
