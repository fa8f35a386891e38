"""Phase-anticipation regression targets on the GPU: ``generate_anticipation_gt(phases, horizon)``
(generate_phase_anticipation.py:33-34) with the reference's signature and output ([T, P] float32)."""
import torch

from . import _lib
from .ops import _chk, _p, _stream


def generate_anticipation_gt(phases, horizon):
    """phases [P, T] (one-hot phase presence, any integer/bool dtype; the reference builds a LongTensor)
    -> [T, P] f32 targets in [0, 1] (generate_phase_anticipation.py:10-34)."""
    _chk(phases, "phases")
    if phases.dim() != 2:
        raise _lib.SvkError(f"svk.generate_anticipation_gt: phases must be [P, T], got {tuple(phases.shape)}")
    codes = phases if phases.dtype == torch.int64 else phases.to(torch.int64)
    codes = codes.contiguous()
    P, T = codes.shape
    out = torch.empty(T, P, device=codes.device, dtype=torch.float32)
    _lib.call("svk_anticipation_gt", _p(codes), T, P, T, float(horizon), _p(out), _stream())
    return out
