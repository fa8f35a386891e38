"""Shared host-side helpers for the drop-in modules."""
import torch
import torch.nn as nn

import svk
from svk import ops


def pair(x):
    return tuple(x) if isinstance(x, (tuple, list)) else (x, x)


def compute_dtype(module):
    dt = getattr(module, "svk_dtype", None)
    return dt if dt is not None else svk.default_dtype()


def check_inference(module, *tensors):
    """The svk path implements the eval-mode forward; fail loudly instead of silently
    mis-computing train-mode semantics (DropPath / Dropout2d / batch-statistics BN)."""
    if module.training:
        raise svk.SvkError(f"{type(module).__name__}: train-mode forward is not implemented by the svk kernels "
                           "yet; call .eval() (DropPath/Dropout/BN-batch-stat semantics would differ)")
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise svk.SvkError(f"{type(module).__name__}: inputs must be on the GPU (got {t.device}); "
                               "the MI355X build has no CPU path")


def to_nhwc(x, dtype):
    """[B, C, H, W] (any float) -> contiguous NHWC in the compute dtype via the svk packing kernel,
    channels zero-padded per svk.pack.pad_channels (2/3-channel inputs -> 8)."""
    from svk.pack import pad_channels
    if x.dtype != torch.float32:
        x = x.float()
    return ops.nchw_to_nhwc(x.contiguous(), dtype, cpad=pad_channels(x.shape[1]))


class DropPath(nn.Module):
    """Stochastic depth (timm.layers.DropPath semantics); identity in eval mode."""

    def __init__(self, drop_prob=0.):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        if self.drop_prob == 0. or not self.training:
            return x
        raise svk.SvkError("DropPath in train mode is not implemented by the svk path yet")

    def extra_repr(self):
        return f"drop_prob={self.drop_prob}"
