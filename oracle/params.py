"""Deterministic parameter generator (oracle / test infrastructure).

Weights are synthetic (no pretrained checkpoints exist in the container).  Every
tensor of a state dict is filled from its own numpy PCG64 stream seeded by
``crc32(name) ^ seed``, so the golden generator (which fills the *reference*
modules) and the tests on the GPU box (which fill the build's modules) get
bit-identical parameters from the key names and shapes alone.

Distributions loosely follow the reference's ``_init_weights``
(mix_transformer_evp.py:94-107: Linear trunc_normal std .02, Conv normal
sqrt(2/fan_out)), but LayerNorm / BatchNorm affine terms, biases and BN running
statistics are randomised so that every affine path is exercised by parity tests.
"""
import zlib

import numpy as np
import torch


def _rng(name, seed):
    return np.random.default_rng((zlib.crc32(name.encode()) ^ (seed * 0x9E3779B1)) & 0xFFFFFFFF)


def fill_tensor(name, shape, seed=0):
    """Return a float32 (or int64) numpy array for parameter ``name``."""
    shape = tuple(int(s) for s in shape)
    if name.endswith("num_batches_tracked"):
        return np.zeros(shape, dtype=np.int64)
    r = _rng(name, seed)
    if name.endswith("running_var"):
        return r.uniform(0.5, 1.5, size=shape).astype(np.float32)
    if name.endswith("running_mean"):
        return (0.1 * r.standard_normal(shape)).astype(np.float32)
    nd = len(shape)
    if nd <= 1:
        if name.endswith("weight"):          # LayerNorm / BatchNorm gamma
            return (1.0 + 0.1 * r.standard_normal(shape)).astype(np.float32)
        return (0.02 * r.standard_normal(shape)).astype(np.float32)   # biases, LN/BN beta
    if nd == 4:                              # Conv2d [Cout, Cin/g, kh, kw]
        cout, cin_g, kh, kw = shape
        fan_out = kh * kw * (1 if cin_g == 1 else cout)  # depthwise: fan_out //= groups
        std = float(np.sqrt(2.0 / fan_out))
        if cin_g != 1:
            std = min(std, float(np.sqrt(1.0 / (cin_g * kh * kw))))
        return (std * r.standard_normal(shape)).astype(np.float32)
    if nd == 3:                              # Conv1d [Cout, Cin, k]
        std = float(np.sqrt(1.0 / (shape[1] * shape[2])))
        return (std * r.standard_normal(shape)).astype(np.float32)
    if name.endswith("in_proj_weight"):      # nn.MultiheadAttention xavier-like
        std = float(np.sqrt(2.0 / (shape[0] // 3 + shape[1])))
        return (std * r.standard_normal(shape)).astype(np.float32)
    # Linear [out, in]: trunc_normal std .02 is too small to keep signal through deep
    # stacks of random blocks; use 1/sqrt(fan_in) scaled down so activations stay O(1).
    std = float(min(0.05, 1.0 / np.sqrt(shape[1])))
    return (std * np.clip(r.standard_normal(shape), -2.0, 2.0)).astype(np.float32)


def make_state_dict(shapes, seed=0, dtype=torch.float32):
    """``shapes``: mapping name -> shape (e.g. ``{k: v.shape for k, v in m.state_dict().items()}``)."""
    out = {}
    for name, shape in shapes.items():
        a = fill_tensor(name, shape, seed)
        t = torch.from_numpy(a)
        if t.is_floating_point():
            t = t.to(dtype)
        out[name] = t
    return out


def fill_module_(module, seed=0):
    """Load deterministic parameters into an nn.Module in place (works for reference and build)."""
    sd = module.state_dict()
    new = make_state_dict({k: v.shape for k, v in sd.items()}, seed)
    module.load_state_dict(new, strict=True)
    return module
