"""Functional CPU restatement of mstcn.CausalMambaModel (oracle / test infrastructure only).

The reference's model (mstcn.py:282-343) stacks ``mamba_ssm.Mamba`` blocks (imported at mstcn.py:9).
``mamba_ssm`` is a third-party package that is absent from /root/reference and from this image, and the
reference pins no version (no requirements file); the restatement follows the published Mamba v1 block
(``mamba_ssm/modules/mamba_simple.py``: ``Mamba.forward`` and the reference scan
``mamba_ssm/ops/selective_scan_interface.py::selective_scan_ref``, mamba_ssm 1.x/2.x, identical in both):

    xz = in_proj(x)                          (bias=False)      x, z = xz.chunk(2)
    x  = silu(conv1d(x)[..., :L])            depthwise, kernel d_conv, padding d_conv-1, bias=True
    dt, B, C = split(x_proj(x), [dt_rank, d_state, d_state])   (x_proj bias=False)
    delta = softplus(dt_proj.weight @ dt + dt_proj.bias)
    h_t = exp(delta_t * A) h_{t-1} + delta_t * B_t * x_t,   A = -exp(A_log)
    y_t = C_t . h_t + D * x_t ;  y = y * silu(z) ;  out = out_proj(y)   (bias=False)

**Parity unpinned**: no golden vectors exist for Mamba (the package cannot run here and the reference holds
no fixtures); the GPU kernels are checked against this restatement only.  ``init_state_dict`` follows
mamba_simple.py's parameter initialisation semantics (A_log = log(1..d_state), D = 1, dt bias =
softplus^-1 of a log-uniform dt in [1e-3, 1e-1]) from the deterministic per-name streams of params.py.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import params


def mamba_shapes(f_dim, f_maps, layers, classes, d_state=64, d_conv=4, expand=2):
    """State-dict shapes of CausalMambaModel (mstcn.py:316-326) with mamba_ssm Mamba v1 blocks."""
    di = expand * f_maps
    R = math.ceil(f_maps / 16)
    s = {"in_proj.weight": (f_maps, f_dim), "in_proj.bias": (f_maps,)}
    for l in range(layers):
        p = f"blocks.{l}."
        s.update({p + "A_log": (di, d_state), p + "D": (di,), p + "in_proj.weight": (2 * di, f_maps),
                  p + "conv1d.weight": (di, 1, d_conv), p + "conv1d.bias": (di,),
                  p + "x_proj.weight": (R + 2 * d_state, di), p + "dt_proj.weight": (di, R),
                  p + "dt_proj.bias": (di,), p + "out_proj.weight": (f_maps, di)})
    s.update({"norm.weight": (f_maps,), "norm.bias": (f_maps,), "head.weight": (classes, f_maps),
              "head.bias": (classes,)})
    return s


def init_state_dict(shapes, seed=0):
    sd = params.make_state_dict(shapes, seed)
    for k, v in list(sd.items()):
        r = params._rng(k, seed)
        if k.endswith("A_log"):
            n = v.shape[1]
            sd[k] = torch.log(torch.arange(1, n + 1, dtype=torch.float32)).repeat(v.shape[0], 1)
        elif k.endswith(".D"):
            sd[k] = torch.from_numpy((1.0 + 0.1 * r.standard_normal(v.shape)).astype(np.float32))
        elif k.endswith("dt_proj.bias"):
            dt = np.exp(r.uniform(size=v.shape) * (math.log(0.1) - math.log(1e-3)) + math.log(1e-3))
            dt = np.maximum(dt, 1e-4)
            sd[k] = torch.from_numpy((dt + np.log(-np.expm1(-dt))).astype(np.float32))
    return sd


def selective_scan(u, delta, A, Bm, Cm, D, z):
    """selective_scan_ref: u, delta, z [Bt, L, Di]; A [Di, N]; Bm, Cm [Bt, L, N] -> [Bt, L, Di]."""
    Bt, L, Di = u.shape
    h = torch.zeros(Bt, Di, A.shape[1], dtype=u.dtype)
    ys = []
    for t in range(L):
        dA = torch.exp(delta[:, t, :, None] * A)
        h = dA * h + (delta[:, t, :, None] * u[:, t, :, None]) * Bm[:, t, None, :]
        ys.append((h * Cm[:, t, None, :]).sum(-1))
    y = torch.stack(ys, 1) + u * D
    return y * F.silu(z)


def mamba_block(x, sd, p, d_state, d_conv):
    """Mamba.forward (mamba_simple.py) on x [Bt, L, d_model]."""
    L = x.shape[1]
    xz = x @ sd[p + "in_proj.weight"].t()
    xi, z = xz.chunk(2, dim=-1)
    di = xi.shape[-1]
    xc = F.conv1d(xi.transpose(1, 2), sd[p + "conv1d.weight"], sd[p + "conv1d.bias"], padding=d_conv - 1,
                  groups=di)[..., :L]
    xc = F.silu(xc).transpose(1, 2)
    xdbl = xc @ sd[p + "x_proj.weight"].t()
    R = sd[p + "dt_proj.weight"].shape[1]
    dt, Bm, Cm = torch.split(xdbl, [R, d_state, d_state], dim=-1)
    delta = F.softplus(dt @ sd[p + "dt_proj.weight"].t() + sd[p + "dt_proj.bias"])
    A = -torch.exp(sd[p + "A_log"])
    y = selective_scan(xc, delta, A, Bm, Cm, sd[p + "D"], z)
    return y @ sd[p + "out_proj.weight"].t()


def causal_mamba(x, sd, layers, d_state=64, d_conv=4, dtype=torch.float64, masks=None):
    """CausalMambaModel.forward (mstcn.py:327-343): x [B, f_dim, T] -> [1, B, classes, T].  Eval: dropout
    identity; ``masks`` [L, B*T, F] (0 or 1/keep, time-major rows b*T + t): the train-mode
    ``x = dropout(x + blk(x))`` draws (mstcn.py:335-336)."""
    sd = {k: v.to(dtype) for k, v in sd.items()}
    h = x.to(dtype).transpose(1, 2) @ sd["in_proj.weight"].t() + sd["in_proj.bias"]
    for l in range(layers):
        h = h + mamba_block(h, sd, f"blocks.{l}.", d_state, d_conv)
        if masks is not None:
            h = h * masks[l].to(dtype).view(h.shape)
    h = F.layer_norm(h, (h.shape[-1],), sd["norm.weight"], sd["norm.bias"], 1e-5)
    logits = h @ sd["head.weight"].t() + sd["head.bias"]
    return logits.transpose(1, 2).unsqueeze(0)
