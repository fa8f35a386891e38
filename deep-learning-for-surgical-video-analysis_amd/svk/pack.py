"""Weight packing for the svk kernels (one-time layout work, cached per module).

Packed forms are derived from a module's fp32 parameters on first use for a given
(dtype, device) and re-derived whenever any parameter's version counter changes
(load_state_dict, optimizer steps and in-place edits all bump it), so the
nn.Module parameters stay the single source of truth and the state_dict keeps the
reference's keys.
"""
import torch


class PackCache:
    def __init__(self):
        self._key = None
        self._val = None

    def get(self, module, dtype, builder):
        params = list(module.parameters()) + [b for b in module.buffers()]
        dev = params[0].device if params else torch.device("cpu")
        key = (dtype, dev, tuple((id(p), p._version) for p in params))
        if key != self._key:
            with torch.no_grad():
                self._val = builder(dtype)
            self._key = key
        return self._val


def get_packed(module, dtype, builder):
    cache = module.__dict__.get("_svk_pack_cache")
    if cache is None:
        cache = PackCache()
        module.__dict__["_svk_pack_cache"] = cache
    return cache.get(module, dtype, builder)


def lin_w(linear, dtype):
    return linear.weight.detach().to(dtype).contiguous()


def lin_b(linear):
    return None if linear.bias is None else linear.bias.detach().float().contiguous()


def pad_channels(cin):
    """Input channel count the NHWC maps of a conv with ``cin`` inputs are stored with: 2/3-channel
    inputs (frames, segmap, flow) are zero-padded to 8 so the implicit-GEMM conv can use 16-byte
    loads (one 8-channel chunk per tap)."""
    return 8 if cin < 8 else cin


def conv_w(weight, dtype, cin_pad=None):
    """[Cout, Cin, k, k] -> [Cout, k*k*Cin'] in (kh, kw, ci) order (the implicit-GEMM K order),
    Cin' = cin_pad (zero weights for the padded input channels) or Cin."""
    co, ci = weight.shape[:2]
    w = weight.detach().permute(0, 2, 3, 1)
    if cin_pad is not None and cin_pad > ci:
        w = torch.nn.functional.pad(w, (0, cin_pad - ci))
    return w.reshape(co, -1).to(dtype).contiguous()


def conv_w_s2d(weight, dtype, s):
    """[Cout, Cin, k, k] (k <= 2s) -> [Cout, 2*2*s*s*Cin] for the 2x2 conv over space-to-depth blocks
    (svk_nchw_to_s2d): K order (by, bx, dy, dx, ci) with tap (ky, kx) = (s*by + dy, s*bx + dx); taps
    beyond k are zero."""
    co, ci, k, _ = weight.shape
    w = torch.nn.functional.pad(weight.detach(), (0, 2 * s - k, 0, 2 * s - k))       # [co, ci, 2s, 2s]
    w = w.reshape(co, ci, 2, s, 2, s).permute(0, 2, 4, 3, 5, 1)                    # [co, by, bx, dy, dx, ci]
    return w.reshape(co, -1).to(dtype).contiguous()


def fold_bn(weight, bias, bn):
    """Fold an eval-mode BatchNorm into the preceding conv: returns fp64 (w', b')."""
    w = weight.detach().double()
    b = bias.detach().double() if bias is not None else torch.zeros(w.shape[0], dtype=torch.float64, device=w.device)
    s = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    w = w * s.reshape(-1, *([1] * (w.dim() - 1)))
    b = (b - bn.running_mean.detach().double()) * s + bn.bias.detach().double()
    return w, b
