"""SegFormer decode head — MI355X build (drop-in for the reference's models/segformer_head.py).

Same submodules and state_dict keys as the reference (``linear_c1..4.proj``,
``linear_fuse.{conv,bn}``, ``fc``, ``fc_ant``).  The eval-mode arithmetic is
restructured, exactly, for the hardware (segformer_head.py:137-179):

* resize-before-linear: the per-token Linear commutes with the bilinear resize
  (both linear, bilinear weights sum to 1), so c1/c2/c3 are resized to the 7x7 c4 grid
  first and never materialised at 2048 channels (the reference builds a
  [B, 2048, 56, 56] map per frame just to sample 196 of its pixels);
* the four per-level Linears, the 1x1 fuse conv and the eval BatchNorm are one linear
  map, so they are folded (in fp64, once per weight version) into a single
  [2048, sum(C_i)] matrix + bias: one MFMA GEMM with a ReLU epilogue over the 49
  resized tokens, then a row-mean for the adaptive average pool.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from svk import ops
from svk.pack import get_packed, lin_w, lin_b
from ._common import check_inference


def resize(input, size=None, scale_factor=None, mode="nearest", align_corners=None, warning=True):
    """Reference helper (segformer_head.py:10-29); torch interpolate, kept for API compatibility."""
    return F.interpolate(input, size, scale_factor, mode, align_corners)


class MLP(nn.Module):
    """Linear embedding (segformer_head.py:32-43)."""

    def __init__(self, input_dim=2048, embed_dim=768):
        super().__init__()
        self.proj = nn.Linear(input_dim, embed_dim)

    def forward(self, x):
        """x [B, C, H, W] (or tokens [B, N, C]) -> [B, H*W, embed_dim]."""
        check_inference(self, x)
        if x.dim() == 4:
            x = x.flatten(2).transpose(1, 2)
        p = get_packed(self, x.dtype, lambda d: dict(w=lin_w(self.proj, d), b=lin_b(self.proj)))
        return ops.gemm(x.contiguous(), p["w"], p["b"])


class ConvModule(nn.Module):
    """mmcv.cnn.ConvModule as configured at segformer_head.py:74-80: 1x1 conv (no bias, a norm
    follows) -> BatchNorm2d named ``bn`` -> ReLU named ``activate``."""

    def __init__(self, in_channels, out_channels, kernel_size, norm_cfg=None, **kw):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, bias=norm_cfg is None)
        if norm_cfg is not None:
            self.bn = nn.BatchNorm2d(out_channels)
        self.activate = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.activate(self.bn(self.conv(x)) if hasattr(self, "bn") else self.conv(x))


class SegFormerHead(nn.Module):
    def __init__(self, in_channels, num_classes):
        super().__init__()
        self.input_transform = "multiple_select"
        self.embedding_dim = 2048
        self.embedding_dim1 = 2048
        self.in_index = [0, 1, 2, 3]
        self.align_corners = False
        self.dropout = nn.Dropout2d(0.1)
        self.in_channels = in_channels
        self.num_classes = num_classes
        c1, c2, c3, c4 = in_channels
        E = self.embedding_dim
        self.linear_c4 = MLP(input_dim=c4, embed_dim=E)
        self.linear_c3 = MLP(input_dim=c3, embed_dim=E)
        self.linear_c2 = MLP(input_dim=c2, embed_dim=E)
        self.linear_c1 = MLP(input_dim=c1, embed_dim=E)
        self.linear_fuse = ConvModule(in_channels=E * 4, out_channels=E, kernel_size=1, norm_cfg=dict(type="BN"))
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Sequential(nn.Linear(2048, 512), nn.ReLU(), nn.Linear(512, 7))
        self.fc_ant = nn.Sequential(nn.Linear(2048, 512), nn.ReLU(), nn.Linear(512, 7))

    def _pack(self, dt):
        """Fold linear_c{4,3,2,1} -> concat -> 1x1 conv -> BN(eval) into W [E, sum C_i] (K order c4|c3|c2|c1)."""
        E = self.embedding_dim
        bn = self.linear_fuse.bn
        wf = self.linear_fuse.conv.weight.detach().double().reshape(E, 4 * E)
        s = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
        ws, bias = [], -bn.running_mean.detach().double()
        for i, lin in enumerate((self.linear_c4, self.linear_c3, self.linear_c2, self.linear_c1)):
            blk = wf[:, i * E:(i + 1) * E]
            ws.append(blk @ lin.proj.weight.detach().double())
            bias = bias + blk @ lin.proj.bias.detach().double()
        w = torch.cat(ws, dim=1) * s[:, None]
        b = bias * s + bn.bias.detach().double()
        heads = {}
        for name, seq in (("fc", self.fc), ("fc_ant", self.fc_ant)):
            heads[name] = (lin_w(seq[0], torch.float32), lin_b(seq[0]), lin_w(seq[2], torch.float32), lin_b(seq[2]))
        return dict(w=w.to(dt).contiguous(), b=b.float().contiguous(), heads=heads)

    def forward_tokens(self, outs, return_features=False):
        """outs: [(tokens [B, H_i*W_i, C_i], H_i, W_i)] for c1..c4 (NHWC token order)."""
        p = get_packed(self, outs[0][0].dtype, self._pack)
        (t1, H1, W1), (t2, H2, W2), (t3, H3, W3), (t4, H4, W4) = outs
        B = t4.shape[0]
        ctot = sum(t.shape[-1] for t, _, _ in outs)
        r = torch.empty(B, H4 * W4, ctot, device=t4.device, dtype=t4.dtype)
        levels = ((t4, H4, W4), (t3, H3, W3), (t2, H2, W2), (t1, H1, W1))   # torch.cat order (:158)
        if ops.RESIZE_MULTI and r.dtype in ops.H16 and all(t.shape[-1] % 8 == 0 for t, _, _ in levels):
            ops.resize_bilinear_multi(levels, H4, W4, r)                         # the four resizes, one launch
        else:
            off = 0
            for t, H, W in levels:
                C = t.shape[-1]
                ops.resize_bilinear(t, H, W, H4, W4, out=r[:, :, off:off + C])
                off += C
        y = ops.gemm(r.view(B * H4 * W4, ctot), p["w"], p["b"], act="relu")
        x = ops.mean_rows(y, H4 * W4)                                            # [B, 2048] f32
        if return_features:
            return x
        outs_ = []
        for name in ("fc", "fc_ant"):
            w0, b0, w2, b2 = p["heads"][name]
            h = ops.gemm(x, w0, b0, act="relu")
            outs_.append(ops.gemm(h, w2, b2))
        return outs_[0], outs_[1]

    def forward(self, inputs, return_features=False):
        """Reference signature: inputs = [c1, c2, c3, c4] NCHW maps (segformer_head.py:137)."""
        check_inference(self, *inputs)
        outs = []
        for c in inputs:
            B, C, H, W = c.shape
            outs.append((c.permute(0, 2, 3, 1).reshape(B, H * W, C).contiguous(), H, W))
        return self.forward_tokens(outs, return_features)
