"""Sequence Transformer over MS-TCN outputs — MI355X build (drop-in for models/adapter_transformer.py).

``Transformer(mstcn_f_maps, mstcn_f_dim, out_features, len_q)`` keeps the reference's
constructor, attributes and state_dict keys (``fc.weight`` + ``transformer.*``,
adapter_transformer.py:290-327).  ``original_forward`` (adapter_transformer.py:329-352)
replaces the per-frame Python loop — one zero-padded slice + ``torch.cat`` + a
``.cuda()`` allocation per frame — with one window-unfold kernel (which also adds
Transformer2_3_1's position table), and ``tanh(fc(long_feature))`` with one GEMM whose
epilogue applies the tanh.
"""
import torch
import torch.nn as nn

from svk import ops, temporal
from svk.pack import get_packed, lin_w
from ._common import check_inference
from .transformer2_3_1 import Transformer2_3_1

sequence_length = 30


class Transformer(nn.Module):
    def __init__(self, mstcn_f_maps, mstcn_f_dim, out_features, len_q, img_size=224, in_chans=3, embed_dim=64,
                 drop_rate=0., norm_layer=nn.LayerNorm, **kwargs):
        super().__init__()
        self.num_f_maps = mstcn_f_maps
        self.dim = mstcn_f_dim
        self.num_classes = out_features
        self.len_q = len_q
        self.chunk_size = 256
        attn_dim = min(64, self.num_f_maps)
        self.transformer = Transformer2_3_1(d_model=out_features, d_ff=self.num_f_maps, d_k=attn_dim, d_v=attn_dim,
                                            n_layers=1, n_heads=4, len_q=sequence_length)
        self.fc = nn.Linear(mstcn_f_dim, out_features, bias=False)

    def original_forward(self, x, long_feature):
        """x [1, classes, T] (MS-TCN last stage), long_feature [1, T, f_dim] -> [T, 1, classes].
        Train mode (tecno_trans.py:226-292): forward and backward on svk kernels (svk.temporal)."""
        if self.training:
            return temporal.transformer_autograd_forward(self, x, long_feature)
        check_inference(self, x, long_feature)
        xt = x[0].t()                                   # [T, classes]
        if xt.dtype != torch.float32 or xt.stride(1) != 1:
            xt = xt.float().contiguous()
        T = xt.shape[0]
        pos = self.transformer.pos_table if self.len_q == self.transformer.len_q else None
        inputs = ops.window_unfold(xt, self.len_q, pos=pos)                     # [T, len_q, classes]
        lf = long_feature[0]
        if lf.dtype != torch.float32 or lf.stride(1) != 1:
            lf = lf.float().contiguous()
        p = get_packed(self, torch.float32, lambda d: dict(w=lin_w(self.fc, torch.float32)))
        feas = ops.gemm(lf, p["w"], None, act="tanh").view(T, 1, self.num_classes)   # tanh(fc(lt)).transpose(0,1)
        if pos is None:
            return self.transformer(inputs, feas)
        return self.transformer.forward_encoded(inputs, feas)

    def forward(self, x, long_feature):
        return self.original_forward(x, long_feature)
