"""Transformer2_3_1 — build-defined (the reference snapshot does not contain transformer2_3_1.py).

Only its call-site contract is known: ``Transformer2_3_1(d_model, d_ff, d_k, d_v, n_layers,
n_heads, len_q)`` (adapter_transformer.py:317-325) and ``forward(enc_inputs [T, len_q,
d_model], dec_inputs [T, 1, d_model]) -> [T, 1, d_model]`` (adapter_transformer.py:348,
trans_SV_output.py:291-296).  This module implements a post-LN encoder (multi-head
self-attention over the len_q window + ReLU FFN, ``n_layers`` deep, a fixed sinusoidal
position table added to the window) and a one-layer decoder in which the single query
token (the spatial embedding) self-attends, cross-attends to the encoded window and goes
through a FFN.  **Parity unpinned**: tests check it against the build's own CPU
restatement (oracle/trans_sv.py), not against the (absent) reference.

Every op runs in svk kernels: fused Q|K|V projection GEMMs, the short-sequence attention
kernel (one workgroup per (frame, head)), output projections with the residual add in the
GEMM epilogue, LayerNorm, and the FFN GEMMs with ReLU epilogues.  f32 throughout.
"""
import math

import torch
import torch.nn as nn

from svk import ops
from svk.pack import get_packed, lin_w, lin_b


def sinusoid_table(n, d):
    pos = torch.arange(n, dtype=torch.float64)[:, None]
    i = torch.arange(d, dtype=torch.float64)[None, :]
    ang = pos / torch.pow(10000.0, 2 * torch.div(i, 2, rounding_mode="floor") / d)
    return torch.where(i % 2 == 0, torch.sin(ang), torch.cos(ang)).float()


class MultiHeadAttention(nn.Module):
    def __init__(self, d_model, d_k, d_v, n_heads):
        super().__init__()
        self.d_k, self.d_v, self.n_heads = d_k, d_v, n_heads
        self.W_Q = nn.Linear(d_model, d_k * n_heads)
        self.W_K = nn.Linear(d_model, d_k * n_heads)
        self.W_V = nn.Linear(d_model, d_v * n_heads)
        self.fc = nn.Linear(n_heads * d_v, d_model)
        self.layer_norm = nn.LayerNorm(d_model)

    def _pack(self, dt):
        f = torch.float32
        return dict(wq=lin_w(self.W_Q, f), bq=lin_b(self.W_Q),
                    wkv=torch.cat([lin_w(self.W_K, f), lin_w(self.W_V, f)], 0).contiguous(),
                    bkv=torch.cat([lin_b(self.W_K), lin_b(self.W_V)], 0).contiguous(),
                    wqkv=torch.cat([lin_w(self.W_Q, f), lin_w(self.W_K, f), lin_w(self.W_V, f)], 0).contiguous(),
                    bqkv=torch.cat([lin_b(self.W_Q), lin_b(self.W_K), lin_b(self.W_V)], 0).contiguous(),
                    wo=lin_w(self.fc, f), bo=lin_b(self.fc),
                    g=self.layer_norm.weight.detach().float().contiguous(),
                    beta=self.layer_norm.bias.detach().float().contiguous())

    def forward(self, Q, K, V):
        """Q [Bt, Lq, D]; K is V (the only use on this path) [Bt, Lk, D] -> LN(fc(attn) + Q)."""
        p = get_packed(self, torch.float32, self._pack)
        hk = self.n_heads * self.d_k
        Q = Q.contiguous()
        if Q is K and K is V:
            qkv = ops.gemm(Q, p["wqkv"], p["bqkv"])
            q, k, v = qkv[:, :, :hk], qkv[:, :, hk:2 * hk], qkv[:, :, 2 * hk:]
        else:
            if K is not V:
                raise ValueError("MultiHeadAttention: separate K and V inputs are not used on this path")
            q = ops.gemm(Q, p["wq"], p["bq"])
            kv = ops.gemm(K.contiguous(), p["wkv"], p["bkv"])
            k, v = kv[:, :, :hk], kv[:, :, hk:]
        o = ops.attention(q, k, v, self.n_heads, 1.0 / math.sqrt(self.d_k))
        o = ops.gemm(o, p["wo"], p["bo"], residual=Q)
        return ops.layernorm(o, p["g"], p["beta"], self.layer_norm.eps, out=o)


class PoswiseFeedForwardNet(nn.Module):
    def __init__(self, d_model, d_ff):
        super().__init__()
        self.fc1 = nn.Linear(d_model, d_ff)
        self.fc2 = nn.Linear(d_ff, d_model)
        self.layer_norm = nn.LayerNorm(d_model)

    def _pack(self, dt):
        f = torch.float32
        return dict(w1=lin_w(self.fc1, f), b1=lin_b(self.fc1), w2=lin_w(self.fc2, f), b2=lin_b(self.fc2),
                    g=self.layer_norm.weight.detach().float().contiguous(),
                    beta=self.layer_norm.bias.detach().float().contiguous())

    def forward(self, x):
        p = get_packed(self, torch.float32, self._pack)
        x = x.contiguous()
        h = ops.gemm(x, p["w1"], p["b1"], act="relu")
        o = ops.gemm(h, p["w2"], p["b2"], residual=x)
        return ops.layernorm(o, p["g"], p["beta"], self.layer_norm.eps, out=o)


class EncoderLayer(nn.Module):
    def __init__(self, d_model, d_ff, d_k, d_v, n_heads):
        super().__init__()
        self.self_attn = MultiHeadAttention(d_model, d_k, d_v, n_heads)
        self.ffn = PoswiseFeedForwardNet(d_model, d_ff)

    def forward(self, x):
        return self.ffn(self.self_attn(x, x, x))


class Encoder(nn.Module):
    def __init__(self, d_model, d_ff, d_k, d_v, n_layers, n_heads):
        super().__init__()
        self.layers = nn.ModuleList([EncoderLayer(d_model, d_ff, d_k, d_v, n_heads) for _ in range(n_layers)])

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
        return x


class DecoderLayer(nn.Module):
    def __init__(self, d_model, d_ff, d_k, d_v, n_heads):
        super().__init__()
        self.self_attn = MultiHeadAttention(d_model, d_k, d_v, n_heads)
        self.cross_attn = MultiHeadAttention(d_model, d_k, d_v, n_heads)
        self.ffn = PoswiseFeedForwardNet(d_model, d_ff)

    def forward(self, dec, enc):
        d = self.self_attn(dec, dec, dec)
        d = self.cross_attn(d, enc, enc)
        return self.ffn(d)


class Transformer2_3_1(nn.Module):
    def __init__(self, d_model, d_ff, d_k, d_v, n_layers, n_heads, len_q):
        super().__init__()
        self.d_model, self.len_q = d_model, len_q
        self.encoder = Encoder(d_model, d_ff, d_k, d_v, n_layers, n_heads)
        self.decoder = DecoderLayer(d_model, d_ff, d_k, d_v, n_heads)
        self.register_buffer("pos_table", sinusoid_table(len_q, d_model), persistent=False)

    def forward_encoded(self, enc_with_pos, dec_inputs):
        """enc_with_pos already carries the position table (fused into the window-unfold kernel)."""
        enc = self.encoder(enc_with_pos)
        return self.decoder(dec_inputs.float().contiguous(), enc)

    def forward(self, enc_inputs, dec_inputs):
        """enc_inputs [T, len_q, d_model], dec_inputs [T, 1, d_model] -> [T, 1, d_model]."""
        enc = ops.add_bcast(enc_inputs.float(), self.pos_table)
        return self.forward_encoded(enc, dec_inputs)
