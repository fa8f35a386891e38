"""Functional CPU restatement of adapter_transformer.Transformer.original_forward (oracle).

Pinned part: the 30-frame causal window construction with zero left-padding and
``feas = tanh(fc(long_feature)).transpose(0, 1)`` (adapter_transformer.py:329-347).

Unpinned part: ``Transformer2_3_1`` — its source (transformer2_3_1.py) is absent from
the reference snapshot (imported at adapter_transformer.py:14, trans_SV_output.py:12).
The build defines it behind the call-site contract (ctor args at
adapter_transformer.py:317-325; ``forward(enc_inputs [T,len_q,d_model],
dec_inputs [T,1,d_model]) -> [T,1,d_model]``, trans_SV_output.py:291-296) as a
post-LN encoder (self-attention over the window + ReLU FFN, ``n_layers`` deep) and a
one-layer decoder whose single query token (the spatial embedding ``feas``)
self-attends, then cross-attends to the encoded window, then goes through a FFN.
A fixed sinusoidal position table over the ``len_q`` window slots is added to the
encoder input.  This module restates *that* design; parity is **unpinned**.
"""
import math

import torch
import torch.nn.functional as F


def window_unfold(x, len_q):
    """The per-frame loop of adapter_transformer.py:336-343 as pad + unfold:
    x [1, C, T] -> inputs [T, len_q, C]; row t = frames t-len_q+1 .. t, zero left-padded."""
    feats = x.transpose(1, 2)[0]                          # [T, C]
    T, C = feats.shape
    padded = torch.cat([feats.new_zeros(len_q - 1, C), feats], dim=0)
    return padded.unfold(0, len_q, 1).transpose(1, 2).contiguous()   # [T, len_q, C]


def sinusoid_table(n, d):
    pos = torch.arange(n, dtype=torch.float64)[:, None]
    i = torch.arange(d, dtype=torch.float64)[None, :]
    ang = pos / torch.pow(10000.0, 2 * torch.div(i, 2, rounding_mode="floor") / d)
    tab = torch.where(i % 2 == 0, torch.sin(ang), torch.cos(ang))
    return tab.float()


def mha(q_in, kv_in, sd, p, n_heads, d_k, d_v):
    """MultiHeadAttention: W_Q/W_K/W_V (bias) -> per-head softmax(QK^T/sqrt(d_k)) V -> fc -> LN(out + q_in)."""
    Bt, Lq, D = q_in.shape
    Lk = kv_in.shape[1]
    q = F.linear(q_in, sd[p + ".W_Q.weight"], sd[p + ".W_Q.bias"]).reshape(Bt, Lq, n_heads, d_k).transpose(1, 2)
    k = F.linear(kv_in, sd[p + ".W_K.weight"], sd[p + ".W_K.bias"]).reshape(Bt, Lk, n_heads, d_k).transpose(1, 2)
    v = F.linear(kv_in, sd[p + ".W_V.weight"], sd[p + ".W_V.bias"]).reshape(Bt, Lk, n_heads, d_v).transpose(1, 2)
    a = ((q @ k.transpose(-1, -2)) / math.sqrt(d_k)).softmax(-1)
    o = (a @ v).transpose(1, 2).reshape(Bt, Lq, n_heads * d_v)
    o = F.linear(o, sd[p + ".fc.weight"], sd[p + ".fc.bias"])
    return F.layer_norm(o + q_in, (D,), sd[p + ".layer_norm.weight"], sd[p + ".layer_norm.bias"], 1e-5)


def ffn(x, sd, p):
    h = F.relu(F.linear(x, sd[p + ".fc1.weight"], sd[p + ".fc1.bias"]))
    o = F.linear(h, sd[p + ".fc2.weight"], sd[p + ".fc2.bias"])
    return F.layer_norm(o + x, (x.shape[-1],), sd[p + ".layer_norm.weight"], sd[p + ".layer_norm.bias"], 1e-5)


def transformer2_3_1(enc_inputs, dec_inputs, sd, p, n_layers, n_heads, d_k, d_v, len_q):
    D = enc_inputs.shape[-1]
    x = enc_inputs + sinusoid_table(len_q, D).to(enc_inputs.dtype)[None]
    for l in range(n_layers):
        x = mha(x, x, sd, f"{p}.encoder.layers.{l}.self_attn", n_heads, d_k, d_v)
        x = ffn(x, sd, f"{p}.encoder.layers.{l}.ffn")
    d = dec_inputs
    d = mha(d, d, sd, f"{p}.decoder.self_attn", n_heads, d_k, d_v)
    d = mha(d, x, sd, f"{p}.decoder.cross_attn", n_heads, d_k, d_v)
    return ffn(d, sd, f"{p}.decoder.ffn")


def original_forward(x, long_feature, sd, f_maps, len_q=30, dtype=torch.float32):
    """Transformer.original_forward (adapter_transformer.py:329-352).
    x [1, 14, T] (MS-TCN last stage), long_feature [1, T, 2048] -> [T, 1, 14]."""
    sd = {k: v.to(dtype) for k, v in sd.items()}
    x = x.to(dtype)
    long_feature = long_feature.to(dtype)
    inputs = window_unfold(x, len_q)
    feas = torch.tanh(F.linear(long_feature, sd["fc.weight"]).transpose(0, 1))
    attn_dim = min(64, f_maps)
    return transformer2_3_1(inputs, feas, sd, "transformer", 1, 4, attn_dim, attn_dim, len_q)
