"""Functional CPU restatement of MixVisionTransformerEVP + SegFormerHead (oracle).

Every function cites the reference lines it restates (paths relative to the
reference checkout).  Works on a plain ``{name: tensor}`` state dict whose keys are
exactly the reference module's ``state_dict()`` keys, in eval mode (dropout,
Dropout2d and DropPath are identities; BatchNorm uses running statistics).
Arithmetic follows the reference op order; ``dtype`` may be float64 for a
higher-precision check.
"""
import torch
import torch.nn.functional as F

# mix_transformer_evp.py:893-944 — the mit_b*_evp family differs only in dims / depths.
CONFIGS = {
    "mit_b0_evp": dict(embed_dims=(32, 64, 160, 256), depths=(2, 2, 2, 2)),
    "mit_b1_evp": dict(embed_dims=(64, 128, 320, 512), depths=(2, 2, 2, 2)),
    "mit_b2_evp": dict(embed_dims=(64, 128, 320, 512), depths=(3, 4, 6, 3)),
    "mit_b3_evp": dict(embed_dims=(64, 128, 320, 512), depths=(3, 4, 18, 3)),
    "mit_b4_evp": dict(embed_dims=(64, 128, 320, 512), depths=(3, 8, 27, 3)),
    "mit_b5_evp": dict(embed_dims=(64, 128, 320, 512), depths=(3, 6, 40, 3)),
}
NUM_HEADS = (1, 2, 5, 8)      # mix_transformer_evp.py:897-943
SR_RATIOS = (8, 4, 2, 1)
BLOCK_EPS = 1e-6              # norm_layer=partial(nn.LayerNorm, eps=1e-6) (:898)
DEFAULT_EPS = 1e-5            # plain nn.LayerNorm: patch-embed (:190), sr norm (:90), cross-attn (:876)
SCALE_FACTOR = 4              # PromptGenerator scale_factor (:278)


def _ln(x, sd, p, eps):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


def _lin(x, sd, p, bias=True):
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias") if bias else None)


def overlap_patch_embed(x, sd, p, stride):
    """OverlapPatchEmbed.forward (mix_transformer_evp.py:209-215): conv(k, s, k//2) -> tokens -> LN."""
    w = sd[p + ".proj.weight"]
    k = w.shape[-1]
    x = F.conv2d(x, w, sd[p + ".proj.bias"], stride=stride, padding=k // 2)
    _, _, H, W = x.shape
    x = x.flatten(2).transpose(1, 2)
    return _ln(x, sd, p + ".norm", DEFAULT_EPS), H, W


def attention(x, H, W, sd, p, num_heads, sr):
    """Attention.forward (mix_transformer_evp.py:110-131): efficient self-attention with sequence reduction."""
    B, N, C = x.shape
    hd = C // num_heads
    q = _lin(x, sd, p + ".q").reshape(B, N, num_heads, hd).permute(0, 2, 1, 3)
    if sr > 1:
        x_ = x.permute(0, 2, 1).reshape(B, C, H, W)
        x_ = F.conv2d(x_, sd[p + ".sr.weight"], sd[p + ".sr.bias"], stride=sr).reshape(B, C, -1).permute(0, 2, 1)
        x_ = _ln(x_, sd, p + ".norm", DEFAULT_EPS)
    else:
        x_ = x
    kv = _lin(x_, sd, p + ".kv").reshape(B, -1, 2, num_heads, hd).permute(2, 0, 3, 1, 4)
    k, v = kv[0], kv[1]
    attn = (q @ k.transpose(-2, -1)) * (hd ** -0.5)
    attn = attn.softmax(dim=-1)
    x = (attn @ v).transpose(1, 2).reshape(B, N, C)
    return _lin(x, sd, p + ".proj")


def mlp(x, H, W, sd, p):
    """Mlp.forward + DWConv.forward (mix_transformer_evp.py:60-67, 24-30): MixFFN."""
    x = _lin(x, sd, p + ".fc1")
    B, N, C = x.shape
    x = x.transpose(1, 2).reshape(B, C, H, W)
    x = F.conv2d(x, sd[p + ".dwconv.dwconv.weight"], sd[p + ".dwconv.dwconv.bias"], padding=1, groups=C)
    x = x.flatten(2).transpose(1, 2)
    x = F.gelu(x)
    return _lin(x, sd, p + ".fc2")


def block(x, H, W, sd, p, num_heads, sr):
    """Block.forward (mix_transformer_evp.py:167-171)."""
    x = x + attention(_ln(x, sd, p + ".norm1", BLOCK_EPS), H, W, sd, p + ".attn", num_heads, sr)
    x = x + mlp(_ln(x, sd, p + ".norm2", BLOCK_EPS), H, W, sd, p + ".mlp")
    return x


def gaussian_filter(img):
    """GaussianFilter.conv_gauss (mix_transformer_evp.py:500-514): reflect pad 2, depthwise binomial 5x5 /256."""
    k = torch.tensor([[1., 4., 6., 4., 1], [4., 16., 24., 16., 4.], [6., 24., 36., 24., 6.],
                      [4., 16., 24., 16., 4.], [1., 4., 6., 4., 1.]], dtype=img.dtype) / 256.
    k = k.repeat(img.shape[1], 1, 1, 1)
    img = F.pad(img, (2, 2, 2, 2), mode="reflect")
    return F.conv2d(img, k, groups=img.shape[1])


def init_prompts(y, sd):
    """PromptGenerator.init_prompts, input_type 'gaussian' (mix_transformer_evp.py:718-747)."""
    x = gaussian_filter(y)
    B = x.shape[0]
    feats = []
    prev = x
    for s, stride in zip((1, 2, 3, 4), (4, 2, 2, 2)):
        f, H, W = overlap_patch_embed(prev, sd, f"prompt_generator.handcrafted_generator{s}", stride)
        feats.append(f)
        prev = f.reshape(B, H, W, -1).permute(0, 3, 1, 2).contiguous()
    return feats


def get_prompt(x, hc, emb, sd, s, i):
    """PromptGenerator.get_prompt, adaptor 'adaptor' (mix_transformer_evp.py:776-815)."""
    feat = hc + emb
    feat = F.gelu(_lin(feat, sd, f"prompt_generator.lightweight_mlp{s}_{i}.0"))
    feat = _lin(feat, sd, f"prompt_generator.shared_mlp{s}")
    return x + feat


def forward_features(x, y, sd, depths):
    """MixVisionTransformerEVP.forward_features (mix_transformer_evp.py:352-416); returns NHWC-token
    stage outputs (the reference's NCHW ``outs`` are exactly these re-laid)."""
    x = x.reshape(-1, 3, 224, 224)
    y = y.reshape(-1, 3, 224, 224)
    B = x.shape[0]
    hcs = init_prompts(y, sd)
    outs = []
    for s in range(4):
        stride = 4 if s == 0 else 2
        x, H, W = overlap_patch_embed(x, sd, f"patch_embed{s + 1}", stride)
        emb = _lin(x, sd, f"prompt_generator.embedding_generator{s + 1}")    # init_prompt (:749-756)
        for i in range(depths[s]):
            x = get_prompt(x, hcs[s], emb, sd, s + 1, i)
            x = block(x, H, W, sd, f"block{s + 1}.{i}", NUM_HEADS[s], SR_RATIOS[s])
        x = _ln(x, sd, f"norm{s + 1}", BLOCK_EPS)
        outs.append((x, H, W))
        x = x.reshape(B, H, W, -1).permute(0, 3, 1, 2).contiguous()
    return outs


def _bn_eval(x, sd, p, eps=1e-5):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        False, 0.0, eps)


def flow_encoder(flow, sd):
    """OpticalFlowEncoder.forward (mix_transformer_evp.py:838-859), BN in eval mode."""
    if flow.dim() == 5:
        B, T, C, H, W = flow.shape
        flow = flow.reshape(B * T, C, H, W)
    x = flow
    feats = []
    for i, stride, pad in ((1, 4, 3), (2, 2, 1), (3, 2, 1), (4, 2, 1)):
        x = F.conv2d(x, sd[f"flow_encoder.conv{i}.weight"], sd[f"flow_encoder.conv{i}.bias"], stride=stride, padding=pad)
        x = F.relu(_bn_eval(x, sd, f"flow_encoder.bn{i}"))
        feats.append(x)
    return feats[2].flatten(2).transpose(1, 2), feats[3].flatten(2).transpose(1, 2)


def cross_attention(xv, xf, sd, p, num_heads=8):
    """MotionGuidedCrossAttention.forward (mix_transformer_evp.py:878-890) with nn.MultiheadAttention
    (batch_first, q = visual, k = v = flow) spelled out: in_proj, per-head softmax(q k^T/sqrt(hd)) v, out_proj."""
    B, Nq, E = xv.shape
    Nk = xf.shape[1]
    hd = E // num_heads
    w = sd[p + ".cross_attn.in_proj_weight"]
    b = sd[p + ".cross_attn.in_proj_bias"]
    q = F.linear(xv, w[:E], b[:E]).reshape(B, Nq, num_heads, hd).transpose(1, 2)
    k = F.linear(xf, w[E:2 * E], b[E:2 * E]).reshape(B, Nk, num_heads, hd).transpose(1, 2)
    v = F.linear(xf, w[2 * E:], b[2 * E:]).reshape(B, Nk, num_heads, hd).transpose(1, 2)
    a = ((q * (hd ** -0.5)) @ k.transpose(-2, -1)).softmax(-1)
    o = (a @ v).transpose(1, 2).reshape(B, Nq, E)
    o = F.linear(o, sd[p + ".cross_attn.out_proj.weight"], sd[p + ".cross_attn.out_proj.bias"])
    return _ln(xv + o, sd, p + ".norm", DEFAULT_EPS)


def _resize_nhwc(t, H, W, size=7):
    """resize(..., mode='bilinear', align_corners=False) of a token map (segformer_head.py:150-156)."""
    B, N, C = t.shape
    nchw = t.transpose(1, 2).reshape(B, C, H, W)
    if H != size:
        nchw = F.interpolate(nchw, (size, size), None, "bilinear", False)
    return nchw


def segformer_head(outs, sd, return_features):
    """SegFormerHead.forward (segformer_head.py:137-179), eval mode, in the reference op order
    (per-token Linear C_i->2048, resize to the c4 grid, concat [c4,c3,c2,c1], 1x1 conv, BN, ReLU, avg-pool)."""
    (c1, H1, W1), (c2, H2, W2), (c3, H3, W3), (c4, H4, W4) = outs
    maps = []
    for t, H, W, name in ((c4, H4, W4, "linear_c4"), (c3, H3, W3, "linear_c3"),
                          (c2, H2, W2, "linear_c2"), (c1, H1, W1, "linear_c1")):
        e = _lin(t, sd, f"head.{name}.proj")                  # MLP.forward (:40-43)
        maps.append(_resize_nhwc(e, H, W, H4))
    c = torch.cat(maps, dim=1)
    c = F.conv2d(c, sd["head.linear_fuse.conv.weight"])      # ConvModule: conv(bias=False) -> BN -> ReLU
    c = F.relu(_bn_eval(c, sd, "head.linear_fuse.bn"))
    x = c.mean(dim=(2, 3))                                    # AdaptiveAvgPool2d((1,1)) + flatten (:167-169)
    if return_features:
        return x
    y = F.linear(F.relu(_lin(x, sd, "head.fc.0")), sd["head.fc.2.weight"], sd["head.fc.2.bias"])
    y_ant = F.linear(F.relu(_lin(x, sd, "head.fc_ant.0")), sd["head.fc_ant.2.weight"], sd["head.fc_ant.2.bias"])
    return y, y_ant


def forward(x, y, sd, variant="mit_b2_evp", flow=None, return_features=False, dtype=torch.float32):
    """MixVisionTransformerEVP.forward (mix_transformer_evp.py:418-449)."""
    sd = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in sd.items()}
    x = x.to(dtype)
    y = y.to(dtype)
    depths = CONFIGS[variant]["depths"]
    outs = forward_features(x, y, sd, depths)
    if flow is not None:
        f3, f4 = flow_encoder(flow.to(dtype), sd)
        c3, H3, W3 = outs[2]
        outs[2] = (cross_attention(c3, f3, sd, "cross_attn_s3"), H3, W3)
        c4, H4, W4 = outs[3]
        outs[3] = (cross_attention(c4, f4, sd, "cross_attn_s4"), H4, W4)
    return segformer_head(outs, sd, return_features)
