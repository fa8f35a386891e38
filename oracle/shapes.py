"""State-dict key/shape tables restated from the reference constructors (oracle).

These let the oracle build parameter dicts without instantiating any nn.Module
(neither the reference's nor the build's); tests check them against the key lists
recorded from the reference (tests/golden/reference_golden.npz) and against the
build's modules.
"""
from .mit_evp import CONFIGS, SR_RATIOS, SCALE_FACTOR


def _lin(d, p, o, i, bias=True):
    d[p + ".weight"] = (o, i)
    if bias:
        d[p + ".bias"] = (o,)


def _ln(d, p, c):
    d[p + ".weight"] = (c,)
    d[p + ".bias"] = (c,)


def _bn(d, p, c):
    _ln(d, p, c)
    d[p + ".running_mean"] = (c,)
    d[p + ".running_var"] = (c,)
    d[p + ".num_batches_tracked"] = ()


def _conv(d, p, o, i, k, bias=True):
    d[p + ".weight"] = (o, i, k, k)
    if bias:
        d[p + ".bias"] = (o,)


def mit_evp_shapes(variant="mit_b2_evp"):
    """MixVisionTransformerEVP.__init__ (mix_transformer_evp.py:219-298) for one mit_b*_evp variant."""
    cfg = CONFIGS[variant]
    dims, depths = cfg["embed_dims"], cfg["depths"]
    d = {}
    cin = 3
    for s in range(4):                                     # patch_embed1..4 (:228-235)
        k = 7 if s == 0 else 3
        _conv(d, f"patch_embed{s + 1}.proj", dims[s], cin, k)
        _ln(d, f"patch_embed{s + 1}.norm", dims[s])
        cin = dims[s]
    for s in range(4):                                     # block1..4 + norm1..4 (:240-269)
        C, sr = dims[s], SR_RATIOS[s]
        for i in range(depths[s]):
            p = f"block{s + 1}.{i}"
            _ln(d, p + ".norm1", C)
            _lin(d, p + ".attn.q", C, C)
            _lin(d, p + ".attn.kv", 2 * C, C)
            _lin(d, p + ".attn.proj", C, C)
            if sr > 1:
                _conv(d, p + ".attn.sr", C, C, sr)
                _ln(d, p + ".attn.norm", C)
            _ln(d, p + ".norm2", C)
            _lin(d, p + ".mlp.fc1", 4 * C, C)
            d[p + ".mlp.dwconv.dwconv.weight"] = (4 * C, 1, 3, 3)
            d[p + ".mlp.dwconv.dwconv.bias"] = (4 * C,)
            _lin(d, p + ".mlp.fc2", C, 4 * C)
        _ln(d, f"norm{s + 1}", C)
    E = 2048                                               # SegFormerHead (segformer_head.py:50-106)
    for i, c in zip((4, 3, 2, 1), (dims[3], dims[2], dims[1], dims[0])):
        _lin(d, f"head.linear_c{i}.proj", E, c)
    d["head.linear_fuse.conv.weight"] = (E, 4 * E, 1, 1)
    _bn(d, "head.linear_fuse.bn", E)
    for p in ("head.fc", "head.fc_ant"):
        _lin(d, p + ".0", 512, E)
        _lin(d, p + ".2", 7, 512)
    pg = "prompt_generator"                                # PromptGenerator (:550-698)
    cin = 3
    for s in range(4):
        k = 7 if s == 0 else 3
        co = dims[s] // SCALE_FACTOR
        _conv(d, f"{pg}.handcrafted_generator{s + 1}.proj", co, cin, k)
        _ln(d, f"{pg}.handcrafted_generator{s + 1}.norm", co)
        cin = co
    for s in range(4):
        _lin(d, f"{pg}.embedding_generator{s + 1}", dims[s] // SCALE_FACTOR, dims[s])
    for s in range(4):
        c4 = dims[s] // SCALE_FACTOR
        for i in range(depths[s]):
            _lin(d, f"{pg}.lightweight_mlp{s + 1}_{i}.0", c4, c4)
        _lin(d, f"{pg}.shared_mlp{s + 1}", dims[s], c4)
    fe = "flow_encoder"                                    # OpticalFlowEncoder (:818-836)
    for i, (o, ci, k) in enumerate(((64, 2, 7), (128, 64, 3), (dims[2], 128, 3), (dims[3], dims[2], 3))):
        _conv(d, f"{fe}.conv{i + 1}", o, ci, k)
        _bn(d, f"{fe}.bn{i + 1}", o)
    for s, C in (("cross_attn_s3", dims[2]), ("cross_attn_s4", dims[3])):   # (:862-876)
        d[f"{s}.cross_attn.in_proj_weight"] = (3 * C, C)
        d[f"{s}.cross_attn.in_proj_bias"] = (3 * C,)
        _lin(d, f"{s}.cross_attn.out_proj", C, C)
        _ln(d, f"{s}.norm", C)
    return d


def mstcn_shapes(stages, layers, f_maps, f_dim, out_features):
    """MultiStageModel_S.__init__ (mstcn.py:95-120) / SingleStageModel / DilatedResidualLayer."""
    d = {}

    def single(p, dim):
        d[p + ".conv_1x1.weight"] = (f_maps, dim, 1)
        d[p + ".conv_1x1.bias"] = (f_maps,)
        for l in range(layers):
            d[f"{p}.layers.{l}.conv_dilated.weight"] = (f_maps, f_maps, 3)
            d[f"{p}.layers.{l}.conv_dilated.bias"] = (f_maps,)
            d[f"{p}.layers.{l}.conv_1x1.weight"] = (f_maps, f_maps, 1)
            d[f"{p}.layers.{l}.conv_1x1.bias"] = (f_maps,)
        d[p + ".conv_out_classes.weight"] = (out_features, f_maps, 1)
        d[p + ".conv_out_classes.bias"] = (out_features,)

    single("stage1_phase", f_dim)
    for s in range(stages - 1):
        single(f"stages.{s}", out_features)
    return d


def transformer_shapes(f_maps, f_dim, out_features, n_layers=1, n_heads=4):
    """adapter_transformer.Transformer (adapter_transformer.py:291-327) + the build's Transformer2_3_1."""
    dk = min(64, f_maps)
    D = out_features
    d = {"fc.weight": (out_features, f_dim)}

    def mha(p):
        _lin(d, p + ".W_Q", n_heads * dk, D)
        _lin(d, p + ".W_K", n_heads * dk, D)
        _lin(d, p + ".W_V", n_heads * dk, D)
        _lin(d, p + ".fc", D, n_heads * dk)
        _ln(d, p + ".layer_norm", D)

    def ffn(p):
        _lin(d, p + ".fc1", f_maps, D)
        _lin(d, p + ".fc2", D, f_maps)
        _ln(d, p + ".layer_norm", D)

    for l in range(n_layers):
        mha(f"transformer.encoder.layers.{l}.self_attn")
        ffn(f"transformer.encoder.layers.{l}.ffn")
    mha("transformer.decoder.self_attn")
    mha("transformer.decoder.cross_attn")
    ffn("transformer.decoder.ffn")
    return d
