"""Train-mode restatement of the frozen-backbone training step (oracle; test infrastructure only).

Follows train_evp.py:362-515: every parameter whose name does not contain one of
``head / prompt / flow_encoder / cross_attn_s3 / cross_attn_s4`` is frozen (:379-382), the model
runs in train mode (timm DropPath with the linear drop-path rule, drop_path_rate 0.1
(mix_transformer_evp.py:238, 899-926); Dropout2d(0.1) on the fused head map
(segformer_head.py:88, 163); BatchNorm with batch statistics in the head's linear_fuse and the
flow encoder), the loss is CrossEntropyLoss(sum) + SmoothL1Loss(sum) (:390-391, 500-509), and
the optimizer is SGD(lr 5e-4, momentum 0.9, dampening 0, weight decay 1e-5, nesterov False)
(:35-41, 405-419).  GradScaler (:443, 512-515) is a numerical no-op when no overflow occurs.

The stochastic masks are explicit inputs (values 0 or 1/keep, exactly what timm's DropPath and
nn.Dropout2d multiply by), so the build's kernels and this restatement see the same draws.
Gradients come from torch autograd over the functional forward in oracle.mit_evp.
"""
import torch
import torch.nn.functional as F

from . import mit_evp as M

TRAINABLE = ("head", "prompt", "flow_encoder", "cross_attn_s3", "cross_attn_s4")   # train_evp.py:379-382
BN_BUFFERS = ("running_mean", "running_var", "num_batches_tracked")
DROP_PATH_RATE = 0.1      # mit_b*_evp (mix_transformer_evp.py:899-926)
HEAD_DROPOUT = 0.1        # SegFormerHead.dropout = nn.Dropout2d(0.1) (segformer_head.py:88)
BN_MOMENTUM = 0.1
SGD = dict(lr=5e-4, momentum=0.9, dampening=0.0, weight_decay=1e-5, nesterov=False)   # train_evp.py:35-41


def is_trainable(name):
    return any(k in name for k in TRAINABLE) and not name.endswith(BN_BUFFERS)


def drop_path_rates(variant):
    """dpr = linspace(0, drop_path_rate, sum(depths)) (mix_transformer_evp.py:238)."""
    depths = M.CONFIGS[variant]["depths"]
    dpr = torch.linspace(0, DROP_PATH_RATE, sum(depths)).tolist()
    out, cur = [], 0
    for d in depths:
        out.append(dpr[cur:cur + d])
        cur += d
    return out


def make_masks(B, variant, seed=0, enabled=True):
    """Per block two per-frame DropPath masks (attn branch, mlp branch) and the [B, 2048]
    Dropout2d channel mask; each value is 0 or 1/keep.  enabled=False gives all-ones masks."""
    g = torch.Generator().manual_seed(seed)
    blocks = []
    for rates in drop_path_rates(variant):
        st = []
        for r in rates:
            pair = []
            for _ in range(2):
                if enabled and r > 0:
                    keep = 1.0 - r
                    pair.append((torch.rand(B, generator=g) < keep).float() / keep)
                else:
                    pair.append(torch.ones(B))
            st.append(tuple(pair))
        blocks.append(st)
    if enabled:
        keep = 1.0 - HEAD_DROPOUT
        d2 = (torch.rand(B, 2048, generator=g) < keep).float() / keep
    else:
        d2 = torch.ones(B, 2048)
    return {"blocks": blocks, "dropout2d": d2}


def _bn_train(x, sd, p, stats, eps=1e-5):
    """nn.BatchNorm2d in train mode on NCHW x; records (batch mean, unbiased var) for the running update."""
    mean = x.mean(dim=(0, 2, 3))
    var = x.var(dim=(0, 2, 3), unbiased=False)
    n = x.numel() // x.shape[1]
    stats[p] = (mean.detach(), (var * n / max(n - 1, 1)).detach())
    xh = (x - mean[None, :, None, None]) / torch.sqrt(var[None, :, None, None] + eps)
    return xh * sd[p + ".weight"][None, :, None, None] + sd[p + ".bias"][None, :, None, None]


def _relu(x, site, gates, pre):
    """F.relu at a named ReLU site.  ``pre`` (a dict) records the pre-activation; ``gates`` maps a site to a
    boolean tensor of x's shape that replaces the gate (x > 0) — used to evaluate the oracle on the branch an
    f32 implementation took for elements within its rounding of the kink (ReLU is not differentiable at 0, and
    torch's relu backward takes the x > 0 side there)."""
    if pre is not None:
        pre[site] = x.detach().clone()
    if gates is not None and site in gates:
        return x * gates[site].to(device=x.device, dtype=x.dtype)
    return F.relu(x)


def _block_train(x, H, W, sd, p, heads, sr, ma, mm):
    """Block.forward with DropPath (mix_transformer_evp.py:167-171)."""
    x = x + ma[:, None, None] * M.attention(M._ln(x, sd, p + ".norm1", M.BLOCK_EPS), H, W, sd, p + ".attn", heads, sr)
    x = x + mm[:, None, None] * M.mlp(M._ln(x, sd, p + ".norm2", M.BLOCK_EPS), H, W, sd, p + ".mlp")
    return x


def forward_train(x, y, flow, sd, variant, masks, stats, gates=None, pre=None):
    """MixVisionTransformerEVP.forward in train mode -> (logits [B, 7], anticipation [B, 7]).  ReLU sites
    (``gates`` / ``pre``, see _relu): flow_encoder.bn1..4 and head.linear_fuse.bn (NCHW), head.fc.0 and
    head.fc_ant.0 ([B, 512])."""
    depths = M.CONFIGS[variant]["depths"]
    x = x.reshape(-1, 3, 224, 224)
    y = y.reshape(-1, 3, 224, 224)
    B = x.shape[0]
    hcs = M.init_prompts(y, sd)
    outs = []
    for s in range(4):
        stride = 4 if s == 0 else 2
        x, H, W = M.overlap_patch_embed(x, sd, f"patch_embed{s + 1}", stride)
        emb = M._lin(x, sd, f"prompt_generator.embedding_generator{s + 1}")
        for i in range(depths[s]):
            x = M.get_prompt(x, hcs[s], emb, sd, s + 1, i)
            ma, mm = masks["blocks"][s][i]
            x = _block_train(x, H, W, sd, f"block{s + 1}.{i}", M.NUM_HEADS[s], M.SR_RATIOS[s], ma, mm)
        x = M._ln(x, sd, f"norm{s + 1}", M.BLOCK_EPS)
        outs.append((x, H, W))
        x = x.reshape(B, H, W, -1).permute(0, 3, 1, 2).contiguous()
    # flow encoder, BN in train mode (mix_transformer_evp.py:838-859)
    f = flow.reshape(-1, 2, 224, 224)
    feats = []
    for i, st, pad in ((1, 4, 3), (2, 2, 1), (3, 2, 1), (4, 2, 1)):
        f = F.conv2d(f, sd[f"flow_encoder.conv{i}.weight"], sd[f"flow_encoder.conv{i}.bias"], stride=st, padding=pad)
        f = _relu(_bn_train(f, sd, f"flow_encoder.bn{i}", stats), f"flow_encoder.bn{i}", gates, pre)
        feats.append(f)
    f3, f4 = feats[2].flatten(2).transpose(1, 2), feats[3].flatten(2).transpose(1, 2)
    c3, H3, W3 = outs[2]
    outs[2] = (M.cross_attention(c3, f3, sd, "cross_attn_s3"), H3, W3)
    c4, H4, W4 = outs[3]
    outs[3] = (M.cross_attention(c4, f4, sd, "cross_attn_s4"), H4, W4)
    # head (segformer_head.py:137-179), reference op order, BN train + Dropout2d
    maps = []
    for (t, h, w), name in zip(reversed(outs), ("linear_c4", "linear_c3", "linear_c2", "linear_c1")):
        maps.append(M._resize_nhwc(M._lin(t, sd, f"head.{name}.proj"), h, w, H4))
    c = F.conv2d(torch.cat(maps, dim=1), sd["head.linear_fuse.conv.weight"])
    c = _relu(_bn_train(c, sd, "head.linear_fuse.bn", stats), "head.linear_fuse.bn", gates, pre)
    c = c * masks["dropout2d"].to(c.dtype)[:, :, None, None]
    feat = c.mean(dim=(2, 3))
    yl = F.linear(_relu(M._lin(feat, sd, "head.fc.0"), "head.fc.0", gates, pre), sd["head.fc.2.weight"],
                  sd["head.fc.2.bias"])
    ya = F.linear(_relu(M._lin(feat, sd, "head.fc_ant.0"), "head.fc_ant.0", gates, pre), sd["head.fc_ant.2.weight"],
                  sd["head.fc_ant.2.bias"])
    return yl, ya


def loss_and_grads(x, y, flow, labels, ant_targets, sd, variant, masks, dtype=torch.float64, gates=None, pre=None):
    """One train_model inner iteration up to backward (train_evp.py:473-512).  Returns
    (loss_phase, loss_ant, {trainable name: grad}, {bn prefix: (batch mean, unbiased var)}).  ``gates`` /
    ``pre``: ReLU gate overrides / pre-activation capture (forward_train)."""
    p = {k: (v.detach().to(dtype).clone() if v.is_floating_point() else v) for k, v in sd.items()}
    for k in p:
        if is_trainable(k) and p[k].is_floating_point():
            p[k].requires_grad_(True)
    m = {"blocks": [[(a.to(dtype), b.to(dtype)) for a, b in st] for st in masks["blocks"]],
         "dropout2d": masks["dropout2d"].to(dtype)}
    stats = {}
    yl, ya = forward_train(x.to(dtype), y.to(dtype), flow.to(dtype), p, variant, m, stats, gates, pre)
    lp = F.cross_entropy(yl, labels, reduction="sum")
    la = F.smooth_l1_loss(ya, ant_targets.to(dtype), reduction="sum")
    (lp + la).backward()
    grads = {k: v.grad.detach() for k, v in p.items() if isinstance(v, torch.Tensor) and v.requires_grad}
    return lp.detach(), la.detach(), grads, stats


def sgd_step(params, grads, bufs=None, **hp):
    """torch.optim.SGD update (train_evp.py:405-419) on {name: tensor}; returns (new params, new bufs)."""
    h = dict(SGD, **hp)
    new_p, new_b = {}, {}
    for k, w in params.items():
        d = grads[k] + h["weight_decay"] * w
        if h["momentum"]:
            b = d.clone() if bufs is None else h["momentum"] * bufs[k] + (1 - h["dampening"]) * d
            new_b[k] = b
            d = d + h["momentum"] * b if h["nesterov"] else b
        new_p[k] = w - h["lr"] * d
    return new_p, new_b
