"""CPU emulation of where the 16-bit path loses precision on mit_b3 (VERDICT r04 "next" #2).

Runs the oracle's functional forward in float64 with F.linear / F.conv2d replaced by "fp16 in, exact
accumulate, fp16 out" (torch.autocast's rounding points for those ops), then compares the logits with the
float64 forward, in variants:
  autocast   residual stream and LayerNorm in full precision (what torch.autocast(float16) does:
             LayerNorm outputs f32, x + attn(...) promotes to f32 — mix_transformer_evp.py:167-171)
  res16      additionally the residual stream rounded to fp16 after every add (the round-4 16-bit path)
  res16_s12  res16 in stages 1-2 only, full-precision residual in stages 3-4
  head_only / backbone_only   autocast rounding in the SegFormer head only / everywhere but the head

    python tools/precision_emulation.py [B]
"""
import os
import sys
import types

import torch
import torch.nn.functional as TF

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
from oracle import inputs as I, params as P, mit_evp as M, shapes as SH  # noqa: E402

r16 = lambda t: t.to(torch.float16).to(t.dtype)


class _F(types.SimpleNamespace):
    def __getattr__(self, k):
        return getattr(TF, k)


def linear16(x, w, b=None):
    y = TF.linear(r16(x), r16(w), None if b is None else b)
    return r16(y)


def conv16(x, w, b=None, **kw):
    y = TF.conv2d(r16(x), r16(w), b, **kw)
    return r16(y)


def run(x, y, fl, sd, variant, mode):
    orig_block, orig_prompt = M.block, M.get_prompt
    orig_head = M.segformer_head
    if mode != "f64":
        M.F = _F(linear=linear16, conv2d=conv16)
    if mode == "head_only":             # only the SegFormer head's GEMMs in fp16
        M.F = TF

        def head(*a, **k):
            M.F = _F(linear=linear16, conv2d=conv16)
            try:
                return orig_head(*a, **k)
            finally:
                M.F = TF
        M.segformer_head = head
    if mode == "backbone_only":         # everything but the head in fp16
        def head(*a, **k):
            M.F = TF
            return orig_head(*a, **k)
        M.segformer_head = head
    if mode.startswith("res16"):
        def block(x, H, W, sd, p, nh, sr):
            s = int(p[5])
            rr = r16 if (mode == "res16" or s <= 2) else (lambda t: t)
            x = rr(x + M.attention(M._ln(x, sd, p + ".norm1", M.BLOCK_EPS), H, W, sd, p + ".attn", nh, sr))
            return rr(x + M.mlp(M._ln(x, sd, p + ".norm2", M.BLOCK_EPS), H, W, sd, p + ".mlp"))

        def get_prompt(x, hc, emb, sd, s, i):
            rr = r16 if (mode == "res16" or s <= 2) else (lambda t: t)
            return rr(orig_prompt(x, hc, emb, sd, s, i))
        M.block, M.get_prompt = block, get_prompt
    try:
        with torch.no_grad():
            feat = M.forward(x, y, sd, variant, fl, return_features=True, dtype=torch.float64)
            f = TF
            yl = f.linear(f.relu(f.linear(feat, sd["head.fc.0.weight"].double(), sd["head.fc.0.bias"].double())),
                          sd["head.fc.2.weight"].double(), sd["head.fc.2.bias"].double())
    finally:
        M.F, M.block, M.get_prompt, M.segformer_head = TF, orig_block, orig_prompt, orig_head
    return feat, yl


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.set_num_threads(os.cpu_count())
    variant = "mit_b3_evp"
    sd = P.make_state_dict(SH.mit_evp_shapes(variant), 3)
    x, y, fl = I.frames(B, 23), I.segmaps(B, 23), I.flow(B, 23)
    ref_f, ref_l = run(x, y, fl, sd, variant, "f64")
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["autocast", "res16", "res16_s12", "head_only", "backbone_only"]
    for mode in modes:
        f, l = run(x, y, fl, sd, variant, mode)
        print(f"{mode:10s} B={B}: feat max|d| {(f - ref_f).abs().max():.3e}  logits max|d| {(l - ref_l).abs().max():.3e}"
              f"  logits rms {(l - ref_l).pow(2).mean().sqrt():.3e}", flush=True)


if __name__ == "__main__":
    main()
