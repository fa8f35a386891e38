"""Precision of the extraction path per compute dtype at the benched configuration (MiT-b2 + flow,
B frames, return_features and logits) against the fp32 oracle (the reference's op graph on torch CPU
ops).  Prints one JSON line per dtype: max / mean |diff| of features and logits, relative errors and
the argmax agreement rate of the phase logits.  Diagnostic tool (GPU box); the asserted bars live in
tests/test_headline_gpu.py.

Usage: python tools/precision_report.py [B] [dtypes...]"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd"))

from oracle import inputs as I, params as P, mit_evp as M, shapes as SH   # noqa: E402


def head_logits(feat, sd):
    f = torch.nn.functional
    y = f.linear(f.relu(f.linear(feat, sd["head.fc.0.weight"], sd["head.fc.0.bias"])), sd["head.fc.2.weight"],
                 sd["head.fc.2.bias"])
    ya = f.linear(f.relu(f.linear(feat, sd["head.fc_ant.0.weight"], sd["head.fc_ant.0.bias"])),
                  sd["head.fc_ant.2.weight"], sd["head.fc_ant.2.bias"])
    return y, ya


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    dts = sys.argv[2:] or ["fp32", "fp16", "bf16"]
    from models import mix_transformer_evp as mte
    dev = torch.device("cuda", 0)
    variant = "mit_b2_evp"
    sd = P.make_state_dict(SH.mit_evp_shapes(variant), 0)
    x, y, fl = I.frames(B, 21), I.segmaps(B, 21), I.flow(B, 21)
    t0 = time.time()
    with torch.no_grad():
        ref = M.forward(x, y, sd, variant, fl, return_features=True)
        rl, ra = head_logits(ref, sd)
    print(f"oracle B={B}: {time.time() - t0:.1f} s on {torch.get_num_threads()} threads", flush=True)
    m = getattr(mte, variant)()
    m.load_state_dict(sd)
    m = m.to(dev).eval()
    for name in dts:
        m.svk_dtype = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[name]
        with torch.no_grad():
            f = m(x.to(dev), y.to(dev), fl.to(dev), return_features=True).float().cpu()
            gl, ga = m(x.to(dev), y.to(dev), fl.to(dev))
        gl, ga = gl.float().cpu(), ga.float().cpu()
        df, dl, da = (f - ref).abs(), (gl - rl).abs(), (ga - ra).abs()
        rec = {"dtype": name, "B": B,
               "feat_max_abs": df.max().item(), "feat_mean_abs": df.mean().item(),
               "feat_ref_max": ref.abs().max().item(), "feat_ref_mean": ref.abs().mean().item(),
               "feat_rel_l2": ((f - ref).norm() / ref.norm()).item(),
               "logit_max_abs": dl.max().item(), "logit_ref_max": rl.abs().max().item(),
               "ant_max_abs": da.max().item(),
               "argmax_agree": (gl.argmax(1) == rl.argmax(1)).float().mean().item(),
               "ref_logit_top2_gap_min": (rl.topk(2, 1).values[:, 0] - rl.topk(2, 1).values[:, 1]).min().item()}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
