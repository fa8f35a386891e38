"""Debug helper: bf16 MiT-b2 features at batch B under the current env knobs vs the oracle.
Usage (GPU box): B=8 SVK_NO_PK=1 python tools/dbg_b8.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd"))
import torch  # noqa: E402

from oracle import inputs as I, params as P, mit_evp as M, shapes as SH  # noqa: E402
from models import mix_transformer_evp as mte  # noqa: E402

B = int(os.environ.get("B", "8"))
dev = torch.device("cuda:0")
m = mte.mit_b2_evp()
m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0))
m.svk_dtype = torch.bfloat16
m = m.to(dev).eval()
x, y, fl = I.frames(B, 3), I.segmaps(B, 3), I.flow(B, 3)
with torch.no_grad():
    f = m(x.to(dev), y.to(dev), fl.to(dev), return_features=True)
    outs = m.forward_features(x.to(dev), y.to(dev))
    f3, f4 = m.flow_encoder(fl.to(dev))
torch.cuda.synchronize()
sd = P.make_state_dict(SH.mit_evp_shapes("mit_b2_evp"), 0)
with torch.no_grad():
    ref = M.forward(x, y, sd, "mit_b2_evp", fl, return_features=True)
err = (f.float().cpu() - ref).abs()
env = {k: v for k, v in os.environ.items() if k.startswith("SVK")}
print(f"env {env} B {B} feat max err {float(err.max()):.4g} nan {bool(torch.isnan(f).any())} "
      f"zero frac {float((f == 0).float().mean()):.3f}", flush=True)
for i, o in enumerate(outs):
    o = o.float()
    print(f"  stage {i + 1} nan {bool(torch.isnan(o).any())} absmax {float(o.abs().max()):.4g}", flush=True)
for nm, t in (("flow s3", f3), ("flow s4", f4)):
    print(f"  {nm} nan {bool(torch.isnan(t.float()).any())} absmax {float(t.float().abs().max()):.4g}", flush=True)
