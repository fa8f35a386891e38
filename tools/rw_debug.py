"""mixffn_rw vs mixffn_fused at growing batch / forced grid sizes (debugging)."""
import os
import sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402

dev = torch.device("cuda:0")
C, W = 64, 56
g = torch.Generator().manual_seed(0)
r = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc)
w1 = r(4 * C, C, sc=C ** -0.5).half().to(dev); b1 = r(4 * C, sc=0.1).to(dev)
taps = r(9, 4 * C, sc=0.3).to(dev); db = r(4 * C, sc=0.1).to(dev)
w2 = r(C, 4 * C, sc=(4 * C) ** -0.5).half().to(dev); b2 = r(C, sc=0.1).to(dev)
tpk = ops.mixffn_pack_taps(taps, db, torch.float16)
for B, H in [tuple(map(int, a.split("x"))) for a in sys.argv[1:]]:
    xn = r(B, H, W, C).half().to(dev); x = r(B, H, W, C).half().to(dev)
    got = ops.mixffn_rw(xn, x, w1, b1, taps, db, w2, b2)
    torch.cuda.synchronize()
    ref = ops.mixffn_fused(xn, x, w1, b1, tpk, w2, b2)
    torch.cuda.synchronize()
    d = (got.float() - ref.float()).abs().max().item()
    print(f"B={B} H={H} grid={os.environ.get('SVK_RW_GRID', 'auto')}: max |rw - fused| = {d:.3e}", flush=True)
