import sys, torch
sys.path.insert(0, "deep-learning-for-surgical-video-analysis_amd")
from svk import ops
x = torch.randn(256, 3, 224, 224, device="cuda")
for cp in (3, 8):
    ops.gauss5x5_reflect(x, torch.float16, cpad=cp); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20): ops.gauss5x5_reflect(x, torch.float16, cpad=cp)
    e.record(); torch.cuda.synchronize()
    print("cpad", cp, s.elapsed_time(e) / 20 * 1e3, "us")
