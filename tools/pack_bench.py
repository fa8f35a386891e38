"""Input-packing kernels at the extraction batch (B = 256, 224 x 224): NCHW f32 -> NHWC f16 (8 channels) for
frames (C = 3) and flow (C = 2), and the reflect-padded 5x5 Gaussian (C = 3)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pk_cfg_sweep import timeit  # noqa: E402
from svk import ops  # noqa: E402

dev = torch.device("cuda:0")
x3 = torch.randn(256, 3, 224, 224, device=dev)
x2 = torch.randn(256, 2, 224, 224, device=dev)
for name, fn, nbytes in (("nchw C=3", lambda: ops.nchw_to_nhwc(x3, torch.float16, cpad=8), x3.numel() * 4 + 256 * 224 * 224 * 16),
                         ("nchw C=2", lambda: ops.nchw_to_nhwc(x2, torch.float16, cpad=8), x2.numel() * 4 + 256 * 224 * 224 * 16),
                         ("gauss C=3", lambda: ops.gauss5x5_reflect(x3, torch.float16, cpad=8), x3.numel() * 4 + 256 * 224 * 224 * 16)):
    ms = timeit(fn, 20)
    print(f"{name:10s} {ms * 1e3:7.1f} us  {nbytes / ms / 1e9:6.0f} GB/s (GR={os.environ.get('SVK_GAUSS_GR', '8')})", flush=True)
