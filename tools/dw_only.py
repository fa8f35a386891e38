"""Run only the stage-1 depthwise conv (B = 256, 56 x 56 x 256, GELU) a few times (PMC target)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402

dev = torch.device("cuda:0")
H, C = int(os.environ.get("H", "56")), int(os.environ.get("C", "256"))
x = torch.randn(256, H, H, C, device=dev).to(torch.bfloat16)
taps = torch.randn(9, C, device=dev)
bias = torch.randn(C, device=dev)
for _ in range(4):
    ops.dwconv3x3(x, taps, bias, act="gelu")
torch.cuda.synchronize()
print("ok")
