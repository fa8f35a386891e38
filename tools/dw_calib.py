"""FETCH_SIZE / WRITE_SIZE calibration and timing for the depthwise conv: the stage-3
(B = 256, 14 x 14, 1280 channels) and stage-4 (7 x 7, 2048 channels) f16 maps through dwconv3x3_strip, next
to a known-byte stream of the same map (torch's copy_: read 1 map + write 1 map).  Run under
`rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes); per-kernel averages give bytes per
launch to compare with the algorithmic 2 maps.  SVK_DW_XCD=0/1 selects the dispatch-order / XCD-grouped
block order (read once per process).
GPU box: python tools/dw_calib.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))
from svk import ops  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    for B, W, K in ((256, 14, 1280), (256, 7, 2048)):
        h = torch.randn(B, W, W, K, device=dev).half()
        taps = torch.randn(9, K, device=dev) * 0.3
        db = torch.randn(K, device=dev) * 0.1
        out = torch.empty_like(h)
        for _ in range(2):
            ops.dwconv3x3(h, taps, db, act="gelu")
            out.copy_(h)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        for _ in range(iters):
            ops.dwconv3x3(h, taps, db, act="gelu")
        ev[1].record()
        for _ in range(iters):
            out.copy_(h)
        ev[2].record()
        torch.cuda.synchronize()
        nb = h.numel() * 2
        tdw = ev[0].elapsed_time(ev[1]) * 1e3 / iters
        tcp = ev[1].elapsed_time(ev[2]) * 1e3 / iters
        print(f"xcd={os.environ.get('SVK_DW_XCD', '1')} map {B}x{W}x{W}x{K}: {nb / 1e6:.1f} MB; dwconv {tdw:.1f} us "
              f"({2 * nb / tdw / 1e6:.2f} TB/s algorithmic); copy {tcp:.1f} us ({2 * nb / tcp / 1e6:.2f} TB/s)",
              flush=True)


if __name__ == "__main__":
    main()
