"""Address bounds of the shipped matrix-core MixFFN back half (csrc/dwfc2.hip, ``dwrw::dwfc2_rw``), proved on the
host by enumerating the kernel's own index formulas for every tile, wave, lane and K-step (VERDICT r05 weak #9:
a diagnostic build of the pre-packing kernel faulted with an out-of-range address under ablation bits that were
never committed; this pins that the SHIPPED addressing cannot leave its operands).

Restated from dwfc2_rw (csrc/dwfc2.hip, round 5-6): the H-tile LDS-DMA source ``hsrc[j] + kt * 128`` with
``kt <= nk - 1`` (the prologue's ``min(1, nk - 1)``, ``min(2, nk - 1)`` and the loop's ``min(kt + 3, nk - 1)``),
its LDS destination, and the dwconv B-fragment LDS reads ``hoff[kk] + m * 2048`` from the slot base.  Reference
arithmetic: mix_transformer_evp.py:19-30 (DWConv) and :60-67 (Mlp), which this kernel fuses."""
import numpy as np
import pytest


class Cfg:
    """dwrw::Cfg<N, WI> (csrc/dwfc2.hip)."""

    def __init__(self, N, WI):
        self.N, self.WI, self.BK = N, WI, 64
        self.SW = 8 if WI <= 7 else (16 if WI <= 14 else 32)
        self.NMB = 8 if N == 128 else 4
        self.R = 16 * self.NMB // self.SW
        self.XROW = 1 if self.SW == WI + 1 else 0
        self.NW = 4 if N == 320 else 8
        self.MPW = 4 * self.NMB // self.NW
        self.HROWS = self.R + 2 + self.XROW
        self.HCH = self.HROWS * self.SW * 8
        self.DPW = (self.HCH + 64 * self.NW - 1) // (64 * self.NW)
        self.HBYTES = self.DPW * self.NW * 1024
        self.HSTRIDE = self.HBYTES + 1024
        self.NHB = 3
        self.GBYTES = self.NMB * 16 * 128
        self.G_OFF = self.NHB * self.HSTRIDE
        self.LDS = self.G_OFF + 2 * self.GBYTES
        self.TILES_PER_FRAME = (WI + self.R - 1) // self.R


@pytest.mark.parametrize("N,WI,K", [(320, 14, 1280), (512, 7, 2048), (128, 28, 512), (320, 14, 64)])
def test_dwfc2_mx_dma_and_lds_addresses_in_bounds(N, WI, K):
    c = Cfg(N, WI)
    B = 3                                               # the last frame's tiles are the ones at the map's end
    M = B * WI * WI
    nk = K // c.BK
    lane = np.arange(64)
    fr, fq = lane & 15, lane >> 4
    kts = sorted({0, min(1, nk - 1), min(2, nk - 1)} | {min(kt + 3, nk - 1) for kt in range(nk - 1)})
    assert max(kts) <= nk - 1
    for tile in range(B * c.TILES_PER_FRAME):
        frame, y0 = tile // c.TILES_PER_FRAME, (tile % c.TILES_PER_FRAME) * c.R
        fbase = frame * WI * WI
        for wave in range(c.NW):
            for j in range(c.DPW):
                q = (wave + c.NW * j) * 64 + lane
                L = q >> 3
                i, sl, ch = L // c.SW, L % c.SW, (q & 7) ^ (L & 7)
                y = y0 - 1 + i
                real = (i < c.HROWS) & (sl >= 1) & (sl <= WI) & (y >= 0) & (y < WI)
                # element offset of the lane's 16-byte chunk (8 elements), plus the K-step advance
                off = (fbase + y * WI + (sl - 1)) * K + ch * 8
                for kt in kts:
                    e = off[real] + kt * 64
                    assert e.size == 0 or (e.min() >= 0 and e.max() + 8 <= M * K), (tile, wave, j, kt)
                # LDS destination of the wave-instruction (1 KiB) inside its ring slot
                dst = c.HSTRIDE * 2 + 128 + (wave + c.NW * j) * 1024
                assert dst + 1024 <= c.G_OFF
        # dwconv B-fragment reads (every wave's channel block / m-blocks), inside the H slot they belong to
        for wave in range(c.NW):
            cb, mb0 = wave & 3, (wave >> 2) * c.MPW
            for kk in range(5):
                t = np.minimum(2 * kk + (fq >> 1), 8)
                dy, dx = t // 3, t % 3
                L = fr + dy * c.SW + dx - 1
                cc = 2 * cb + (fq & 1)
                hoff = (L + 1) * 128 + ((cc ^ (L & 7)) << 4)
                for m in range(c.MPW):
                    a = mb0 * 2048 + hoff + m * 2048
                    assert a.min() >= 0 and a.max() + 16 <= c.HSTRIDE, (wave, kk, m)
    assert c.LDS <= 160 * 1024
