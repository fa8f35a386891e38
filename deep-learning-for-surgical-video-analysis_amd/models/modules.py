"""Drop-in for the reference's ``models/modules.py`` — star-imported by trans_SV_output.py:16 and
tecno_trans.py:12, whose code then uses none of its names (an older copy of the EVP
prompt-generator building blocks).  The import must resolve and export the same public names:
``OverlapPatchEmbed``, ``PromptGenerator`` and ``GaussianFilter`` are the svk-backed classes of
``models.mix_transformer_evp`` (identical constructor signatures and state-dict keys); ``SRMFilter``
(modules.py:370-412) keeps its fixed, frozen 5x5 SRM high-pass bank as the parameter container
``srm_layer`` that the reference's 'srm' prompt input calls directly.
"""
import math  # noqa: F401  (re-exported by the reference's star import)

import torch
import torch.nn as nn

from .mix_transformer_evp import OverlapPatchEmbed, PromptGenerator, GaussianFilter  # noqa: F401

__all__ = ["OverlapPatchEmbed", "PromptGenerator", "GaussianFilter", "SRMFilter", "torch", "nn", "math"]

_SRM_1 = [[0, 0, 0, 0, 0],
          [0, -1 / 4, 2 / 4, -1 / 4, 0],
          [0, 2 / 4, -4 / 4, 2 / 4, 0],
          [0, -1 / 4, 2 / 4, -1 / 4, 0],
          [0, 0, 0, 0, 0]]
_SRM_2 = [[-1 / 12, 2 / 12, -2 / 12, 2 / 12, -1 / 12],
          [2 / 12, -6 / 12, 8 / 12, -6 / 12, 2 / 12],
          [-2 / 12, 8 / 12, -12 / 12, 8 / 12, -2 / 12],
          [2 / 12, -6 / 12, 8 / 12, -6 / 12, 2 / 12],
          [-1 / 12, 2 / 12, -2 / 12, 2 / 12, -1 / 12]]
_SRM_3 = [[0, 0, 0, 0, 0],
          [0, 0, 0, 0, 0],
          [0, 1 / 2, -2 / 2, 1 / 2, 0],
          [0, 0, 0, 0, 0],
          [0, 0, 0, 0, 0]]


class SRMFilter(nn.Module):
    """Three fixed SRM residual filters (each applied to the sum of the RGB channels), frozen."""

    def __init__(self):
        super().__init__()
        self.srm_layer = nn.Conv2d(3, 3, kernel_size=5, stride=1, padding=2)
        with torch.no_grad():
            self.srm_layer.weight.copy_(torch.tensor([[f, f, f] for f in (_SRM_1, _SRM_2, _SRM_3)]))
        for p in self.srm_layer.parameters():
            p.requires_grad = False
