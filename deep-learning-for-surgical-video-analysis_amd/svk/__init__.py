"""svk — MI355X (gfx950) kernels for the surgical-phase hot path, bound through a C ABI.

``svk.ops`` holds the torch-facing wrappers, ``svk._lib`` the ctypes binding of
``include/svk.h``, ``svk.pack`` the weight-packing cache used by ``models.*``.
"""
from . import _lib, ops, pack  # noqa: F401
from ._lib import SvkError, load, version  # noqa: F401


def default_dtype():
    """Compute dtype when a caller does not pin one: the autocast dtype inside a CUDA autocast
    region (the reference's train_evp.py:493/637/760 regions are torch.autocast(float16): f16
    MFMA with f32 accumulation, same MFMA rate as bf16 on gfx950), else fp32 (the reference's
    generate_evp_LFB / trans_SV_output run fp32)."""
    import torch
    if torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        return dt if dt in (torch.float16, torch.bfloat16) else torch.float16
    return torch.float32
