"""svk — MI355X (gfx950) kernels for the surgical-phase hot path, bound through a C ABI.

``svk.ops`` holds the torch-facing wrappers, ``svk._lib`` the ctypes binding of
``include/svk.h``, ``svk.pack`` the weight-packing cache used by ``models.*``.
"""
from . import _lib, ops, pack  # noqa: F401
from ._lib import SvkError, load, version  # noqa: F401


def default_dtype():
    """Compute dtype when a caller does not pin one: bf16 under a CUDA autocast region
    (train_evp.py:493 runs fp16 autocast; gfx950 prefers bf16), else fp32 (the
    reference's generate_evp_LFB / trans_SV_output run fp32)."""
    import torch
    if torch.is_autocast_enabled("cuda"):
        return torch.bfloat16
    return torch.float32
