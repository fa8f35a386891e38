"""ctypes binding of the svk C ABI (include/svk.h).

This is the reference-side binding a maintainer would add: the reference has no
FFI of its own (its boundary is the Python module surface), so the
build's ``models.*`` modules call these symbols through ctypes.  Loading fails
loudly when the shared library is missing — there is no CPU fallback.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SVK_LIB", os.path.join(_HERE, "libsvk.so"))

c_int, c_long, c_float, c_void_p, c_char_p = ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_void_p, ctypes.c_char_p
P = c_void_p

# name -> argtypes; every entry point returns int status except the two string getters.
SIGNATURES = {
    "svk_gemm": [c_int, P, c_long, P, c_long, P, P, c_long, P, c_long, c_int, c_int, c_int, c_int, P],
    "svk_tune": [c_char_p, c_int],
    "svk_conv2d_nhwc": [c_int, P, c_int, c_int, c_int, c_int, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P],
    "svk_layernorm": [c_int, P, c_long, P, c_long, P, P, c_int, c_int, c_float, P],
    "svk_conv2d_ln_nhwc": [c_int, P, c_int, c_int, c_int, c_int, P, P, P, P, c_float, P, c_int, c_int, c_int,
                           c_int, P, c_long, P],
    "svk_attention": [c_int, P, c_long, c_long, P, c_long, c_long, P, c_long, c_long, P, c_long, c_long,
                      c_int, c_int, c_int, c_int, c_int, c_float, P],
    "svk_dwconv3x3": [c_int, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P],
    "svk_mixffn_fc1_dwconv": [c_int, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "svk_mixffn_fc1_dwconv_ex": [c_int, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "svk_nchw_to_nhwc": [c_int, P, P, c_int, c_int, c_int, c_int, c_int, P],
    "svk_gauss5x5_reflect": [c_int, P, P, c_int, c_int, c_int, c_int, c_int, P],
    "svk_nchw_to_s2d": [c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "svk_gauss5x5_s2d": [c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "svk_resize_bilinear": [c_int, P, c_long, P, c_long, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "svk_resize_bilinear_multi": [c_int, c_int, P, P, P, P, P, P, c_long, c_int, c_int, c_int, P],
    "svk_mean_rows": [c_int, P, c_long, P, c_int, c_int, c_int, P],
    "svk_softmax_rows": [P, c_long, P, c_long, c_int, c_int, P],
    "svk_mstcn_layer": [P, P, P, P, P, P, c_int, c_int, c_int, c_int, P],
    "svk_mstcn_layer_ragged": [P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, P],
    "svk_mamba_conv_silu": [P, c_long, P, P, P, c_int, c_int, c_int, c_int, P],
    "svk_mamba_conv_silu_ragged": [P, c_long, P, P, P, P, c_long, c_int, c_int, P],
    "svk_mamba_scan_ragged": [P, P, c_long, P, c_long, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P, P],
    "svk_mamba_scan": [P, P, c_long, P, c_long, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P],
    "svk_mamba_scan_train": [P, P, c_long, P, c_long, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P,
                             P],
    "svk_mamba_scan_bwd": [P, P, c_long, P, c_long, P, P, P, P, P, P, P, P, c_long, P, P, c_long, P, P, c_int, c_int,
                           c_int, c_int, c_int, P, P],
    "svk_mamba_conv_silu_bwd": [P, c_long, P, P, P, P, P, c_long, P, P, c_int, c_int, c_int, c_int, P],
    "svk_mstcn_layer_train": [P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, P],
    "svk_mstcn_layer_bwd": [P, P, P, P, P, P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, P],
    "svk_softmax_rows_bwd": [P, c_long, P, c_long, P, c_long, P, c_long, c_int, c_int, P],
    "svk_neg_exp": [P, P, c_long, P],
    "svk_phase_metrics": [P, P, P, c_int, c_int, c_int, P, P],
    "svk_tecno_loss": [P, c_long, c_long, c_int, c_int, c_int, P, P, P, P, P, P],
    "svk_grad_sqnorm": [P, c_long, P, P, P],
    "svk_norm_parts": [],
    "svk_adamw": [P, P, P, P, c_long, P, c_float, P, c_float, c_float, c_float, c_float, P, P],
    "svk_frame_preproc": [P, P, P, P, P, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P,
                          P],
    "svk_flow_preproc": [P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float, P],
    "svk_train_augment": [P, P, P, P, P, P, P, c_int, P, P, c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                          P, P, P],
    "svk_train_augment_flow": [P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_float, c_float, P],
    "svk_anticipation_gt": [P, c_long, c_int, c_int, ctypes.c_double, P, P],
    "svk_window_unfold": [c_int, P, c_long, P, P, c_int, c_int, c_int, P],
    "svk_add_bcast": [c_int, P, P, P, c_long, c_int, c_int, P],
    "svk_attn_block": [c_int, P, P, P, c_long, P, P, P, P, P, P, c_float, P, P, c_int, c_int, c_int, c_int,
                          c_float, P],
    "svk_prompt_ln": [c_int, P, P, P, P, P, P, P, P, c_float, P, P, c_int, c_int, P],
    "svk_mixffn_fused": [c_int, P, P, P, P, P, P, P, P, P, P, P, c_float, c_int, c_int, c_int, c_int, P],
    "svk_mixffn_rw": [c_int, P, P, P, P, P, P, P, P, P, P, P, P, c_float, c_int, c_int, c_int, c_int, P],
    "svk_mixffn_dw_fc2": [c_int, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P],
    "svk_mixffn_dw_fc2_pack": [c_int, P, P, P, c_int, c_int, c_int, P, P],
    "svk_gemm_ln_pack": [c_int, P, c_int, c_int, P, P],
    "svk_gemm_ln": [c_int, P, c_int, c_int, P, P, P, P, P, c_float, P, P, c_int, P],
    "svk_mixffn_dw_fc2_packed": [c_int, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P],
    "svk_mixffn_dw_fc2_packed_act": [c_int, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "svk_mixffn_dw_fc2_packed_ex": [c_int, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, c_int, P],
    "svk_conv2d_s2d_ln": [c_int, P, c_int, c_int, c_int, c_int, P, P, P, P, c_float, P, c_int, P],
    "svk_cast": [c_int, P, c_int, P, c_long, P],
    # training step
    "svk_dwconv3x3_ex": [c_int, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P],
    "svk_gemm_ex": [c_int, P, c_long, P, c_long, P, P, c_int, P, c_long, c_int, P, c_long, P, c_long, c_int, c_int,
                    c_int, c_int, P],
    "svk_gemm_unpatchify": [c_int, P, c_long, P, c_long, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "svk_gemm_wgrad": [c_int, P, c_long, P, c_long, P, c_long, P, c_int, c_int, c_int, P],
    "svk_gemm_skinny": [c_int, P, c_long, P, c_long, P, P, c_long, c_int, P, c_long, P, c_long, c_int, c_int, c_int, c_int, P],
    "svk_wgrad_skinny": [P, c_long, P, c_long, P, c_long, P, c_int, c_int, c_int, P],
    "svk_conv2d_wgrad_nhwc": [c_int, P, c_int, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int, P, P, P],
    "svk_conv2d_dgrad_nhwc": [c_int, P, c_int, c_int, c_int, c_int, P, P, P, c_int, c_int, c_int, c_int, c_int,
                              c_int, P],
    "svk_unpatchify": [c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "svk_col2im_nhwc": [c_int, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "svk_attention_bwd": [c_int, P, c_long, c_long, P, c_long, c_long, P, c_long, c_long, P, c_long, c_long,
                          P, c_long, c_long, P, c_long, c_long, P, P, c_long, c_long, P, c_long, c_int, c_int, c_int,
                          c_int, c_int, c_float, P],
    "svk_layernorm_bwd": [c_int, P, c_long, P, c_long, P, P, c_long, P, c_long, P, P, c_int, c_int, c_float, P],
    "svk_act_bwd": [c_int, P, P, P, P, c_long, c_int, P],
    "svk_colstats": [c_int, P, c_long, c_int, c_int, P, P, P, P],
    "svk_colstats_set": [c_int, P, c_long, c_int, c_int, P, P, P],
    "svk_bn_apply": [c_int, P, P, P, P, P, P, c_int, c_int, c_float, c_int, P],
    "svk_bn_bwd": [c_int, P, P, P, P, P, P, P, P, P, c_int, c_int, c_float, c_int, P, P],
    "svk_bn_update_running": [P, P, c_int, c_int, c_float, P, P, P],
    "svk_resize_bilinear_bwd": [c_int, P, c_long, P, c_int, c_int, c_int, c_int, c_int, c_int, P],
    "svk_bcast_rows": [c_int, P, P, c_float, P, c_int, c_int, c_int, P],
    "svk_row_scale": [c_int, P, P, P, c_long, c_int, c_int, P],
    "svk_mul_f32": [P, P, P, c_long, P],
    "svk_keep_mask": [P, c_long, c_float, ctypes.c_uint, P, P],
    "svk_keep_mask_multi": [P, c_long, c_int, P, P, P, P],
    "svk_phase_loss": [P, P, P, P, c_int, c_int, P, P, P, P],
    "svk_sgd": [P, P, P, c_long, c_float, c_float, c_float, c_float, c_int, c_int, P],
    "svk_pack_params": [c_int, P, c_int, c_long, P, P, P],
    "svk_pack_params8": [c_int, P, c_int, c_long, P, P, P],
    "svk_pack_transpose": [c_int, P, c_int, P, P, P],
}
STRING_FUNCS = ("svk_version", "svk_last_error", "svk_last_kernel")
LONG_FUNCS = {"svk_attention_bwd_workspace": [c_int, c_int, c_int, c_int, c_int, c_int],
              "svk_mixffn_dw_fc2_packed_bytes": [c_int, c_int, c_int, c_int],
              "svk_gemm_ln_packed_bytes": [c_int, c_int, c_int],
              "svk_conv2d_ln_workspace": [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int],
              "svk_mamba_scan_workspace": [c_int, c_int, c_int, c_int, c_int],
              "svk_mamba_scan_bwd_workspace": [c_int, c_int, c_int, c_int],
              "svk_mamba_scan_ragged_workspace": [c_int, c_int, c_int],
              "svk_mstcn_bwd_workspace": [c_int, c_int],
              "svk_stats_ws_floats": [c_int, c_int]}
INT_QUERIES = {"svk_mixffn_supported": [c_int, c_int], "svk_mixffn_rw_supported": [c_int, c_int, c_int],
               "svk_mixffn_dw_fc2_supported": [c_int, c_int, c_int, c_int],
               "svk_conv2d_s2d_ln_supported": [c_int, c_int, c_int, c_int], "svk_mstcn_tile_size": []}

_lib = None


class SvkError(RuntimeError):
    pass


def load():
    """Load libsvk.so once and declare every signature.  Raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SvkError(f"svk: HIP kernel library not found at {LIB_PATH}; build it with "
                       f"`python -c 'import __graft_entry__ as g; g.build()'` (make -C csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:          # an older library build (SVK_LIB): the symbol fails when called
            continue
        fn.argtypes = argtypes
        fn.restype = c_int
    for name in STRING_FUNCS:
        fn = getattr(lib, name)
        fn.argtypes = []
        fn.restype = c_char_p
    for name, argtypes in LONG_FUNCS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = argtypes
        fn.restype = c_long
    for name, argtypes in INT_QUERIES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = argtypes
        fn.restype = c_int
    _lib = lib
    return lib


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise SvkError(f"{name} failed ({rc}): {load().svk_last_error().decode()}")


def version():
    return load().svk_version().decode()
