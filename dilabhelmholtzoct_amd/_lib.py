"""ctypes binding of liboctsam_hip.so (the C ABI declared in include/octsam.h).

The library is loaded after ``torch`` so that the HIP runtime torch already mapped
(libamdhip64.so.7) is the one the library binds to: one runtime, one set of streams.
There is no fallback: if the library or a GPU is missing, every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# OCTSAM_LIB: another build of the same ABI (A/B diagnostics in scripts/, never set by the package itself)
LIB_PATH = os.environ.get("OCTSAM_LIB") or os.path.join(_HERE, "liboctsam_hip.so")

ACT_NONE, ACT_RELU, ACT_GELU = 0, 1, 2

c_void_p = ctypes.c_void_p
c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_float = ctypes.c_float


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("A", c_void_p), ("B", c_void_p), ("C", c_void_p), ("bias", c_void_p), ("R", c_void_p),
        ("C_pre", c_void_p), ("row_map", c_void_p), ("A2", c_void_p), ("B2", c_void_p),
        ("M", c_int32), ("N", c_int32), ("K", c_int32), ("batch", c_int32),
        ("lda", c_int64), ("ldb", c_int64), ("ldc", c_int64), ("ldr", c_int64),
        ("stride_a", c_int64), ("stride_b", c_int64), ("stride_c", c_int64), ("stride_r", c_int64),
        ("alpha", c_float), ("beta", c_float),
        ("act", c_int32), ("a_mode", c_int32), ("b_mode", c_int32),
        ("c_f32", c_int32), ("r_f32", c_int32), ("pre_f32", c_int32), ("conv_c", c_int32),
        ("a2_rows", c_int32), ("b2_rows", c_int32),
        ("a_blk", c_int32), ("a_rep", c_int32), ("b_blk", c_int32), ("b_rep", c_int32),
        ("r_blk", c_int32), ("r_rep", c_int32), ("k_total", c_int32), ("c_rows", c_int32),
        ("a_colsum", c_void_p), ("b_colsum", c_void_p),
    ]


# name -> (restype, argtypes); every symbol here is declared in include/octsam.h
_SIGNATURES = {
    "octsam_abi_version": (c_int32, []),
    "octsam_last_error": (ctypes.c_char_p, []),
    "octsam_gemm": (c_int32, [ctypes.POINTER(GemmArgs), c_void_p]),
    "octsam_gemm_f16": (c_int32, [ctypes.POINTER(GemmArgs), c_void_p]),
    "octsam_gemm_set_fast_path": (None, [c_int32]),
    "octsam_gemm_last_path": (c_int32, []),
    "octsam_gemm_debug_stamps": (c_int32, [c_void_p, c_int32]),
    "octsam_splitk_reduce": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_float, c_void_p]),
    "octsam_wgrad_supported": (c_int32, [c_int64, c_int32, c_int32]),
    "octsam_wgrad_tok": (c_int32, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_float,
                                   c_void_p, c_void_p]),
    "octsam_wgrad_tok_group": (c_int32, [c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "octsam_wgrad_workspace": (c_int64, [c_int64, c_int32, c_int32]),
    "octsam_wgrad": (c_int32, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_int32, c_void_p, c_float,
                               c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_void_p]),
    "octsam_cubical_ph": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p]),
    "octsam_layernorm_fwd": (c_int32, [c_void_p, c_int32, c_void_p, c_int64, c_int32, c_void_p, c_void_p,
                                       c_float, c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_void_p,
                                       c_void_p]),
    "octsam_layernorm_bwd": (c_int32, [c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_int32, c_int64, c_int32, c_void_p, c_int32, c_float,
                                       c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    "octsam_relu_bwd": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_int64, c_void_p]),
    "octsam_group_sum": (c_int32, [c_void_p, c_int64, c_int32, c_int32, c_int32, c_int64, c_void_p, c_void_p]),
    "octsam_vit_attention": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                       c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "octsam_attention_set_variant": (None, [c_int32]),
    "octsam_axpby": (c_int32, [c_void_p, c_int32, c_void_p, c_int32, c_int64, c_float, c_float, c_void_p,
                               c_int32, c_void_p, c_int64, c_void_p]),
    "octsam_colsum": (c_int32, [c_void_p, c_int32, c_int64, c_int32, c_void_p, c_int32, c_void_p]),
    "octsam_prompt_tokens": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_float, c_void_p, c_void_p]),
    "octsam_mask_embed": (c_int32, [c_void_p, c_int32, c_void_p, c_float, c_void_p, c_void_p]),
    "octsam_image_pe": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p]),
    "octsam_cast_bf16": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    "octsam_cast_f16": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    "octsam_patchify_bf16": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p]),
    "octsam_patchify_f16": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p]),
    "octsam_cc_label": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_int32, c_void_p,
                                  c_void_p]),
    "octsam_cc_assign": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int32, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_int32, c_void_p]),
    "octsam_sam_preprocess": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int64, c_void_p, c_int32,
                                        c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_int32,
                                        c_int32, c_void_p]),
    "octsam_dec_tok_attn_fwd": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                          c_void_p]),
    "octsam_dec_tok_attn_bwd": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32,
                                          c_void_p, c_void_p, c_void_p, c_void_p]),
    "octsam_dec_t2i_workspace": (c_int64, [c_int32, c_int32]),
    "octsam_dec_t2i_fwd": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_int32,
                                     c_void_p, c_void_p, c_void_p, c_void_p]),
    "octsam_dec_t2i_fwd_bias": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_int32,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "octsam_dec_t2i_bwd": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_int32,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                     c_void_p, c_void_p]),
    "octsam_dec_t2i_bwd_sum_workspace": (c_int64, [c_int32, c_int32, c_int32]),
    "octsam_dec_t2i_bwd_sum": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_int32,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                         c_void_p, c_void_p]),
    "octsam_dec_t2i_fwd2": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_int32,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "octsam_dec_t2i_bwd2": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_int32,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                      c_void_p, c_void_p]),
    "octsam_dec_t2i_bwd_sum2": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_int32,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_int64, c_void_p, c_void_p]),
    "octsam_dec_i2t_fwd": (c_int32, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                     c_void_p, c_int64, c_void_p]),
    "octsam_dec_i2t_bwd_partials": (c_int64, [c_int32, c_int32, c_int32]),
    "octsam_dec_i2t_bwd_sum_partials": (c_int64, [c_int32, c_int32, c_int32]),
    "octsam_dec_i2t_bwd_sum": (c_int32, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                         c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
    "octsam_dec_i2t_bwd": (c_int32, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                     c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
    "octsam_upmask_fwd": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    "octsam_upmask_bwd_workspace": (c_int64, [c_int32, c_int32]),
    "octsam_upmask_set_grid": (None, [c_int32, c_int32]),
    "octsam_upmask_bwd": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "octsam_upmask_ln_bwd": (c_int32, [c_void_p] * 5 + [c_int32, c_int32] + [c_void_p] * 13),
    "octsam_upmask_ln_bwd_strided": (c_int32, [c_void_p] * 5 + [c_int32, c_int32] + [c_void_p] * 6 + [c_int64] +
                                     [c_void_p] * 7),
    "octsam_postproc_fwd": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                                      c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    "octsam_dice_partials": (c_int32, [c_void_p, c_void_p, c_int32, c_int64, c_void_p, c_int32, c_void_p]),
    "octsam_confusion": (c_int32, [c_void_p, c_void_p, c_int32, c_int64, c_void_p, c_void_p]),
    "octsam_dice_reduce": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "octsam_dicece_bwd": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int64, c_float, c_float,
                                    c_void_p, c_void_p, c_int32, c_void_p]),
    "octsam_loss_finalize": (c_int32, [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int64, ctypes.c_double,
                                       ctypes.c_double, c_void_p, c_void_p]),
    "octsam_postproc_bwd": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "octsam_dicece_pp_rows": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_float,
                                        c_float, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p]),
    "octsam_pp_bwd_rows_maps": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_void_p]),
    "octsam_pp_bwd_cols": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p]),
    "octsam_topo_bwd_compact": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                                          c_void_p, c_float, c_void_p, c_void_p]),
    "octsam_topo_down": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32,
                                   c_int32, c_void_p, c_void_p, c_void_p]),
    "octsam_topo_bwd": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                                  c_void_p, c_float, c_void_p, c_void_p]),
    "octsam_w2_host": (c_int32, [c_void_p, c_int32, c_void_p, c_int32, ctypes.c_double, c_void_p, c_void_p]),
    "octsam_topo_host": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                   c_int32, c_int32, ctypes.c_double, ctypes.c_double, c_int32, c_void_p,
                                   c_void_p]),
    "octsam_topo_w2_workspace": (c_int64, [c_int32, c_int32]),
    "octsam_topo_w2": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                 c_void_p, c_int32, c_int32, ctypes.c_double, ctypes.c_double, c_int32, c_void_p,
                                 c_int64, c_void_p, c_void_p, c_void_p]),
    "octsam_adam": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, ctypes.c_double, ctypes.c_double, c_float,
                              c_float, c_float, c_float, c_void_p, c_void_p]),
}

_lib = None


class OctsamError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load the shared library (no GPU needed). Raises if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OctsamError(f"liboctsam_hip.so not built at {LIB_PATH}; run __graft_entry__.build()")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def symbols() -> list[str]:
    return list(_SIGNATURES)


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().octsam_last_error().decode(errors="replace")
        raise OctsamError(f"{what} failed (code {rc}): {msg}")


def stream_handle(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def call(name: str, *args) -> None:
    """Call a C-ABI entry point whose last argument is the stream; raise on error."""
    fn = getattr(load(), name)
    rc = fn(*args, c_void_p(stream_handle()))
    check(rc, name)


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def resolve_device(device) -> torch.device:
    """torch.device with an explicit index ("cuda" -> "cuda:<current>"), so device checks compare equal."""
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d
