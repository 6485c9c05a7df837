"""ctypes binding of libfervit.so (declarations: `include/fervit.h`).

The product path has no CPU fallback: if the library is missing or fails to load,
`lib()` raises. Build it with `python __graft_entry__.py` (or `make -C fer-vit_amd/csrc`).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FERVIT_LIB", os.path.join(_HERE, "libfervit.so"))

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_int64
u32 = C.c_uint32
u64 = C.c_uint64
f32 = C.c_float
fp = C.c_void_p  # float* / any device pointer


class GemmDesc(C.Structure):
    _fields_ = [("dtype", i32), ("A", vp), ("lda", i64), ("a_kc", i32), ("B", vp), ("ldb", i64), ("b_kc", i32),
                ("M", i32), ("N", i32), ("K", i32), ("ws", vp), ("ws_bytes", i64)]


class Epilogue(C.Structure):
    _fields_ = [("c", vp), ("ldc", i64), ("c_f32", i32), ("accumulate", i32), ("alpha", f32),
                ("bias", vp), ("act", i32), ("pre", vp), ("ldp", i64), ("res", vp), ("ldr", i64),
                ("drop_thresh", u32), ("drop_scale", f32), ("seed", u64), ("drop_ld", i64),
                ("aux", vp), ("ldx", i64), ("aux_act", i32), ("post_scale", vp), ("colsum", vp),
                ("colsum_accumulate", i32)]


class WgradItem(C.Structure):
    _fields_ = [("dy", vp), ("ld_dy", i64), ("x", vp), ("ld_x", i64), ("dw", vp), ("ld_dw", i64),
                ("M", i32), ("N", i32), ("K", i32), ("accumulate", i32)]


class AdamWSegment(C.Structure):
    _fields_ = [("offset", i64), ("numel", i64), ("lr", f32), ("weight_decay", f32), ("beta1", f32),
                ("beta2", f32), ("eps", f32), ("step", i32)]


class ImageAug(C.Structure):
    _fields_ = [("flip_p", f32), ("degrees", f32), ("brightness", f32), ("contrast", f32), ("saturation", f32),
                ("hue", f32), ("translate", f32), ("scale_lo", f32), ("scale_hi", f32)]


# name -> (restype, argtypes)
SIGNATURES = {
    "fer_gemm": (i32, [C.POINTER(GemmDesc), C.POINTER(Epilogue), vp]),
    "fer_gemm_set_config": (i32, [i32]),
    "fer_set_persistent_mode": (i32, [i32]),
    "fer_stream_create_cu_mask": (i32, [C.POINTER(C.c_uint32), i32, i32, C.POINTER(C.c_void_p)]),
    "fer_stream_destroy": (i32, [vp]),
    "fer_gemm_colsum_ws": (i64, [i32, i32]),
    "fer_wgrad_group": (i32, [C.POINTER(WgradItem), i32, i32, fp, i64, vp]),
    "fer_wgrad_group_ws": (i64, [C.POINTER(WgradItem), i32, i32]),
    "fer_layernorm_fwd": (i32, [i32, vp, i64, fp, fp, i32, i32, vp, i64, fp, fp, i32, i32, f32, vp]),
    "fer_layernorm_bwd_ws": (i64, [i32, i32]),
    "fer_layernorm_bwd": (i32, [i32, vp, i64, vp, i64, fp, fp, fp, i32, i32, vp, i64, vp, i64, vp, u32, f32, u64,
                                fp, fp, fp, i32, fp, i64, i32, i32, vp]),
    "fer_attention_ws": (i64, [i32, i32, i32, i32]),
    "fer_attention_set_fwd_kernel": (i32, [i32]),
    "fer_attention_saved_floats": (i64, [i32, i32, i32, i32, i32, u32]),
    "fer_attention_fwd": (i32, [i32, vp, i64, vp, i64, fp, i64, i32, i32, i32, i32, f32, u32, f32, u64, fp, i64, vp]),
    "fer_attention_bwd": (i32, [i32, vp, i64, vp, i64, vp, i64, fp, i64, vp, i64, fp, i64, i32, i32, i32, i32, f32, u32,
                                f32, u64, fp, i32, vp]),
    "fer_colsum_ws": (i64, [i32, i32]),
    "fer_colsum": (i32, [i32, vp, i64, i32, i32, fp, i32, fp, fp, i64, vp]),
    "fer_reduce_defer": (i32, [i32, vp, i64, vp]),
    "fer_reduce_flush": (i32, []),
    "fer_im2col_patch": (i32, [i32, fp, i32, i32, i32, i32, i32, vp, i64, vp]),
    "fer_tokens_fwd": (i32, [i32, vp, fp, fp, vp, i32, i32, i32, u32, f32, u64, vp]),
    "fer_tokens_bwd_ws": (i64, [i32, i32, i32]),
    "fer_tokens_bwd": (i32, [i32, vp, vp, fp, fp, i32, i32, i32, i32, u32, f32, u64, fp, i64, vp]),
    "fer_head_fwd": (i32, [i32, vp, i64, fp, fp, f32, fp, fp, fp, fp, i32, i32, i32, u32, f32, u64, vp]),
    "fer_head_bwd_ws": (i64, [i32, i32, i32]),
    "fer_head_bwd": (i32, [i32, vp, i64, fp, fp, fp, fp, fp, vp, i32, i32, i32, fp, fp, fp, fp, i32, i32, i32, i32,
                           u32, f32, u64, fp, i64, vp]),
    "fer_cross_entropy": (i32, [fp, vp, fp, i32, i32, f32, f32, fp, fp, vp]),
    "fer_wplus_ws": (i64, [i32, i32, i32]),
    "fer_wplus_fwd": (i32, [fp, fp, i32, i32, i32, fp, fp, vp, fp, fp, fp, fp, f32, fp, vp]),
    "fer_wplus_bwd": (i32, [fp, fp, fp, fp, i32, i32, i32, fp, fp, vp, fp, fp, fp, fp, f32, fp, fp, fp, fp, fp, fp,
                            i32, fp, i64, vp]),
    "fer_decompose": (i32, [fp, fp, i32, i32, i32, i32, f32, i32, fp, fp, vp]),
    "fer_cast_f32_bf16": (i32, [fp, vp, i64, vp]),
    "fer_cast_bf16_f32": (i32, [vp, fp, i64, vp]),
    "fer_axpy": (i32, [i32, vp, vp, fp, vp, i64, vp]),
    "fer_dot": (i32, [i32, vp, vp, i64, fp, i32, fp, i64, vp]),
    "fer_dropout": (i32, [i32, vp, vp, i64, u32, f32, u64, vp]),
    "fer_adamw": (i32, [fp, fp, fp, fp, vp, vp, i32, i64, f32, fp, vp, vp]),
    "fer_set_step_counter": (i32, [vp]),
    "fer_latent_augment": (i32, [fp, i64, i32, f32, f32, f32, f32, u64, vp]),
    "fer_step_advance": (i32, [vp, vp]),
    "fer_transpose_bf16_segments": (i32, [vp, vp, vp, i32, i64, vp]),
    "fer_image_aug_draw": (i32, [fp, i32, i32, vp, u64, vp]),
    "fer_image_augment": (i32, [vp, vp, vp, i32, i32, fp, i32, vp, vp, fp, vp]),
    "fer_sumsq": (i32, [fp, i64, fp, fp, i64, vp]),
    "fer_clip_coef": (i32, [fp, f32, f32, fp, vp]),
    "fer_last_error": (C.c_char_p, []),
    "fer_version": (C.c_char_p, []),
}

_LIB = None


class FerError(RuntimeError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise FerError(f"libfervit.so not found at {LIB_PATH}: build it with `python __graft_entry__.py` "
                           "(hipcc, gfx950). There is no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().fer_last_error().decode()
        raise FerError(f"fervit {what}: {msg} (rc={rc})")
