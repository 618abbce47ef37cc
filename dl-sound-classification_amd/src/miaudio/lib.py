"""ctypes binding of libmiaudio.so (include/miaudio.h).

This is the whole native boundary: every entry point is an ``extern "C"`` function taking
plain pointers, sizes and a hipStream_t.  The library is loaded from the package's ``lib/``
directory (built in-tree by ``make``); there is no fallback — a missing library raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch

PKG_ROOT = Path(__file__).resolve().parents[2]
LIB_PATH = Path(os.environ.get("MIAUDIO_LIB") or PKG_ROOT / "lib" / "libmiaudio.so")

F32, BF16, U8 = 0, 1, 2
# model compute mode (not a tensor dtype): bf16 compute with the AST block linears' forward GEMMs on MX-fp8
# operands (trainer.precision=fp8-mixed)
MXFP8 = 16
OP_DENSE, OP_CONV, OP_CONVROW = 0, 1, 2
KC, RC = 0, 1
PRE_NONE, PRE_AFFINE, PRE_AFFINE_RELU, PRE_GELU = 0, 1, 2, 3
ACT_NONE, ACT_RELU, ACT_GELU, DACT_NZ, DACT_GELU, ACT_ADD_AUX, ACT_GELU_SAVE = 0, 1, 2, 3, 4, 5, 6
ACT_GELU_SAVE_D, DACT_MUL = 7, 8

vp = C.c_void_p
i32 = C.c_int32
i64 = C.c_int64
f32 = C.c_float


class MiaOperand(C.Structure):
    _fields_ = [("ptr", vp), ("kind", i32), ("dtype", i32), ("layout", i32), ("pre", i32),
                ("rows", i64), ("cols", i64), ("ld", i64),
                ("n", i32), ("h", i32), ("w", i32), ("c", i32),
                ("oh", i32), ("ow", i32), ("kh", i32), ("kw", i32),
                ("sh", i32), ("sw", i32), ("ph", i32), ("pw", i32),
                ("pre_scale", vp), ("pre_shift", vp)]


class MiaEpilogue(C.Structure):
    _fields_ = [("ptr", vp), ("dtype", i32), ("act", i32), ("accumulate", i32), ("aux_dtype", i32),
                ("ldc", i64), ("rm_inner", i64), ("rm_outer", i64), ("rm_istride", i64),
                ("rm_offset", i64), ("bias", vp), ("aux", vp), ("ldaux", i64),
                ("alpha", f32), ("act_scale", f32), ("sqsum", vp), ("colsum", vp), ("mx_q", vp),
                ("mx_scales", vp), ("a_colsum", vp)]


class MiaPackJob(C.Structure):
    _fields_ = [("src", vp), ("dst", vp), ("dtype", i32), ("cout", i32), ("cin", i32), ("kh", i32), ("kw", i32),
                ("mode", i32)]


PACK_BATCH = 16  # MIA_PACK_BATCH
RM_DROP = -1  # MIA_RM_DROP: MiaEpilogue.rm_offset sentinel of the drop-mode row map


class MiaMelCfg(C.Structure):
    _fields_ = [("sample_rate", i32), ("n_fft", i32), ("win_length", i32), ("hop", i32),
                ("n_mels", i32), ("normalize", i32), ("top_db", f32), ("target_mean", f32),
                ("target_std", f32)]


P = C.POINTER
# name -> (restype, argtypes)
SIGNATURES = {
    "mia_gemm_workspace_bytes": (i64, [i64, i64, i32]),
    "mia_gemm_workspace_bytes_ex": (i64, [P(MiaOperand), P(MiaOperand), P(MiaEpilogue), i64, i64, i64, i32, i32]),
    "mia_gemm_sqsum_slots": (i64, [i64, i64]),
    "mia_gemm_sqsum_only": (C.c_int, [P(MiaOperand), P(MiaOperand), i64, i64, i64, vp, vp]),
    "mia_gemm_adam": (C.c_int, [P(MiaOperand), P(MiaOperand), i64, i64, i64, vp, vp, vp, vp, i64, vp, f32, f32, f32,
                                f32, f32, f32, vp]),
    "mia_gemm": (C.c_int, [P(MiaOperand), P(MiaOperand), P(MiaEpilogue), i64, i64, i64, i32, i32, vp, vp]),
    "mia_gemm_path": (C.c_int, [P(MiaOperand), P(MiaOperand), i64, i64, i64, i32, i32]),
    "mia_mx_quantize": (C.c_int, [vp, i32, i64, i64, i64, vp, i64, vp, vp]),
    "mia_gemm_mxfp8": (C.c_int, [vp, vp, i64, vp, vp, i64, P(MiaEpilogue), i64, i64, i64, vp]),
    "mia_mx_quantize_t": (C.c_int, [vp, i32, i64, i64, i64, vp, i64, vp, vp]),
    "mia_gemm_mxfp8_workspace_bytes": (i64, [i64, i64, i32]),
    "mia_gemm_mxfp8_ex": (C.c_int, [vp, vp, i64, vp, vp, i64, P(MiaEpilogue), i64, i64, i64, vp, vp]),
    "mia_layernorm_fwd_mx": (C.c_int, [vp, i32, vp, vp, vp, vp, vp, vp, vp, i64, i32, f32, vp]),
    "mia_attn_fwd_mx": (C.c_int, [vp, vp, vp, vp, vp, i32, i32, i32, f32, vp]),
    "mia_splitk_reduce": (C.c_int, [vp, i32, i64, i64, P(MiaEpilogue), vp]),
    "mia_logmel_workspace_bytes": (i64, [i64, i64]),
    "mia_logmel_fwd": (C.c_int, [vp, i64, i64, i64, P(MiaMelCfg), vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "mia_bn_partial_bytes": (i64, [i64, i32]),
    "mia_bn_fwd_stats": (C.c_int, [vp, i32, i64, i32, vp, vp, vp, vp, f32, f32, i32, vp, vp, vp, vp, vp, vp]),
    "mia_bn_relu_bwd_reduce": (C.c_int, [vp, vp, vp, i32, i64, i32, vp, vp, vp, vp, vp, vp, vp, vp]),
    "mia_bn_bwd_apply": (C.c_int, [vp, vp, vp, i32, i64, i32, vp, vp, vp, vp, vp, vp, vp, vp]),
    "mia_bn_relu_bwd_apply": (C.c_int, [vp, vp, vp, i32, i64, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "mia_pool_bwd_gather": (C.c_int, [vp, i32, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp,
                                      vp, vp, vp]),
    "mia_pool_bn_relu_bwd_apply": (C.c_int, [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp,
                                             vp, vp, vp]),
    "mia_pool_fwd": (C.c_int, [vp, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, i32, vp, vp, vp]),
    "mia_pool_bwd_bn_relu_reduce": (C.c_int, [vp, i32, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp,
                                              vp, vp, vp, vp, vp, vp]),
    "mia_colsum": (C.c_int, [vp, i32, i64, i32, i64, vp, vp, vp]),
    "mia_col2im_rows": (C.c_int, [vp, i32, i32, i32, i32, vp, i32, vp]),
    "mia_conv1ch_dgrad": (C.c_int, [vp, vp, vp, i32, i32, i32, vp]),
    "mia_fe_conv2_fwd": (C.c_int, [vp, vp, vp, vp, vp, vp, i32, i32, i32, vp]),
    "mia_fe_conv2_dgrad": (C.c_int, [vp, vp, vp, i32, i32, i32, vp]),
    "mia_bn_relu_apply": (C.c_int, [vp, i64, i32, vp, vp, vp, vp]),
    "mia_shift_pad_w2": (C.c_int, [vp, i64, i32, i32, vp, vp]),
    "mia_pad_w2": (C.c_int, [vp, i64, i32, i32, vp, vp, i32, vp]),
    "mia_drop_last_col": (C.c_int, [vp, i64, i32, i32, vp, vp]),
    "mia_fe_conv1_fwd": (C.c_int, [vp, vp, vp, vp, vp, i32, i32, i32, vp]),
    "mia_fe_conv3_fwd": (C.c_int, [vp, vp, vp, vp, vp, i32, i32, i32, i32, vp]),
    "mia_pool_raw_stats": (C.c_int, [vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, i32, vp]),
    "mia_pool_apply": (C.c_int, [vp, i32, i32, i32, i32, vp, vp, vp, i32, i32, vp]),
    "mia_conv3_wgrad": (C.c_int, [vp, vp, vp, vp, i32, i32, i32, i32, vp]),
    "mia_conv3_wgrad_workspace_bytes": (C.c_int64, [i32]),
    "mia_conv3_wgrad_bn": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp]),
    "mia_trunk_conv8": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "mia_trunk_conv8_dgrad_bn": (C.c_int, [vp, vp, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "mia_bn_finalize_shifted": (C.c_int, [vp, i32, i64, i32, vp, vp, vp, vp, vp, C.c_float, C.c_float, i32, vp, vp, vp,
                                          vp, vp]),
    "mia_fe_conv2_wgrad": (C.c_int, [vp, vp, vp, vp, vp, i32, i32, i32, vp, i64, vp]),
    "mia_fe_conv1_wgrad_bn": (C.c_int, [vp, vp, vp, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp]),
    "mia_pack_weight": (C.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "mia_pack_weights": (C.c_int, [P(MiaPackJob), i32, vp]),
    "mia_dropout": (C.c_int, [vp, i32, i64, f32, C.c_uint64, vp]),
    "mia_soft_ce": (C.c_int, [vp, vp, i32, i32, i32, vp, vp, vp, vp]),
    "mia_adam_workspace_bytes": (i64, [i32]),
    "mia_adam_coef_offset": (i64, [i32]),
    "mia_clip_adam": (C.c_int, [vp, vp, vp, vp, vp, vp, i32, i64, i64, f32, f32, f32, f32, f32, i32, f32, vp, vp, vp, vp,
                                vp, vp]),
    "mia_layernorm_fwd": (C.c_int, [vp, i32, vp, vp, vp, i32, vp, vp, i64, i32, f32, vp]),
    "mia_layernorm_bwd": (C.c_int, [vp, i32, vp, i32, vp, vp, vp, vp, i32, i32, vp, i32, vp, vp, vp, i64, i32, vp]),
    "mia_layernorm_partial_bytes": (i64, [i64, i32]),
    "mia_layernorm_bwd_colsum": (C.c_int, [vp, i32, vp, i32, vp, vp, vp, vp, i32, i32, vp, i32, vp, vp, vp, vp, i64,
                                           i32, vp]),
    "mia_layernorm_bwd_colsum_mx": (C.c_int, [vp, i32, vp, i32, vp, vp, vp, vp, i32, i32, vp, vp, vp, vp, vp, vp, vp, i64, i32, vp]),
    "mia_attn_fwd": (C.c_int, [vp, vp, vp, i32, i32, i32, i32, f32, vp]),
    "mia_attn_bwd": (C.c_int, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, vp]),
    "mia_attn_bwd_workspace_bytes": (C.c_int64, [i32, i32, i32, i32]),
    "mia_attn_saved_q_bytes": (C.c_int64, [i32, i32, i32]),
    "mia_attn_bwd_chain_bytes": (C.c_int64, [i32, i32, i32]),
    "mia_attn_bwd_onepass": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, i32, vp]),
    "mia_attn_fwd_save_q": (C.c_int, [vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, vp]),
    "mia_attn_bwd_saved_q": (C.c_int, [vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, vp]),
    "mia_attn_bwd_two_pass": (C.c_int, [vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, i32, vp]),
    "mia_attn_bwd_fused": (C.c_int, [vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, i32, vp]),
    "mia_attn_bwd_error_offset": (C.c_int64, [i32, i32, i32]),
    "mia_stream_copy": (C.c_int, [vp, vp, i64, vp]),
    "mia_mfma_rate_sink_floats": (i64, [i32]),
    "mia_mfma_rate": (C.c_int, [vp, i32, i32, vp]),
    "mia_tokens_fwd": (C.c_int, [vp, vp, vp, vp, i32, i32, i32, vp]),
    "mia_tokens_bwd": (C.c_int, [vp, vp, vp, vp, i32, i32, i32, vp]),
    "mia_ast_patches": (C.c_int, [vp, i32, i32, i32, i32, i32, vp, vp]),
    "mia_tokens_fwd_inplace": (C.c_int, [vp, vp, vp, i32, i32, i32, vp]),
    "mia_cast": (C.c_int, [vp, i32, vp, i32, i64, vp]),
    "mia_add_inplace": (C.c_int, [vp, vp, i32, i64, vp]),
    "mia_bc_mix": (C.c_int, [vp, vp, i64, i32, vp, vp, vp, vp, i32, vp, vp, vp, vp, vp]),
    "mia_bc_partner": (C.c_int, [vp, i32, vp, i32, vp, vp, vp]),
    "mia_stretch_gain": (C.c_int, [vp, i64, i32, vp, vp, vp, vp]),
    "mia_spec_augment_mixup":(C.c_int, [vp, vp, vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp]),
    "mia_last_error_string": (C.c_char_p, []),
    "mia_device_arch": (C.c_int, [C.c_char_p, i32]),
}

_LIB = None


def load(path: Path | str | None = None):
    """Load libmiaudio.so once; raise RuntimeError if it is missing (no fallback path)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise RuntimeError(f"libmiaudio.so not found at {p}: build it with `make -C {PKG_ROOT}` "
                           "(the MI355X kernels have no CPU fallback)")
    lib = C.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def exported_symbols():
    lib = load()
    return {n for n in SIGNATURES if hasattr(lib, n)}


def check(rc: int, what: str):
    if rc != 0:
        msg = load().mia_last_error_string()
        raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.uint8:
        return U8
    raise TypeError(f"unsupported dtype {t.dtype}")


def torch_dtype(code: int):
    return {F32: torch.float32, BF16: torch.bfloat16, U8: torch.uint8}[code]


def require_device(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"{what}: tensors must live on the MI355X (got {t.device}); "
                           "this implementation has no CPU path")


def device_arch() -> str:
    buf = C.create_string_buffer(64)
    check(load().mia_device_arch(buf, 64), "mia_device_arch")
    return buf.value.decode()
