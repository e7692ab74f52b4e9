"""ctypes binding of libmapfed.so (the C ABI declared in include/mapfed.h).

The product path has no fallback: if the library is missing or fails to load, `lib()` raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "lib" / "libmapfed.so"

P, I, L, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float

# name -> argtypes (all return int status unless listed in _RET)
SIGNATURES = {
    "mf_abi_version": [],
    "mf_gemm_nt": [P, L, P, L, P, L, I, I, I, P, P, P, L, I, I, P],
    "mf_gemm": [P, L, I, P, L, I, P, L, I, I, I, P, P, P, L, I, I, P],
    "mf_layernorm_fwd": [P, L, P, P, P, P, L, P, P, I, I, P],
    "mf_layernorm_bwd_blocks": [I],
    "mf_layernorm_bwd": [P, L, P, L, P, P, P, P, P, L, P, L, P, P, P, I, I, I, P],
    "mf_col_reduce_desc_bytes": [],
    "mf_col_reduce_batch": [P, I, I, P],
    "mf_attention_fwd": [P, L, P, L, P, I, I, I, I, I, P],
    "mf_attention_fwd_rows": [P, L, P, L, P, I, I, I, I, I, I, P],
    "mf_attention_bwd": [P, L, P, L, P, L, P, P, I, P, L, I, I, I, I, P],
    "mf_qkv_attention_fwd": [P, L, I, P, P, P, L, P, L, P, I, I, I, I, I, P],
    "mf_qkv_attention_supported": [I, I, I, I],
    "mf_im2col_patch": [P, I, P, I, I, I, P],
    "mf_vision_assemble": [P, P, P, P, P, I, I, I, I, P],
    "mf_text_assemble": [P, P, P, P, P, I, I, I, I, P],
    "mf_prompt_inject_fwd": [P, P, I, I, I, I, I, P],
    "mf_prompt_inject_bwd": [P, I, I, I, I, I, P, I, I, I, P],
    "mf_transpose_f16": [P, L, P, L, I, I, P],
    "mf_colsum_blocks": [I],
    "mf_colsum_f16": [P, L, I, I, P, I, P, P],
    "mf_cast_f16_f32": [P, P, L, P],
    "mf_small_linear_fwd": [P, P, P, P, I, I, I, I, P],
    "mf_small_linear_bwd": [P, P, P, P, P, P, I, I, I, I, I, P],
    "mf_gemm_splitk_ws_floats": [I, I, I, I],
    "mf_small_linear_desc_bytes": [],
    "mf_small_linear_fwd_batch": [P, I, I, P],
    "mf_small_linear_bwd_batch": [P, I, I, I, I, P],
    "mf_clip_head_fwd": [P, P, I, I, I, P, P, P, P, P, P, P],
    "mf_clip_loss_fwd_bwd": [P, P, P, P, P, P, P, I, I, I, P, P, P, P, P, P, P, P, P],
    "mf_layernorm_bwd_inject": [P, L, P, L, P, P, P, P, L, P, L, P, I, I, P, I, I, I, P],
    "mf_layernorm_fwd_inject": [P, L, P, P, P, L, P, P, I, I, P, I, I, I, P],
    "mf_gemm_splitk": [P, L, I, P, L, I, P, L, I, I, I, P, L, I, I, P],
    "mf_clip_loss_soft_fwd_bwd": [P, P, P, P, P, P, P, I, I, I, P, P, P, P, P, P, P, P, P, P],
    "mf_argmax_correct": [P, I, I, P, P, P, P],
    "mf_optim_chunk_bytes": [],
    "mf_optim_chunk_elems": [],
    "mf_clip_grad_norm": [P, P, P, I, F, P, P, P],
    "mf_sgd_step": [P, P, P, L, I, P, P, P],
    "mf_optimizer_step": [P, P, P, L, P, P, P, L, P, I, F, P, P, P, P, P, P],
    "mf_fedavg_pack": [P, L, P, L, P, P, P],
    "mf_fedavg_unpack": [P, P, L, P, L, P, P, P],
    "mf_fedavg_reduce_ordered": [P, I, L, L, P, P],
    "mf_seq_grow": [P, P, P, P, I, I, I, I, I, P],
    "mf_seq_grow_bwd": [P, P, I, I, I, I, I, P],
    "mf_seq_scatter": [P, L, P, L, I, I, I, I, P],
    "mf_layernorm_bwd_live": [P, L, P, L, P, P, P, P, L, P, L, P, I, I, I, I, P, I, I, P],
    "mf_caption_pool": [P, I, I, P, I, P, I, P, P],
    "mf_nonfinite_flag": [P, L, I, P, P],
    "mf_augment_ws_bytes": [I, I, I, I],
    "mf_augment": [P, L, P, P, P, I, I, I, I, F, F, F, F, F, F, P, I, P, L, P],
}
# functions that return a value, not a status
_VALUE_FUNCS = {"mf_abi_version", "mf_layernorm_bwd_blocks", "mf_colsum_blocks", "mf_optim_chunk_bytes",
                "mf_optim_chunk_elems", "mf_col_reduce_desc_bytes", "mf_small_linear_desc_bytes",
                "mf_gemm_splitk_ws_floats", "mf_augment_ws_bytes", "mf_qkv_attention_supported"}
# value functions whose return type is not int
_RESTYPES = {"mf_augment_ws_bytes": ctypes.c_int64}

_LIB = None


class MapfedError(RuntimeError):
    pass


def lib():
    """Load libmapfed.so once; raise (never fall back) if it is missing."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.environ.get("MAPFED_LIB", str(LIB_PATH))
    if not os.path.exists(path):
        raise MapfedError(f"libmapfed.so not found at {path}: run __graft_entry__.build() "
                          "(make -C federated_multi_modal_amd/csrc)")
    h = ctypes.CDLL(path)
    h.mf_last_error.restype = ctypes.c_char_p
    h.mf_last_error.argtypes = []
    for name, args in SIGNATURES.items():
        fn = getattr(h, name)
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    _LIB = h
    return h


def exported_symbols():
    return ["mf_last_error"] + list(SIGNATURES)


def call(name: str, *args):
    h = lib()
    rc = getattr(h, name)(*args)
    if name in _VALUE_FUNCS:
        return rc
    if rc != 0:
        raise MapfedError(f"{name} failed ({rc}): {h.mf_last_error().decode(errors='replace')}")
    return rc
