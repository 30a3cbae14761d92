"""ctypes binding of ``libdl4ss_hip.so`` (the C ABI in ``include/dl4ss_hip.h``).

The product path has no CPU fallback: if the library is missing or a call
returns a non-zero ``hipError_t`` this raises ``RuntimeError`` with the HIP error
string.  Tensors are passed as raw device pointers; every call is enqueued on
torch's current HIP stream.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DL4SS_LIB", os.path.join(_HERE, "libdl4ss_hip.so"))

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
F = ctypes.c_float
U = ctypes.c_uint

# name -> argtypes (all return int hipError_t)
SIGNATURES = {
    "dl4ss_stft_fwd": [P, LL, I, I, I, I, P, P, P],
    "dl4ss_stft_fwd_ex": [P, LL, I, I, I, I, P, P, P, LL, LL, P],
    "dl4ss_istft": [P, LL, I, I, I, I, P, P],
    "dl4ss_mix_sources": [P, P, I, I, I, P, P, P, P],
    "dl4ss_gemm": [I, I, I, I, I, P, LL, P, LL, P, LL, P, I, F, I, I, P],
    "dl4ss_f32_to_bf16": [P, P, LL, P],
    "dl4ss_f32_to_bf16_2d": [P, LL, I, I, P, LL, P],
    "dl4ss_f32_to_bf16_hilo": [P, LL, I, I, P, LL, I, I, U, P],
    "dl4ss_birnn_bias_reduce": [I, I, I, I, P, P, P, P],
    "dl4ss_birnn_bias_reduce_ex": [I, I, I, I, P, P, P, F, P],
    "dl4ss_colsum_bf16": [P, LL, I, I, P, P],
    "dl4ss_colsum_bf16_part_bytes": [I, I],
    "dl4ss_colsum_bf16_det": [P, LL, I, I, P, P, LL, P],
    "dl4ss_colsum_bf16_det_ex": [P, LL, I, I, P, P, LL, F, P],
    "dl4ss_gemm_bf16_gl_ws_bytes": [I, I, I, I, I],
    "dl4ss_gemm_gl_set_config": [I],
    "dl4ss_gemm_bf16_gl": [I, I, I, I, I, P, LL, P, LL, P, LL, P, I, F, I, I, LL, LL, LL, P, LL, P],
    "dl4ss_gemm_bf16_gl_grouped_ws_bytes": [I, P, P, P, P],
    "dl4ss_gemm_bf16_gl_grouped": [I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, LL, P],
    "dl4ss_gemm_bf16_gl_grouped_ex": [I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, LL, I, I, I, P, P],
    "dl4ss_birnn_fwd_ex": [I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, LL, P, P],
    "dl4ss_birnn_fwd_xw": [I, I, I, I, P, I, LL, P, LL, P, P, P, P, P, P, P, P, P, P, LL, P, P, I],
    "dl4ss_birnn_fwd_mean": [I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, LL, P, P],
    "dl4ss_birnn_fwd_xw_ex": [I, I, I, I, P, I, LL, P, LL, P, P, P, P, P, P, P, P, P, P, P, LL, P, P, I],
    "dl4ss_birnn_fwd_xw_supported": [I, I, I, I, I],
    "dl4ss_birnn_bwd_ex": [I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, LL, P, P],
    "dl4ss_mask_attn_loss_ex": [I, I, I, I, I, I, I, P, P, P, LL, P, LL, LL, P, F, F, P, P, LL, P, P, P, P, P],
    "dl4ss_birnn_workspace_bytes": [I, I, I],
    "dl4ss_birnn_fwd": [I, I, I, I, I, P, P, P, P, P, P, P, P, LL, P, P],
    "dl4ss_birnn_bwd": [I, I, I, I, I, P, P, P, P, P, P, P, P, P, LL, P, P],
    "dl4ss_attn_nblk": [I, I],
    "dl4ss_mask_attn_loss": [I, I, I, I, I, I, I, P, P, P, LL, P, LL, LL, P, F, F, P, P, P, P, P, P],
    "dl4ss_pit_select": [P, I, I, I, P, P],
    "dl4ss_loss_finalize": [P, I, I, I, P, F, F, P, P, I, P, P],
    "dl4ss_query_fwd": [P, I, I, I, P, P, P, I, I, P, P, P],
    "dl4ss_query_bwd": [P, I, I, I, P, P, P, P, I, I, P, P, P, P],
    "dl4ss_query_bwd_ex": [P, I, I, I, P, P, P, P, I, I, P, P, P, I, F, P],
    "dl4ss_colsum": [P, LL, I, I, P, P],
    "dl4ss_adam": [P, P, P, P, LL, F, F, F, F, I, P],
    "dl4ss_istft_apply": [P, P, LL, I, I, I, I, P, P],
    "dl4ss_tanh_bwd": [P, P, P, LL, P],
    "dl4ss_attn_dot_nblk": [I],
    "dl4ss_attn_dot_fwd": [P, P, I, I, I, I, I, P, P],
    "dl4ss_attn_dot_bwd": [P, P, I, P, P, I, I, I, I, P, P, P, P],
    "dl4ss_top_k_mask": [P, I, I, F, I, P, P, P, P],
    "dl4ss_attn_dot_fwd_ex": [P, P, I, I, I, I, I, P, LL, P],
    "dl4ss_classifier_select": [P, I, I, F, I, P, I, P, P, P, P],
    "dl4ss_mask_split": [P, P, LL, P, P, P],
    "dl4ss_time_mean": [P, I, I, I, P, P],
    "dl4ss_bss_corr": [P, I, I, I, I, P, P],
    "dl4ss_mix_sources_ex": [P, P, P, I, I, I, P, P, P, P],
    "dl4ss_mix_sources_rot": [P, P, P, P, I, I, I, P, P, P, P],
    "dl4ss_f32_to_bf16_2d_multi": [I, P, P, P, P, P, P, P],
    "dl4ss_mask_attn_loss_bf16v": [I, I, I, I, I, I, I, P, P, P, LL, P, LL, LL, P, F, F, P, P, LL, P, P, P, P, P],
    "dl4ss_bss_gram": [P, I, I, I, I, P, P, P, P],
    "dl4ss_adam_guarded": [P, P, P, P, LL, F, F, F, F, I, P, P, P],
    "dl4ss_adam_guarded_dp": [P, P, P, P, LL, F, F, F, F, I, P, P, P, P],
    "dl4ss_adam_guarded_dp_scaled": [P, P, P, P, LL, F, F, F, F, I, P, P, F, P, P],
    "dl4ss_adam_guarded_dp_scaled_bf16": [P, P, P, P, LL, F, F, F, F, I, P, P, F, P, I, P, P, P, P, P, P],
    "dl4ss_status_flag": [P, P, P],
    "dl4ss_birnn_plan_info": [I, I, I, I, I, P],
    "dl4ss_debug_set_spin_limit": [ctypes.c_uint],
    "dl4ss_debug_set_place_force": [ctypes.c_int],
    "dl4ss_debug_set_rnn_max_wg": [ctypes.c_int],
}
# entry points that return a value rather than a hipError_t
RESTYPES = {"dl4ss_birnn_workspace_bytes": ctypes.c_longlong, "dl4ss_colsum_bf16_part_bytes": ctypes.c_longlong,
            "dl4ss_gemm_bf16_gl_ws_bytes": ctypes.c_longlong,
            "dl4ss_gemm_bf16_gl_grouped_ws_bytes": ctypes.c_longlong, "dl4ss_attn_nblk": ctypes.c_int,
            "dl4ss_attn_dot_nblk": ctypes.c_int, "dl4ss_debug_set_spin_limit": None,
            "dl4ss_debug_set_place_force": None, "dl4ss_debug_set_rnn_max_wg": None}

_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"dl4ss HIP library not found at {LIB_PATH}; run `python -m dl4ss_amd.build` "
            "(there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = RESTYPES.get(name, ctypes.c_int)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipGetErrorString.restype = ctypes.c_char_p
    hip.hipGetErrorString.argtypes = [ctypes.c_int]
    lib._hip = hip
    _lib = lib
    return lib


def lib():
    return _load()


def exported_symbols():
    return list(SIGNATURES)


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t, strided=False):
    """Raw device pointer of a CUDA tensor.  Unless the call site passes the
    strides itself (``strided=True``), the tensor must be contiguous: a kernel
    sees only the pointer, so a transposed view would be silently misread."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("dl4ss HIP op received a CPU tensor (no CPU fallback)")
    if not strided and not t.is_contiguous():
        raise RuntimeError("dl4ss HIP op received a non-contiguous tensor")
    return ctypes.c_void_p(t.data_ptr())


def query(name, *args):
    """Call an entry point that returns a value (sizes), not an error code."""
    return getattr(_load(), name)(*args)


def call(name, *args):
    lb = _load()
    rc = getattr(lb, name)(*args)
    if rc != 0:
        msg = lb._hip.hipGetErrorString(rc).decode()
        raise RuntimeError(f"{name} failed: hipError {rc} ({msg})")
    return rc
