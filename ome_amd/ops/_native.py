"""ctypes binding of the in-tree HIP kernel library (``ome_amd/_lib/libome_kernels.so``).

Every launcher has the C signature ``int ome_xxx(..., hipStream_t)``; a non-zero return is a
HIP error code (or a negative argument-check code) and is raised as :class:`NativeError`.

Policy (the round contract): on a GPU the native path is mandatory — if the
library is missing we raise, we never fall back to eager PyTorch silently.  CPU tensors use
the reference implementations in :mod:`ome_amd.ops.reference` (that is how the engine and the
scheduler are tested without a GPU).
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

# OME_LIB_DIR: load the native libraries from another in-tree directory (compiler-flag A/B runs,
# scripts/build_variant.py); default ome_amd/_lib
# (a library missing there comes from the default directory)
_LIB_DIR = Path(__file__).resolve().parent.parent / "_lib"
_LIB_OVERRIDE = Path(os.environ["OME_LIB_DIR"]).resolve() if os.environ.get("OME_LIB_DIR") else None
_lock = threading.Lock()
_libs: dict[str, C.CDLL] = {}

vp, i32, i64, f32, u64 = C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_uint64

_SIGNATURES = {
    "ome_kernels": {
        "ome_rmsnorm": [vp, i64, vp, vp, i64, i32, i32, f32, vp],
        "ome_fused_add_rmsnorm": [vp, i64, vp, i64, vp, i32, i32, f32, vp],
        "ome_norm_set_threads": [i32],
        "ome_copy_mapped": [vp, vp, i64, vp],
        "ome_host_device_ptr": [vp, vp],
        "ome_rope_set_split": [i32],
        # KV-cache ops end in (kv_fmt, k_scale, v_scale, stream)
        "ome_rope_qkv_cache": [vp, i64, vp, vp, i32, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, f32,
                               i32, f32, f32, vp],
        "ome_kv_cache_write": [vp, vp, i64, vp, vp, vp, i32, i32, i32, i32, i32, f32, f32, vp],
        "ome_act_and_mul": [vp, vp, i64, i32, i32, vp],
        "ome_act": [vp, i64, i32, vp],
        "ome_ssm_conv1d": [vp, i64, vp, vp, vp, i64, vp, vp, vp, vp, i32, i32, i32, vp],
        "ome_dyn_conv1d": [vp, i64, vp, i64, i32, vp, i64, vp, vp, vp, vp, i32, i32, i32, vp],
        "ome_qk_norm_rope": [vp, i64, vp, vp, i32, i32, i32, f32, vp, i64, vp, vp],
        "ome_ssm_scan": [vp, i64, vp, i64, vp, vp, i64, vp, vp, vp, f32, vp, vp, i64, vp, vp, vp, i32, i32, i32,
                         i32, i32, vp],
        "ome_gdn_scan": [vp, vp, vp, i64, vp, vp, i64, vp, vp, vp, vp, i64, vp, vp, vp, i32, i32, i32, i32, i32,
                         i32, vp, vp],
        "ome_gated_rmsnorm": [vp, i64, vp, i64, vp, vp, i64, i32, i32, i32, f32, i32, vp],
        "ome_layernorm": [vp, i64, vp, i64, vp, vp, vp, i64, i32, i32, f32, vp],
        "ome_embedding": [vp, vp, vp, i32, i32, i32, i32, vp],
        "ome_pool": [vp, vp, vp, i32, i32, i32, i32, vp],
        "ome_fill_pending": [vp, vp, vp, i32, vp],
        "ome_apply_penalties": [vp, i32, i64, i32, i32, vp, i64, vp, vp, vp, vp, vp],
        "ome_update_counts": [vp, i64, vp, vp, vp, vp, vp, i32, vp],
        "ome_moe_route": [vp, i32, i64, i32, i32, i32, i32, i32, vp, i32, i32, i32, vp, vp, vp],
        "ome_mla_attn": [vp, i64, vp, vp, i32, vp, vp, i32, i32, i32, i32, f32, i32, vp, i64, vp, vp, vp],
        "ome_moe_align": [vp, i32, i32, vp, vp, vp, vp],
        "ome_moe_gemm": [vp, i64, vp, i32, vp, vp, i32, i32, i32, i32, vp, i64, vp, i32, vp],
        "ome_moe_gemm_fp8": [vp, i64, vp, vp, i32, vp, vp, vp, i32, i32, i32, i32, vp, i64, vp],
        "ome_moe_gemm_fp8_tile": [vp, i64, vp, vp, i32, vp, vp, vp, i32, i32, i32, i32, i32, vp, i64, vp],
        "ome_moe_combine": [vp, vp, vp, i32, i32, i32, vp, f32, vp],
        "ome_moe_combine_add": [vp, vp, vp, i32, i32, i32, vp, vp, f32, vp],
        "ome_paged_decode": [vp, i64, vp, vp, vp, i32, vp, vp, i64, vp, vp, i32, i32, i32, i32, i32, i32, i32, f32,
                             i32, vp, i32, f32, f32, f32, vp, vp, vp, i64, vp],
        "ome_paged_prefill": [vp, i64, vp, vp, vp, i32, vp, vp, vp, i32, vp, i64, i32, i32, i32, i32, f32, i32,
                              i32, f32, f32, f32, vp, vp, vp, i32, i64, vp],
        "ome_paged_prefill_split": [vp, i64, vp, vp, vp, i32, vp, vp, vp, i32, vp, i32, i32, vp, vp, vp, i64, i32,
                                    i32, f32, i32, i32, f32, f32, f32, vp, vp, i64, vp],
        "ome_varlen_attention": [vp, i64, vp, i64, vp, i64, vp, vp, vp, i32, vp, i64, i32, i32, i32, f32, i32, vp],
        "ome_skinny_gemm": [vp, i64, vp, vp, vp, i64, i32, i32, i32, i32, vp, vp, vp],
        "ome_w8a16_gemm": [vp, i64, vp, i64, vp, i32, vp, vp, i64, i32, i32, i32, i32, vp, vp, vp],
        "ome_w8a16_mgemv": [vp, i64, vp, i64, vp, i32, vp, vp, i64, i32, i32, i32, i32, vp, vp, vp],
        "ome_stream_gemm": [vp, i64, vp, vp, vp, i64, i32, i32, i32, i32, i32, vp, vp, vp],
        "ome_gemv": [vp, i64, vp, vp, vp, i64, i32, i32, i32, vp],
        "ome_gemv_act": [vp, i64, vp, vp, vp, i64, i32, i32, i32, vp],
        "ome_gemm": [vp, i64, vp, i64, vp, i64, i32, i32, i32, i32, i32, vp, vp],
        "ome_gemm_set_variant": [i32],
        "ome_gemm_sk": [vp, i64, vp, i64, vp, vp, i64, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp],
        "ome_gemm_pp": [vp, i64, vp, i64, vp, vp, i64, vp, i64, i32, i32, i32, i32, vp],
        "ome_gemm_xl": [vp, i64, vp, i64, vp, vp, i64, i32, i32, i32, i32, i32, i32, vp, vp, i32, vp],
        "ome_mla_prep": [vp, i64, i32, i32, i32, vp, f32, vp, vp, vp, vp, i64, vp, i64, i64, i32, i32, vp, i64, i64,
                         i32, vp],
        "ome_gemm_sk_fp8": [vp, i64, vp, vp, i64, vp, i32, vp, vp, i64, i32, i32, i32, i32, i32, i32, i32, vp, vp,
                            vp],
        "ome_fp8_gemm_mx": [vp, i64, vp, vp, i64, vp, i32, i32, i32, i32, vp, i64, vp, vp],
        "ome_fp8_quant": [vp, i64, i32, i32, vp, vp, i32, vp],
        "ome_fp8_gemm": [vp, i64, vp, vp, vp, i32, i32, i32, i32, vp, i64, vp, vp],
        "ome_sample": [vp, i32, i64, i32, i32, vp, vp, vp, vp, vp, u64, vp, vp, vp],
    },
    "ome_comm": {
        "ome_comm_create": [i32, i32, C.c_size_t, C.POINTER(vp), vp, vp],
        "ome_comm_handle_size": [],
        "ome_comm_open": [vp, vp, vp],
        "ome_comm_all_reduce": [vp, vp, vp, i64, i32, i32, vp],
        "ome_comm_all_reduce_add_rmsnorm": [vp, vp, vp, vp, vp, i32, i32, f32, i32, vp],
        "ome_comm_all_gather": [vp, vp, vp, i64, i64, i32, vp],
        "ome_comm_error": [vp],
        "ome_comm_host_error": [vp],
        "ome_comm_set_fault": [vp, C.c_uint32],
        "ome_comm_destroy": [vp],
        "ome_ep_create": [i32, i32, i32, i32, C.POINTER(vp), vp, vp],
        "ome_ep_open": [vp, vp, vp],
        "ome_ep_dispatch": [vp, vp, i64, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp, vp],
        "ome_ep_combine": [vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, vp, i64, vp],
        "ome_ep_error": [vp],
        "ome_ep_host_error": [vp],
        "ome_ep_set_fault": [vp, C.c_uint32],
        "ome_ep_destroy": [vp],
        "ome_kvlink_export": [vp, vp, C.POINTER(i64)],
        "ome_kvlink_handle_size": [],
        "ome_kvlink_open": [vp, C.POINTER(vp)],
        "ome_kvlink_close": [vp],
        "ome_kvlink_copy": [vp, vp, vp, vp, i32, i32, i64, i64, vp],
    },
}


class NativeError(RuntimeError):
    pass


def lib_path(name: str = "ome_kernels") -> Path:
    if _LIB_OVERRIDE is not None and (_LIB_OVERRIDE / f"lib{name}.so").exists():
        return _LIB_OVERRIDE / f"lib{name}.so"
    return _LIB_DIR / f"lib{name}.so"


def load(name: str = "ome_kernels") -> C.CDLL:
    """Load (once) an in-tree native library; raise if it was not built."""
    lib = _libs.get(name)
    if lib is not None:
        return lib
    with _lock:
        if name in _libs:
            return _libs[name]
        path = lib_path(name)
        if not path.exists():
            if os.environ.get("OME_AUTOBUILD", "1") == "1":
                from ome_amd import build as _b

                _b.build(verbose=False)
            if not path.exists():
                raise NativeError(f"{path} missing — run `python -m ome_amd.build` (hipcc, gfx950)")
        lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
        for fn, argt in _SIGNATURES.get(name, {}).items():
            f = getattr(lib, fn)
            f.argtypes = argt
            f.restype = C.c_int
        _libs[name] = lib
        return lib


def available(name: str = "ome_kernels") -> bool:
    try:
        load(name)
        return True
    except (NativeError, OSError):
        return False


def call(fn: str, *args, lib: str = "ome_kernels") -> None:
    rc = getattr(load(lib), fn)(*args)
    if rc != 0:
        raise NativeError(f"{fn} failed with code {rc}")


def stream_ptr(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()
