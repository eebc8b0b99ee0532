"""ctypes bindings of the in-tree native libraries (see ``csrc/include/fls.h``).

``kernels()`` / ``runtime()`` raise if the library is missing — on a GPU the
HIP path must be the one that runs (no silent fallback); CPU-only code paths
call ``runtime_or_none()``.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
_KERNELS = os.path.join(HERE, "libfls_kernels.so")
_RUNTIME = os.path.join(HERE, "libfls_runtime.so")
_COMM = os.path.join(HERE, "libfls_comm.so")

_lock = threading.Lock()
_libs = {}

c_void_p, c_int, c_int64, c_uint64, c_float, c_char_p = (
    ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float, ctypes.c_char_p)


def _bind(lib, name, restype, *argtypes):
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = list(argtypes)


def _load_runtime():
    lib = ctypes.CDLL(_RUNTIME)
    _bind(lib, "fls_rt_version", c_int)
    _bind(lib, "fls_pinned_alloc", c_void_p, c_uint64)
    _bind(lib, "fls_pinned_free", c_int, c_void_p)
    _bind(lib, "fls_pinned_register", c_int, c_void_p, c_uint64)
    _bind(lib, "fls_host_device_ptr", c_void_p, c_void_p)
    _bind(lib, "fls_pinned_unregister", c_int, c_void_p)
    _bind(lib, "fls_memcpy_async", c_int, c_void_p, c_void_p, c_uint64, c_int, c_void_p)
    _bind(lib, "fls_pread_into", c_int64, c_char_p, c_uint64, c_uint64, c_void_p, c_int)
    _bind(lib, "fls_pwrite_from", c_int64, c_char_p, c_uint64, c_uint64, c_void_p, c_int, c_int)
    _bind(lib, "fls_gather_blocks", c_int, c_void_p, c_void_p, c_uint64, c_void_p, c_int64, c_int)
    _bind(lib, "fls_st_open", c_void_p, c_char_p)
    _bind(lib, "fls_st_count", c_int, c_void_p)
    _bind(lib, "fls_st_info", c_int, c_void_p, c_int, c_char_p, c_int, c_char_p, c_int,
          c_void_p, c_void_p, c_void_p, c_void_p)
    _bind(lib, "fls_st_data_offset", c_uint64, c_void_p)
    _bind(lib, "fls_st_close", None, c_void_p)
    _bind(lib, "fls_mem_info", c_int, c_void_p, c_void_p)
    _bind(lib, "fls_device_alloc", c_void_p, c_int, c_uint64)
    _bind(lib, "fls_device_free", c_int, c_int, c_void_p)
    _bind(lib, "fls_streamer_create", c_void_p, c_int, c_uint64, c_int, c_int, c_int)
    _bind(lib, "fls_streamer_pinned_bytes", c_uint64, c_void_p)
    _bind(lib, "fls_streamer_load", c_int64, c_void_p, c_char_p, c_void_p, c_int, c_void_p, c_void_p)
    _bind(lib, "fls_stream_read_host", c_int64, c_char_p, c_void_p, c_int, c_void_p, c_int)
    _bind(lib, "fls_streamer_stats", c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p)
    _bind(lib, "fls_streamer_destroy", None, c_void_p)
    _bind(lib, "fls_f32_to_f16", None, c_void_p, c_void_p, c_uint64)
    return lib


class Piece(ctypes.Structure):
    """fls_piece_t (csrc/include/fls.h)."""
    _fields_ = [("file_off", ctypes.c_uint64), ("nbytes", ctypes.c_uint64), ("dst_off", ctypes.c_uint64),
                ("kind", ctypes.c_int32), ("pad", ctypes.c_int32)]


KERNELS_ABI = 33   # bumped whenever a C signature in csrc/include/fls.h (or an accepted argument) changes


def _load_kernels(path: str = _KERNELS):
    """Load and bind a kernel library (``path``: the in-tree build, or an A/B variant build of the
    same sources, ``build.py --variant``)."""
    lib = ctypes.CDLL(path)
    _bind(lib, "fls_kernels_version", c_int)
    if lib.fls_kernels_version() != KERNELS_ABI:
        raise RuntimeError(f"{path} is a stale build (ABI {lib.fls_kernels_version()} != {KERNELS_ABI}); "
                           "rebuild with python -m flexible_llm_sharding_amd._native.build")
    _bind(lib, "fls_gemm", c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
          c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
          c_float, c_void_p, c_int, c_void_p, c_uint64, c_void_p)
    _bind(lib, "fls_rstd_from_ss", c_int, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p)
    _bind(lib, "fls_row_ss", c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p)
    _bind(lib, "fls_row_stat", c_int, c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p)
    _bind(lib, "fls_argmax_rows", c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p)
    _bind(lib, "fls_row_rstd", c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p)
    _bind(lib, "fls_fold_norm", c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p)
    _bind(lib, "fls_copy_d2d", c_int, c_void_p, c_void_p, c_uint64, c_int, c_int, c_void_p)
    _bind(lib, "fls_copy_rows", c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p)
    _bind(lib, "fls_gemm_set_splitk", c_int, c_int)
    _bind(lib, "fls_gemm_set_row_chunk", c_int, c_int)
    _bind(lib, "fls_gemm_set_mid", c_int, c_int)
    _bind(lib, "fls_gemm_set_mid_bn", c_int, c_int)
    _bind(lib, "fls_gemm_set_mid_waves", c_int, c_int)
    _bind(lib, "fls_gemm_set_mid_rows", c_int, c_int)
    _bind(lib, "fls_moe_route", c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
          c_void_p)
    _bind(lib, "fls_moe_router_route", c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
          c_int, c_void_p, c_void_p, c_void_p)
    _bind(lib, "fls_moe_plan_scratch", c_int, c_int, c_int)
    _bind(lib, "fls_moe_plan", c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
          c_void_p)
    _bind(lib, "fls_moe_gemm", c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
          c_void_p, c_void_p, c_void_p, c_int, ctypes.c_longlong, c_int, c_void_p)
    _bind(lib, "fls_moe_combine", c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
          c_int, c_int, c_void_p, c_int, c_void_p)
    _bind(lib, "fls_gemm_set_order", c_int, c_int)
    _bind(lib, "fls_gemm_set_v11", c_int, c_int)
    _bind(lib, "fls_gemm_set_v11_cost", c_int, c_int)
    _bind(lib, "fls_gemm_v11_pays", c_int, c_int, c_int)
    _bind(lib, "fls_gemm_set_skinny", c_int, c_int, c_int)
    _bind(lib, "fls_gemm_set_skinny_bn", c_int, c_int)
    _bind(lib, "fls_attention_set_hpb", c_int, c_int)
    _bind(lib, "fls_attention_set_split", c_int, c_int)
    _bind(lib, "fls_attention_set_persistent", c_int, c_int)
    _bind(lib, "fls_attention", c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
          c_int, c_int, c_float, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_uint64, c_int,
          c_void_p)
    _bind(lib, "fls_rmsnorm", c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
          c_int, c_float, c_void_p)
    _bind(lib, "fls_headnorm_rope", c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
          c_void_p, c_void_p, c_int, c_float, c_void_p)
    _bind(lib, "fls_embed", c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p)
    _bind(lib, "fls_softmax_rows", c_int, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p)
    _bind(lib, "fls_cast_f16", c_int, c_void_p, c_void_p, c_int, c_uint64, c_void_p)
    _bind(lib, "fls_gemv_skinny", c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
          c_void_p)
    _bind(lib, "fls_fill_random", c_int, c_void_p, c_uint64, c_uint64, c_float, c_float, c_void_p)
    return lib


def _load_comm():
    lib = ctypes.CDLL(_COMM)
    _bind(lib, "fls_rccl_version", c_int)
    _bind(lib, "fls_rccl_id_bytes", c_int)
    _bind(lib, "fls_rccl_unique_id", c_int, c_void_p)
    _bind(lib, "fls_rccl_init", c_void_p, c_int, c_int, c_void_p, c_int)
    _bind(lib, "fls_rccl_all_gather", c_int, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p)
    _bind(lib, "fls_rccl_all_reduce_f32", c_int, c_void_p, c_void_p, c_uint64, c_int, c_void_p)
    _bind(lib, "fls_rccl_destroy", c_int, c_void_p)
    return lib


def _get(key, path, loader, required):
    with _lock:
        if key in _libs:
            return _libs[key]
        if not os.path.exists(path):
            if required:
                raise RuntimeError(
                    f"native library {path} is missing — build it with "
                    f"`python -m flexible_llm_sharding_amd._native.build`")
            return None
        _libs[key] = loader()
        return _libs[key]


def kernels():
    return _get("k", _KERNELS, _load_kernels, True)


def runtime():
    return _get("r", _RUNTIME, _load_runtime, True)


def comm():
    """The native RCCL communicator library (csrc/comm/rccl_comm.cpp)."""
    return _get("c", _COMM, _load_comm, True)


def runtime_or_none():
    try:
        return _get("r", _RUNTIME, _load_runtime, False)
    except OSError:
        return None


def loaded_libraries():
    return {k: getattr(v, "_name", None) for k, v in _libs.items()}
