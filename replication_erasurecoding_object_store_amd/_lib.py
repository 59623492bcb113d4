"""ctypes loader for librsgpu.so (the C-ABI declared in include/rsgpu.h).

The library is built in-tree by ``__graft_entry__.build()`` (csrc/Makefile).  There
is no fallback: if the shared object is missing, :func:`lib` raises, so a product
path can never silently run anything but the HIP engine.
"""
from __future__ import annotations

import ctypes
import os
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SHIPPED_LIB_PATH = os.path.join(PKG_DIR, "librsgpu.so")
# RSGPU_LIB: load a measurement build by path instead (tools/ceiling_probe.sh runs the
# compute-free RS_PATTERN_ONLY twin this way; the shipped library is never replaced)
LIB_PATH = os.environ.get("RSGPU_LIB") or SHIPPED_LIB_PATH
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "rsgpu.h")

RS_OK = 0
RS_ERR_INV_SHARD_NUM = 1
RS_ERR_MAX_SHARD_NUM = 2
RS_ERR_TOO_FEW_SHARDS = 3
RS_ERR_SHARD_NO_DATA = 4
RS_ERR_SHARD_SIZE = 5
RS_ERR_SHORT_DATA = 6
RS_ERR_SINGULAR = 7
RS_ERR_INVALID_ARG = 16
RS_ERR_NO_DEVICE = 17
RS_ERR_DEVICE = 18
RS_ERR_NOT_SUPPORTED = 19
RS_ERR_BUSY = 20

RS_MEM_DEVICE = 0
RS_MEM_HOST = 1

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u8pp = ctypes.POINTER(_u8p)
_szp = ctypes.POINTER(ctypes.c_size_t)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_i = ctypes.c_int

# name -> (restype, argtypes); mirrors include/rsgpu.h one for one.
SIGNATURES = {
    "rs_create": (_i, [_i, _i, _i, _i, ctypes.POINTER(_vp)]),
    "rs_create_multi": (_i, [_i, _i, ctypes.c_uint64, _i, ctypes.POINTER(_vp)]),
    "rs_create_devices": (_i, [_i, _i, ctypes.POINTER(_i), _i, _i, ctypes.POINTER(_vp)]),
    "rs_device_count": (_i, [_vp]),
    "rs_device_at": (_i, [_vp, _i]),
    "rs_device_launches": (_i, [_vp, _i, ctypes.POINTER(ctypes.c_uint64)]),
    "rs_destroy": (None, [_vp]),
    "rs_data_shards": (_i, [_vp]),
    "rs_parity_shards": (_i, [_vp]),
    "rs_device": (_i, [_vp]),
    "rs_backend": (ctypes.c_char_p, [_vp]),
    "rs_strerror": (ctypes.c_char_p, [_i]),
    "rs_encode_matrix": (_i, [_vp, _u8p]),
    "rs_shard_size": (_sz, [_vp, _sz]),
    "rs_encode": (_i, [_vp, _u8pp, _szp]),
    "rs_reconstruct": (_i, [_vp, _u8pp, _szp]),
    "rs_reconstruct_data": (_i, [_vp, _u8pp, _szp]),
    "rs_verify": (_i, [_vp, _u8pp, _szp, ctypes.POINTER(_i)]),
    "rs_encode_batch": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _i, _vp]),
    "rs_reconstruct_batch": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _u32p, _sz, _i, _vp]),
    "rs_reconstruct_batch_devmask": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _vp]),
    "rs_reconstruct_batch_out": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _sz, _i, _vp, _sz, _vp]),
    "rs_reconstruct_batch_out_packed": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _i, _vp, _vp, _vp]),
    "rs_verify_batch": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _i, _vp]),
    "rs_reconstruct_batch_out_devmask": (_i, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _sz, _vp, _i, _vp, _sz, _vp]),
    "rs_sync": (_i, [_vp, _vp]),
    "rs_stream_release": (_i, [_vp, _vp]),
    "rs_sha256_batch": (_i, [_vp, _vp, _sz, _sz, _sz, _vp, _vp]),
    "rs_sha256_batch_var": (_i, [_vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    "rs_coalescer_create": (_i, [_vp, _vp, _vp]),
    "rs_coalescer_destroy": (None, [_vp]),
    "rs_co_encode": (_i, [_vp, _u8pp, _szp]),
    "rs_co_reconstruct": (_i, [_vp, _u8pp, _szp]),
    "rs_co_reconstruct_data": (_i, [_vp, _u8pp, _szp]),
    "rs_co_verify": (_i, [_vp, _u8pp, _szp, ctypes.POINTER(_i)]),
    "rs_co_stats": (_i, [_vp, _vp, _vp, _vp, _vp]),
    "rs_co_timing": (_i, [_vp, _vp, _vp, _vp, _vp]),
    "rs_co_reconstruct_many": (_i, [_vp, _sz, _u8pp, _szp, ctypes.POINTER(_i)]),
    "rs_co_encode_many": (_i, [_vp, _sz, _u8pp, _szp, ctypes.POINTER(_i)]),
    "rs_co_encode_hash": (_i, [_vp, _u8pp, _szp, _sz, _u8p]),
    "rs_co_submit_encode": (_i, [_vp, _u8pp, _szp, ctypes.c_uint64]),
    "rs_co_submit_reconstruct": (_i, [_vp, _u8pp, _szp, ctypes.c_uint64]),
    "rs_co_reap": (_i, [_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(_i), _i, _i]),
    "rs_co_encode_hash_many": (_i, [_vp, _sz, _u8pp, _szp, _szp, _u8p, ctypes.POINTER(_i)]),
    "rs_host_register": (_i, [_vp, _vp, _sz]),
    "rs_host_unregister": (_i, [_vp, _vp]),
    "rs_host_alloc": (_i, [_vp, _sz, ctypes.POINTER(_vp)]),
    "rs_host_free": (_i, [_vp, _vp]),
    "rs_last_kernel": (ctypes.c_char_p, [_vp]),
    "rs_last_kernel_on": (ctypes.c_char_p, [_vp, _vp]),
    "rs_device_copy": (_i, [_vp, _vp, _vp, _sz, _vp]),
    "rs_set_blocks_per_cu": (_i, [_vp, _i]),
    "rs_set_occupancy_cap": (_i, [_vp, _i]),
    "rs_set_parity_pad_writes": (_i, [_vp, _i]),
    "rs_set_out_pad_writes": (_i, [_vp, _i]),
    "rs_set_host_zero_copy": (_i, [_vp, _i]),
    "rs_last_host_path": (ctypes.c_char_p, [_vp]),
}

_lock = threading.Lock()
_lib = None


class LibraryMissing(RuntimeError):
    pass


def _preload_torch_hip_runtime() -> None:
    """One HIP runtime per process.  PyTorch-ROCm bundles its own libamdhip64 /
    libhsa-runtime64 (soname libamdhip64.so.7).  If librsgpu.so is loaded first its
    dependency resolves to /opt/rocm's copy, torch later maps its own, and the two
    HSA runtimes fight over the device: whichever initialises second sees no GPU
    (measured: tools/runtime_probe.py).  Loading torch's runtime first makes
    librsgpu.so's libamdhip64.so.7 dependency bind to it.  No-op without torch
    (C++/Go callers use /opt/rocm's runtime)."""
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    hip = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(hip):
        ctypes.CDLL(hip, mode=ctypes.RTLD_GLOBAL)


def lib() -> ctypes.CDLL:
    """Load librsgpu.so (raises LibraryMissing if it was not built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise LibraryMissing(
                    f"{LIB_PATH} not found: run __graft_entry__.build() (no CPU fallback exists)")
            _preload_torch_hip_runtime()
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
        return _lib


def strerror(code: int) -> str:
    return lib().rs_strerror(code).decode()
