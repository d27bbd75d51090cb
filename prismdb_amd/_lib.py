"""Loader for the in-tree native library (prismdb_amd/lib/libprismdb_crc32c.so).

There is no fallback: if the library is missing or fails to load, every entry
point raises.  torch is imported first (when installed) so that the library
binds to the HIP runtime torch already loaded (both carry SONAME
libamdhip64.so.7) instead of pulling in a second copy.
"""
from __future__ import annotations

import ctypes
import os
import threading

# PRISMDB_LIB: measurement tools (PMC runs of a variant build) may point the
# package at another build of the same library; unset, the in-tree product.
LIB_PATH = os.environ.get("PRISMDB_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                           "libprismdb_crc32c.so")

# Every symbol include/prismdb_crc32c.h and include/prismdb_synth.h declare.
C_ABI_SYMBOLS = (
    "leveldb_crc32c_extend",
    "leveldb_crc32c_value",
    "leveldb_crc32c_mask",
    "leveldb_crc32c_unmask",
    "leveldb_crc32c_combine",
    "leveldb_crc32c_accelerated",
    "leveldb_crc32c_device_init",
    "leveldb_crc32c_batch_fixed",
    "leveldb_crc32c_batch",
    "leveldb_crc32c_batch_host",
    "leveldb_crc32c_batch_multi",
    "leveldb_crc32c_last_error",
    "prismdb_fill_synthetic",
    "leveldb_sst_block_spans",
    "leveldb_sst_last_error",
    "leveldb_log_scan",
    "leveldb_log_replay",
    "leveldb_log_reason",
)
# The C++ surface (util/crc32c.h): crc32c::Extend(uint32_t, const char*, size_t).
CXX_EXTEND_SYMBOL = "_ZN7leveldb6crc32c6ExtendEjPKcm"

_lock = threading.Lock()
_lib = None


class NativeLibraryError(RuntimeError):
    pass


def _declare(lib: ctypes.CDLL) -> None:
    u32, u64, sz, vp, cp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p
    sig = {
        "leveldb_crc32c_extend": (u32, [u32, cp, sz]),
        "leveldb_crc32c_value": (u32, [cp, sz]),
        "leveldb_crc32c_mask": (u32, [u32]),
        "leveldb_crc32c_unmask": (u32, [u32]),
        "leveldb_crc32c_combine": (u32, [u32, u32, u64]),
        "leveldb_crc32c_accelerated": (ctypes.c_int, []),
        "leveldb_crc32c_device_init": (ctypes.c_int, [ctypes.c_int]),
        "leveldb_crc32c_batch_fixed": (ctypes.c_int, [vp, sz, sz, sz, u32, vp, vp, u32, vp]),
        "leveldb_crc32c_batch": (ctypes.c_int, [vp, vp, vp, vp, sz, vp, vp, u32, vp]),
        "leveldb_crc32c_batch_host": (ctypes.c_int, [vp, vp, vp, vp, sz, vp, vp, u32]),
        "leveldb_crc32c_batch_multi": (ctypes.c_int, [ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, u32, vp]),
        "leveldb_crc32c_last_error": (ctypes.c_char_p, []),
        "prismdb_fill_synthetic": (ctypes.c_int, [vp, sz, u64, u64, vp]),
        "prismdb_crc32c_extend_portable": (u32, [u32, cp, sz]),
        # test hooks (not in the public headers): path pinning -- the setters
        # act only with PRISMDB_ENABLE_TEST_HOOKS=1 in the environment
        "prismdb_crc32c_force_generic": (None, [ctypes.c_int]),
        "prismdb_crc32c_lane_mode": (None, [ctypes.c_int]),
        "prismdb_crc32c_direct_max": (u64, [u64]),
        "prismdb_crc32c_last_split": (ctypes.c_int, [vp]),
        "prismdb_crc32c_last_schedule": (ctypes.c_int, [vp]),
        "prismdb_pipeline_chunk_bytes": (ctypes.c_size_t, [ctypes.c_size_t]),
        "prismdb_crc32c_direct_tickets": (u32, [u32]),
        "prismdb_crc32c_direct_debug": (u32, [u32]),
        "prismdb_crc32c_direct_stats": (ctypes.c_int, [vp]),
        "prismdb_crc32c_direct_set_gen": (ctypes.c_int, [vp, u32]),
        "prismdb_crc32c_multi_fail_after": (ctypes.c_int, [ctypes.c_int]),
        "prismdb_crc32c_windows": (ctypes.c_int, [ctypes.c_int]),
        "prismdb_crc32c_multi_timing": (ctypes.c_int, [ctypes.c_int, vp, vp, vp, vp]),
        "prismdb_crc32c_multi_host_timing": (ctypes.c_int, [ctypes.c_int, vp, vp, vp, vp]),
        "prismdb_crc32c_multi_self_gather": (ctypes.c_int, [ctypes.c_int]),
        "prismdb_crc32c_last_claims": (ctypes.c_int, [vp]),
        "prismdb_test_hooks_enabled": (ctypes.c_int, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib() -> ctypes.CDLL:
    """The loaded native library (loads on first use; raises if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            try:
                import torch  # noqa: F401  (bind to torch's HIP runtime first)
            except ImportError:
                pass
            if not os.path.exists(LIB_PATH):
                raise NativeLibraryError(
                    f"{LIB_PATH} is missing: build it with `python -m prismdb_amd.build` "
                    "(the MI355X engine has no CPU fallback)")
            try:
                handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            except OSError as e:
                raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
            _declare(handle)
            _lib = handle
    return _lib


def last_error() -> str:
    msg = lib().leveldb_crc32c_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise NativeLibraryError(f"{what} failed ({rc}): {last_error()}")
