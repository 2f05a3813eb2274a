"""ctypes binding of libpcr.so (the C ABI declared in include/pcr_api.h).

The library is built in-tree (``pointcloudregistration_amd/libpcr.so``) by
``__graft_entry__.build()`` / ``make -C pointcloudregistration_amd/csrc``.
There is deliberately no fallback: if the HIP library is missing or fails to
load, every op raises ``PcrError`` (the product never routes through a CPU
path or the test oracle).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PCR_LIB", os.path.join(_HERE, "libpcr.so"))

PCR_OK = 0


class PcrError(RuntimeError):
    """Raised when libpcr is unavailable or a libpcr call fails."""


_lib = None
_lock = threading.Lock()

_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_f64 = ctypes.c_double
_u64 = ctypes.c_uint64

# name -> argtypes (restype is always c_int); keep in sync with include/pcr_api.h
SIGNATURES = {
    "pcr_nnd_forward": [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p],
    "pcr_nnd_backward": [_p, _p, _p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p],
}


def load():
    """Load libpcr.so once; raise PcrError (no fallback) if it cannot be loaded."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise PcrError(
                f"libpcr.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` or "
                "`make -C pointcloudregistration_amd/csrc`")
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the box
            raise PcrError(f"failed to load {LIB_PATH}: {e}") from e
        lib.pcr_last_error.restype = ctypes.c_char_p
        lib.pcr_last_error.argtypes = []
        lib.pcr_version.restype = ctypes.c_int
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = ctypes.c_int
            fn.argtypes = args
        _lib = lib
        return lib


def exported_symbols():
    return ["pcr_last_error", "pcr_version"] + list(SIGNATURES)


def call(name, *args):
    """Call a libpcr entry point; raise PcrError with pcr_last_error() on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != PCR_OK:
        msg = lib.pcr_last_error().decode("utf-8", "replace")
        raise PcrError(f"{name} failed ({rc}): {msg}")
    return rc


def stream_handle(device=None):
    """hipStream_t of torch's current stream on `device` (0 = legacy default)."""
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
