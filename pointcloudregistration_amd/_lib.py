"""ctypes binding of libpcr.so (the C ABI declared in include/pcr_api.h).

The library is built in-tree (``pointcloudregistration_amd/libpcr.so``) by
``__graft_entry__.build()`` / ``make -C pointcloudregistration_amd/csrc``.
There is deliberately no fallback: if the HIP library is missing or fails to
load, every op raises ``PcrError`` (the product never routes through a CPU
path or the test oracle).
"""
from __future__ import annotations

import atexit
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



class RansacParams(ctypes.Structure):
    """pcr_ransac_params (include/pcr_api.h)."""
    _fields_ = [("max_correspondence_distance", _f64), ("edge_length_ratio", _f64),
                ("distance_check", _f64), ("confidence", _f64), ("max_iteration", _i32),
                ("ransac_n", _i32), ("mutual_filter", _i32), ("reserved", _i32), ("seed", _u64)]


class IcpParams(ctypes.Structure):
    """pcr_icp_params (include/pcr_api.h)."""
    _fields_ = [("max_correspondence_distance", _f64), ("relative_fitness", _f64),
                ("relative_rmse", _f64), ("max_iteration", _i32), ("reserved", _i32)]


_rp = ctypes.POINTER(RansacParams)
_ip = ctypes.POINTER(IcpParams)

# name -> argtypes (restype is always c_int); keep in sync with include/pcr_api.h
SIGNATURES = {
    "pcr_nnd_forward": [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p],
    "pcr_nnd_backward": [_p, _p, _p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p],
    "pcr_set_workspace_context": [_i32],
    "pcr_set_concurrency": [_i32],
    "pcr_nnd_forward_ragged": [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p],
    "pcr_nnd_forward_f64": [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p, _p],
    "pcr_feature_match": [_p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p, _p],
    "pcr_feature_correspondences": [_p, _p, _i32, _i32, _i32, _i32, _p, _p, _i32, _i32, _p, _p, _p, _p],
    "pcr_correspondences": [_p, _p, _i32, _i32, _i32, _p, _p, _i32, _i32, _p, _p, _p],
    "pcr_ransac_batch": [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _i32, _p, _rp, _p, _p, _p,
                         _p, _p, _p],
    "pcr_register_feature_ransac": [_p, _p, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _rp,
                                    _p, _p, _p, _p, _p, _p],
    "pcr_icp_batch": [_p, _p, _i32, _i32, _i32, _p, _p, _p, _ip, _p, _p, _p, _p, _p],
    "pcr_radius_nn": [_p, _i32, _i32, _p, _p, _i32, _p, _f64, _p, _p, _p],
    "pcr_procrustes_batch": [_p, _p, _p, _i32, _i32, _i32, _f64, _p, _p],
    "pcr_procrustes_batch_f64": [_p, _p, _p, _i32, _i32, _i32, _f64, _p, _p],
    "pcr_lrf_count": [_p, _i32, _i32, _p, _p, _i32, _p, _f64, _p, _p],
    "pcr_lrf_compute": [_p, _i32, _i32, _p, _p, _i32, _p, _f64, _i32, _p, _i32, _p, _p, _p, _p],
    "pcr_ndp_warp": [_p, _i32, _p, _i32, _i32, _i32, _i32, _p, _p, _p, _p],
    "pcr_grid_subsample": [_p, _i32, _p, _i32, _p, _i32, _f32, _i32, _p, _p, _p, _p, _p],
    "pcr_voxel_map_order": [_p, _i32, _p],
    "pcr_voxel_down_sample": [_p, _i32, _p, _i32, _f64, _p, _p, _p, _p, _p, _p, _p, _p],
    "pcr_voxel3i_map_order": [_p, _i32, _p],
    "pcr_legacy_choice_batch": [_p, _p, _p, _i32, _i32, _p],
    "pcr_vote_apply": [_p, _i32, _p, _p, _p, _i32, _f64, _p, _p, _p, _p, _i32, _p, _p],
    "pcr_radius_count": [_p, _i32, _p, _i32, _p, _p, _i32, _f32, _p, _p, _p],
    "pcr_radius_neighbors": [_p, _i32, _p, _i32, _p, _p, _i32, _f32, _i32, _p, _p, _p],
    "pcr_transform_batch": [_p, _i32, _i32, _p, _p, _p],
    "pcr_ndp_control": [_p, _p, _f64, _i32, _f64, _p],
    "pcr_adam_masked": [_p, _i32, _i32, _p, _f64, _f64, _f64, _f64, _p],
    "pcr_set_gate": [_p],
    "pcr_featmut_debug_copy": [_p, _i64, _p],
    "pcr_coop_probe": [_p, _i32, _i32, _p],
    "pcr_ndp_train_forward": [_p, _p],
    "pcr_ndp_train_backward": [_p, _p, _i32, _p, _p],
    "pcr_ndp_chamfer_glue": [_p, _i32, _p, _i32, _p, _i32, _f64, _f64, _p, _p, _p, _p, _p, _i32, _p],
    "pcr_ndp_chamfer_prepare": [_p, _p, _p],
    "pcr_ndp_chamfer_step": [_p, _p],
    "pcr_ndp_chamfer_loss": [_p, _i32, _p, _i32, _p, _i32, _f64, _f64, _p, _p, _p, _i32, _p, _f64, _i32,
                             _f64, _p, _p],
    "pcr_pipeline_step": [_p, _p, _p, _p],
    "pcr_pipeline_records": [_p, _p],
    "pcr_hybrid_search": [_p, _i32, _i32, _p, _f64, _i32, _p, _p, _p, _p],
    "pcr_estimate_normals": [_p, _i32, _i32, _p, _f64, _i32, _p, _p, _p],
    "pcr_compute_fpfh": [_p, _p, _i32, _i32, _p, _f64, _i32, _p, _p, _p, _p],
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
        lib.pcr_workspace_release.restype = ctypes.c_int
        lib.pcr_workspace_release.argtypes = []
        lib.pcr_profile_enable.restype = None
        lib.pcr_profile_enable.argtypes = [_i32]
        lib.pcr_profile_read.restype = ctypes.c_int
        lib.pcr_profile_read.argtypes = [_i32, ctypes.POINTER(_f64), ctypes.POINTER(_i64), _i32]
        lib.pcr_featnn_rescan_rows.restype = ctypes.c_int
        lib.pcr_featnn_rescan_rows.argtypes = [ctypes.POINTER(_i64), ctypes.POINTER(_i64), _i32]
        lib.pcr_featnn_fallback_rows.restype = ctypes.c_int
        lib.pcr_featnn_fallback_rows.argtypes = [ctypes.POINTER(_i64), ctypes.POINTER(_i64), _i32]
        lib.pcr_ndp_train_partial_floats.restype = _i64
        lib.pcr_ndp_train_partial_floats.argtypes = [_i32, _i32, _i32, _i32]
        lib.pcr_ndp_chamfer_scratch_bytes.restype = _i64
        lib.pcr_ndp_chamfer_scratch_bytes.argtypes = [_i32, _i32]
        lib.pcr_ndp_loss_scratch_bytes.restype = _i64
        lib.pcr_ndp_loss_scratch_bytes.argtypes = []
        lib.pcr_ndp_chamfer_gacc_words.restype = _i64
        lib.pcr_ndp_chamfer_gacc_words.argtypes = [_i32]
        lib.pcr_ndp_chamfer_max_points.restype = _i32
        lib.pcr_ndp_chamfer_max_points.argtypes = []
        lib.pcr_shutdown.restype = ctypes.c_int
        lib.pcr_shutdown.argtypes = []
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = ctypes.c_int
            fn.argtypes = args
        _lib = lib
        # free the library's device objects (workspace, profiling events) at
        # interpreter exit, before torch's and the HIP runtime's own teardown
        # (round 3 saw a crash in exit() after a profiled run)
        atexit.register(shutdown)
        return lib


def exported_symbols():
    return ["pcr_last_error", "pcr_version", "pcr_workspace_release", "pcr_profile_enable", "pcr_profile_read",
            "pcr_featnn_rescan_rows", "pcr_featnn_fallback_rows", "pcr_ndp_train_partial_floats", "pcr_ndp_chamfer_scratch_bytes",
            "pcr_ndp_loss_scratch_bytes", "pcr_ndp_chamfer_gacc_words", "pcr_ndp_chamfer_max_points",
            "pcr_shutdown"] + \
        list(SIGNATURES)


PROF_FEAT_SCREEN, PROF_NND_FWD, PROF_RANSAC_VALIDATE, PROF_ICP, PROF_RANSAC_HYP = 0, 1, 2, 3, 4
PROF_FEAT_RESCAN, PROF_FEAT_PACK, PROF_NND_GRID, PROF_FEAT_SCREEN2 = 5, 6, 7, 8
PROF_FEAT_SCREEN1B, PROF_FEAT_SCREEN2B = 9, 10   # the 3-term screens behind the 1-term ones
PROF_FEAT_REGROUP = 11   # featnn_regroup9 + featnn_finish9 (both passes)
PROF_SLOTS = 12   # pcr_internal.h kProfSlots


# bumped by every shutdown(): a HIP graph captured before it points at freed
# workspace buffers and must not be replayed (pipeline.PairPipeline re-captures)
_generation = 0


def generation():
    return _generation


def shutdown():
    """pcr_shutdown(): synchronise and free the library's per-device workspace and
    profiling events (idempotent; the library stays usable and re-allocates on
    the next call).  Graphs captured before it must not be replayed: the
    generation counter tells their owners.  Registered with atexit when the
    library is loaded."""
    global _generation
    if _lib is not None:
        _generation += 1
        _lib.pcr_shutdown()


def profile_enable(on=True):
    load().pcr_profile_enable(1 if on else 0)


def profile_read(pid, reset=True):
    """(total_ms, launches) of kernel slot `pid` since the last reset."""
    ms, cnt = _f64(0.0), _i64(0)
    rc = load().pcr_profile_read(pid, ctypes.byref(ms), ctypes.byref(cnt), 1 if reset else 0)
    if rc != PCR_OK:
        raise PcrError(load().pcr_last_error().decode())
    return ms.value, cnt.value


def featnn_rescan_rows(reset=True):
    """(rows12, rows21) sent to the exact feature-NN rescan since the last reset."""
    a, b = _i64(0), _i64(0)
    rc = load().pcr_featnn_rescan_rows(ctypes.byref(a), ctypes.byref(b), 1 if reset else 0)
    if rc != PCR_OK:
        raise PcrError(load().pcr_last_error().decode())
    return a.value, b.value


def featnn_fallback_rows(reset=True):
    """(rows12, cols21) the 1-term feature screens left to the 3-term ones since
    the last reset."""
    a, b = _i64(0), _i64(0)
    rc = load().pcr_featnn_fallback_rows(ctypes.byref(a), ctypes.byref(b), 1 if reset else 0)
    if rc != PCR_OK:
        raise PcrError(load().pcr_last_error().decode())
    return a.value, b.value


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
