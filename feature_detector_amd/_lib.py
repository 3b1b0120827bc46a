"""ctypes binding of libfdhip.so (include/fd_hip.h). No fallback: a missing library raises."""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.environ.get("FD_LIB_PATH") or os.path.join(LIB_DIR, "libfdhip.so")  # (override: A/B of builds)
CSRC = os.path.join(HERE, "csrc")

FD_OK, FD_ERR_INVALID, FD_ERR_HIP, FD_ERR_CAPACITY = 0, 1, 2, 3
FD_HARRIS, FD_SHI_TOMASI, FD_FAST = 0, 1, 2
ABI_VERSION = 6  # include/fd_hip.h FD_ABI_VERSION this binding's signatures follow

# Every symbol include/fd_hip.h declares (checked by tests/test_capi_symbols.py).
EXPORTS = (
    "fd_ctx_create", "fd_ctx_destroy", "fd_last_error", "fd_ctx_set_stream", "fd_ctx_use_own_stream",
    "fd_ctx_get_stream",
    "fd_ctx_synchronize", "fd_ctx_reserve", "fd_ctx_stage", "fd_ctx_set_tie_order", "fd_ctx_frame_status", "fd_points_detect", "fd_points_candidates", "fd_points_response",
    "fd_points_response_append", "fd_points_select",
    "fd_lsd_map", "fd_lsd_map_pitched", "fd_lsd_lines", "fd_lsd_lines_state", "fd_brief_compute", "fd_nn_select", "fd_nn_select_list", "fd_nn_descriptors",
    "fd_nn_bias_relu", "fd_nn_conv3x3_c1", "fd_nn_conv3x3_c64",
    "fd_nn_heat_softmax", "fd_nn_desc_normalize",
    "fd_build_info", "fd_abi_version", "fd_png_info", "fd_png_decode", "fd_png_frames",
    "fd_ingest_create", "fd_ingest_destroy", "fd_ingest_frames", "fd_ingest_submit", "fd_ingest_wait",
)


class FdError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libfdhip error {code}: {msg}")
        self.code = code


class fd_point_opts(ctypes.Structure):
    _fields_ = [("min_feature_distance", ctypes.c_int32), ("min_valid_response", ctypes.c_float)]


FD_SAMPLE_BILINEAR, FD_SAMPLE_TRUNCATE = 0, 1


class fd_nn_opts(ctypes.Structure):
    _fields_ = [("invalid_boundary", ctypes.c_int32), ("min_feature_distance", ctypes.c_int32),
                ("max_features", ctypes.c_int32), ("min_response", ctypes.c_float), ("max_response", ctypes.c_float)]


class fd_lsd_opts(ctypes.Structure):
    _fields_ = [("min_valid_gradient_norm", ctypes.c_float), ("min_tolerance_angle_residual_rad", ctypes.c_float),
                ("min_valid_line_length", ctypes.c_float), ("max_tolerance_inlier_ratio", ctypes.c_float)]


# fd_lsd_rect as 12 floats: start x, y, end x, y, center x, y, length, width, angle, dir x, y, inlier ratio
LSD_RECT_FLOATS = 12


class fd_brief_opts(ctypes.Structure):
    _fields_ = [("length", ctypes.c_int32), ("half_patch_size", ctypes.c_int32), ("sampler", ctypes.c_int32)]


_lib = None


def load() -> ctypes.CDLL:
    """Load libfdhip.so from the package's lib/ directory (built by __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                          f"or `make -C {CSRC}`; there is no CPU fallback")
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64 (soname libamdhip64.so.7,
    # the same as /opt/rocm's). Loading torch first makes libfdhip bind to that copy, so device
    # pointers, streams and events are shared with torch; without torch, /opt/rocm's runtime is used.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P, i32, i64, u32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32, ctypes.c_float
    sig = {
        "fd_ctx_create": (i32, [i32, ctypes.POINTER(P)]),
        "fd_ctx_destroy": (None, [P]),
        "fd_last_error": (ctypes.c_char_p, [P]),
        "fd_ctx_set_stream": (i32, [P, P]),
        "fd_ctx_use_own_stream": (i32, [P]),
        "fd_ctx_get_stream": (P, [P]),
        "fd_ctx_synchronize": (i32, [P]),
        "fd_ctx_reserve": (i32, [P, i32, i32, i32, i32, i64]),
        "fd_ctx_stage": (i32, [P, P, i64, ctypes.POINTER(P)]),
        "fd_ctx_set_tie_order": (i32, [P, i32]),
        "fd_ctx_frame_status": (i32, [P, P, i32, i32]),
        "fd_points_detect": (i32, [P, i32, P, i32, i32, i32, i32, ctypes.POINTER(fd_point_opts), P, P, u32, P, i32,
                                   P, i32]),
        "fd_points_candidates": (i32, [P, i32, P, i32, i32, i32, i32, ctypes.POINTER(fd_point_opts), P, P, P, P, P,
                                       i64, P, P, i32]),
        "fd_points_select": (i32, [P, i32, i32, i32, ctypes.POINTER(fd_point_opts), P, P, P, P, i64, i32, P, P, u32,
                                   P, i32, P, i32]),
        "fd_points_response": (i32, [P, i32, P, i32, i32, i32, ctypes.POINTER(fd_point_opts), P, P, i64, P]),
        "fd_points_response_append": (i32, [P, i32, P, i32, i32, i32, ctypes.POINTER(fd_point_opts), P, P, i64, P]),
        "fd_lsd_map": (i32, [P, P, i32, i32, i32, i32, f32, P, P, P, P, i64, P, i32]),
        "fd_lsd_map_pitched": (i32, [P, P, i32, i32, i32, i32, f32, P, P, P, i64, P, i64, P, i32]),
        "fd_lsd_lines": (i32, [P, P, i32, i32, i32, i32, ctypes.POINTER(fd_lsd_opts), u32, P, i32, P, i32]),
        "fd_lsd_lines_state": (i32, [P, P, P, P, P, i64, P]),
        "fd_brief_compute": (i32, [P, P, i32, i32, i32, i32, ctypes.POINTER(fd_brief_opts), P, P, i32, P, P, i32]),
        "fd_nn_select": (i32, [P, P, i32, i32, i32, i32, ctypes.POINTER(fd_nn_opts), P, P, P, i32, P, i32]),
        "fd_nn_select_list": (i32, [P, P, P, P, i64, i32, i32, i32, i32, ctypes.POINTER(fd_nn_opts), P, P, P, i32, P,
                                    P, i32, P, i32]),
        "fd_nn_descriptors": (i32, [P, P, i32, i32, i32, i32, i32, i32, P, P, i32, P, i32]),
        "fd_nn_bias_relu": (i32, [P, P, P, i64, P, i32, i32, i32, i32, i32]),
        "fd_nn_conv3x3_c1": (i32, [P, P, P, P, i64, P, i32, i32, i32]),
        "fd_nn_heat_softmax": (i32, [P, P, P, P, i32, i32, i32]),
        "fd_nn_desc_normalize": (i32, [P, P, P, P, i64, i32]),
        "fd_nn_conv3x3_c64": (i32, [P, P, P, P, P, i32, i32, i32, i32, i32, i32]),
        "fd_build_info": (ctypes.c_char_p, []),
        "fd_abi_version": (i32, []),
        "fd_png_info": (i32, [P, ctypes.c_size_t, P, P, P]),
        "fd_png_decode": (i32, [P, ctypes.c_size_t, P, ctypes.c_size_t, P, P]),
        "fd_png_frames": (i32, [P, P, P, i32, i32, i32, P, i32]),
        "fd_ingest_create": (i32, [P, i32, i32, i32, i32, i32, u32, i32, ctypes.POINTER(P)]),
        "fd_ingest_destroy": (None, [P]),
        "fd_ingest_frames": (P, [P, i32]),
        "fd_ingest_submit": (i32, [P, i32, ctypes.POINTER(fd_point_opts)]),
        "fd_ingest_wait": (i32, [P, i32, ctypes.POINTER(P), ctypes.POINTER(P)]),
    }
    for name, (res, args) in sig.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            if os.environ.get("FD_LIB_PATH"):  # an older build under A/B: its missing entry points stay unbound
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    abi = L.fd_abi_version() if hasattr(L, "fd_abi_version") or not os.environ.get("FD_LIB_PATH") else ABI_VERSION
    if abi != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has C ABI version {abi}, this binding needs {ABI_VERSION}: rebuild the library")
    _lib = L
    return L


def check(ctx_ptr, rc: int) -> None:
    if rc != FD_OK:
        msg = load().fd_last_error(ctx_ptr)
        raise FdError(rc, msg.decode() if msg else "")
