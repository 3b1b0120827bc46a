"""MI355X-native feature-detection hot path (Horizon1026/Feature_Detector drop-in for its per-pixel stages).

Layers:
  include/fd_hip.h          C ABI (libfdhip.so: gfx950 HIP kernels + runtime)
  include/feature_detector/ C++ classes with the reference's API (libfeature_detector.so)
  feature_detector_amd      Python batch API over the C ABI (this package), used by tests and bench.py
"""
from ._lib import FD_FAST, FD_HARRIS, FD_SHI_TOMASI, FdError, LIB_PATH, load  # noqa: F401
from .points import Context, DetectResult, default_context, detect_points, lsd_lines, lsd_map, point_candidates, point_response, select_points  # noqa: F401
from .descriptor import brief_compute, to_float, unpack_bits  # noqa: F401
from .ingest import Ingest, load_png, png_frames, png_info  # noqa: F401

__all__ = [
    "FD_HARRIS", "FD_SHI_TOMASI", "FD_FAST", "FdError", "Context", "DetectResult", "default_context",
    "detect_points", "point_candidates", "point_response", "select_points", "lsd_map", "lsd_lines", "load", "brief_compute", "unpack_bits",
    "to_float", "Ingest", "load_png", "png_frames", "png_info",
]
