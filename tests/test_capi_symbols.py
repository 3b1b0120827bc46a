"""CPU: libfdhip.so loads without a GPU and exports every function include/fd_hip.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "fd_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(fd_[a-z_0-9]+)\s*\(", src, flags=re.M)))


def test_header_parses():
    names = declared_functions()
    assert "fd_points_detect" in names and "fd_lsd_map" in names and len(names) >= 10


def test_library_exports_all_declared_symbols():
    import feature_detector_amd as fd

    L = fd.load()
    for name in declared_functions():
        assert hasattr(L, name), name
    from feature_detector_amd._lib import EXPORTS

    assert sorted(EXPORTS) == declared_functions()


def test_build_info_and_no_device_error():
    import feature_detector_amd as fd

    L = fd.load()
    assert b"gfx950" in L.fd_build_info()
    if os.environ.get("HIP_VISIBLE_DEVICES") is None:
        try:
            import torch

            has_gpu = torch.cuda.is_available()
        except Exception:
            has_gpu = False
        if not has_gpu:
            p = ctypes.c_void_p()
            assert L.fd_ctx_create(0, ctypes.byref(p)) != 0  # fails loudly, no CPU fallback
            with pytest.raises(fd.FdError):
                fd.Context(0)


def test_null_context_calls_are_rejected():
    import feature_detector_amd as fd

    L = fd.load()
    assert L.fd_ctx_synchronize(None) != 0
    assert L.fd_ctx_set_stream(None, None) != 0
