"""ctypes binding of the CPU oracle (oracle/fd_oracle.cpp). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker / the timed CPU baseline. The product path (feature_detector_amd) never imports it.
Each wrapper names the reference function it restates (paths relative to /root/reference/src/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "liborc.so")
SRCS = [os.path.join(HERE, f) for f in ("fd_oracle.cpp", "fd_oracle_refflow.cpp", "fd_oracle_lines.cpp",
                                        "fd_oracle_introsort.cpp", "Makefile")]

HARRIS, SHI_TOMASI, FAST = 0, 1, 2
_P = ctypes.c_void_p
_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with the reference build's float semantics (no -march => no FMA)."""
    os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < max(map(os.path.getmtime, SRCS)):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        i32, i64, f32, u32, u8 = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_uint32, ctypes.c_uint8
        sig = {
            "orc_tensor_sums": (None, [_P, i32, i32, _P, _P, _P]),
            "orc_response_map": (None, [_P, i32, i32, i32, f32, _P, _P]),
            "orc_nms": (i64, [_P, i32, i32, f32, _P, _P, _P, i64]),
            "orc_fast_score": (i32, [_P, i32, i32, i32, i32, i32]),
            "orc_fast_candidates": (i64, [_P, i32, i32, f32, _P, _P, _P, _P, i64]),
            "orc_fast_offsets": (None, [i64, _P]),
            "orc_detect": (i64, [i32, _P, i32, i32, i32, f32, u32, _P, i32, i32, _P, i32, _P, _P, _P, _P, i64]),
            "orc_select": (i32, [_P, _P, _P, i64, i32, i32, i32, u32, _P, i32, i32, _P, i32, _P, _P, _P]),
            "orc_prefix_has_ties": (i32, [_P, i64]),
            "orc_sparsify": (None, [_P, i32, i32, i32, i32, i32, u8, u8, _P, _P]),
            "orc_lsd_map": (i64, [_P, i32, i32, f32, _P, _P, _P, _P, i64]),
            "orc_lsd_sort": (None, [_P, _P, i64, i32]),
            "orc_lsd_min_region_size": (u32, [i32, i32, f32]),
            "orc_make_frame": (None, [i32, u32, i32, i32, i32, _P]),
            "orc_brief": (None, [_P, i32, i32, _P, i32, i32, i32, i32, _P, _P, _P, _P]),
            "orc_nn_select": (i32, [_P, i32, i32, i32, i32, i32, f32, _P, i32, _P, i32]),
            "orc_nn_select_list": (i32, [_P, _P, i64, i32, i32, i32, i32, i32, _P, i32, _P, _P, i32]),
            "orc_nn_descriptors": (None, [_P, i32, i32, i32, _P, i32, _P]),
            "orc_lsd_lines": (i64, [_P, i32, i32, _P, u32, _P, i64]),
            "orc_ref_state_new": (_P, []),
            "orc_ref_state_free": (None, [_P]),
            "orc_detect_refflow": (i32, [_P, i32, _P, i32, i32, i32, f32, u32, _P, i32]),
            "orc_std_sort_perm": (None, [_P, i64, _P]),
            "orc_std_sort_restated": (None, [_P, i64, _P, _P]),
            "orc_introsort_killer": (None, [i64, i32, _P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def make_frame(pattern: str, seed: int, rows: int, cols: int, period: int = 16) -> np.ndarray:
    """Seeded synthetic frame: 'noise' (uniform u8) or 'checker' (period-px 60/180 + U[-10,10])."""
    out = np.empty((rows, cols), np.uint8)
    lib().orc_make_frame(0 if pattern == "noise" else 1, seed, rows, cols, period, _ptr(out))
    return out


def response_map(img, kind, thr, mask=None):
    img = np.ascontiguousarray(img, np.uint8)
    R, C = img.shape
    out = np.zeros((R, C), np.float32)
    m = None if mask is None else np.ascontiguousarray(mask, np.int32)
    lib().orc_response_map(_ptr(img), R, C, kind, thr, _ptr(m), _ptr(out))
    return out


def tensor_sums(img):
    img = np.ascontiguousarray(img, np.uint8)
    R, C = img.shape
    a, b, c = (np.zeros((R, C), np.int32) for _ in range(3))
    lib().orc_tensor_sums(_ptr(img), R, C, _ptr(a), _ptr(b), _ptr(c))
    return a, b, c


def nms(resp, thr):
    resp = np.ascontiguousarray(resp, np.float32)
    R, C = resp.shape
    cap = R * C // 2 + 16
    r, x, y = np.zeros(cap, np.float32), np.zeros(cap, np.int32), np.zeros(cap, np.int32)
    n = lib().orc_nms(_ptr(resp), R, C, thr, _ptr(r), _ptr(x), _ptr(y), cap)
    return r[:n], x[:n], y[:n]


def fast_candidates(img, thr, mask=None):
    img = np.ascontiguousarray(img, np.uint8)
    R, C = img.shape
    cap = R * C
    r, x, y = np.zeros(cap, np.float32), np.zeros(cap, np.int32), np.zeros(cap, np.int32)
    m = None if mask is None else np.ascontiguousarray(mask, np.int32)
    n = lib().orc_fast_candidates(_ptr(img), R, C, thr, _ptr(m), _ptr(r), _ptr(x), _ptr(y), cap)
    return r[:n], x[:n], y[:n]


def fast_offsets(n):
    out = np.zeros(n, np.float32)
    lib().orc_fast_offsets(n, _ptr(out))
    return out


def detect(kind, img, dist, thr, need, prior=None, sort_mode=0):
    """FeaturePointDetector::DetectGoodFeatures (feature_point_detector.cpp:7-25) for one frame.

    Returns (new_features[n,2] float32 (x, y), sorted candidates (resp, x, y)).
    sort_mode 0 = reference std::sort order, 1 = stable (response desc, raster asc).
    """
    img = np.ascontiguousarray(img, np.uint8)
    R, C = img.shape
    pr = np.zeros((1, 2), np.float32) if prior is None or len(prior) == 0 else np.ascontiguousarray(prior, np.float32)
    n_prior = 0 if prior is None else len(prior)
    out_cap = max(int(need) + 1, 1)
    out = np.zeros((out_cap, 2), np.float32)
    nout = ctypes.c_int(0)
    cap = R * C
    cr, cx, cy = np.zeros(cap, np.float32), np.zeros(cap, np.int32), np.zeros(cap, np.int32)
    n = lib().orc_detect(kind, _ptr(img), R, C, dist, thr, need, _ptr(pr), n_prior, sort_mode, _ptr(out), out_cap,
                         ctypes.byref(nout), _ptr(cr), _ptr(cx), _ptr(cy), cap)
    return out[: nout.value].copy(), (cr[:n].copy(), cx[:n].copy(), cy[:n].copy())


def select(resp, x, y, rows, cols, dist, need, prior=None, sort_mode=0, sorted_out=False):
    """SelectGoodFeatures (feature_point_detector.cpp:54-74) over caller-supplied candidates in push
    order, with the prior-feature mask (:12-16, :90-98). Returns new features [n,2] float32 (x, y)
    (and, with sorted_out, the candidates as the sort leaves them: (resp, x, y)).
    sort_mode 0 = the reference's std::sort on the pushed order, 1 = response desc, raster index asc."""
    resp = np.ascontiguousarray(resp, np.float32)
    x = np.ascontiguousarray(x, np.int32)
    y = np.ascontiguousarray(y, np.int32)
    pr = np.zeros((1, 2), np.float32) if prior is None or len(prior) == 0 else np.ascontiguousarray(prior, np.float32)
    n_prior = 0 if prior is None else len(prior)
    out_cap = max(int(need) + 1, 1)
    out = np.zeros((out_cap, 2), np.float32)
    sr, sx, sy = (np.zeros(len(resp), np.float32), np.zeros(len(resp), np.int32),
                  np.zeros(len(resp), np.int32)) if sorted_out else (None, None, None)
    n = lib().orc_select(_ptr(resp), _ptr(x), _ptr(y), len(resp), rows, cols, dist, need, _ptr(pr), n_prior,
                         sort_mode, _ptr(out), out_cap, _ptr(sr), _ptr(sx), _ptr(sy))
    feats = out[:min(n, out_cap)].copy()
    return (feats, (sr, sx, sy)) if sorted_out else feats


class RefFlowDetector:
    """DetectGoodFeatures in the reference's data flow (oracle/fd_oracle_refflow.cpp): float sliding
    sums, dense response map, pair list, std::sort, int32 mask. One instance per thread, like the
    reference's detector objects; used as the timed CPU baseline and checked against detect()."""

    def __init__(self):
        self._s = lib().orc_ref_state_new()

    def detect(self, kind, img, dist, thr, need):
        img = np.ascontiguousarray(img, np.uint8)
        R, C = img.shape
        cap = max(int(need), 1)
        out = np.zeros((cap, 2), np.float32)
        n = lib().orc_detect_refflow(self._s, kind, _ptr(img), R, C, dist, thr, need, _ptr(out), cap)
        return out[:min(n, cap)].copy()

    def __del__(self):
        if getattr(self, "_s", None) and _lib is not None:
            _lib.orc_ref_state_free(self._s)
            self._s = None


def std_sort_perm(resp):
    """The visiting order std::sort gives (resp, push index) pairs with the reference comparator
    (feature_point_detector.cpp:58-60): indices into resp."""
    resp = np.ascontiguousarray(resp, np.float32)
    perm = np.zeros(len(resp), np.uint32)
    lib().orc_std_sort_perm(_ptr(resp), len(resp), _ptr(perm))
    return perm


def std_sort_restated(resp):
    """libstdc++ 11's std::sort restated (oracle/fd_oracle_introsort.cpp) -> (perm, stats): stats =
    (heapsorted ranges, frontmost heapsorted range lo, hi (-1: none), smallest depth left)."""
    resp = np.ascontiguousarray(resp, np.float32)
    perm = np.zeros(len(resp), np.uint32)
    stats = np.zeros(4, np.int64)
    lib().orc_std_sort_restated(_ptr(resp), len(resp), _ptr(perm), _ptr(stats))
    return perm, stats


def introsort_killer(n, front=True):
    """Responses (push order) built by McIlroy's adversary against std::sort with the reference
    comparator: the introsort reaches its depth limit (heapsort); front: in the range the greedy visits
    first, which then starts with a run of equal responses."""
    out = np.zeros(n, np.float32)
    lib().orc_introsort_killer(n, 1 if front else 0, _ptr(out))
    return out


def prefix_has_ties(sorted_resp, n_scanned):
    a = np.ascontiguousarray(sorted_resp, np.float32)
    return bool(lib().orc_prefix_has_ties(_ptr(a), int(n_scanned)))


def sparsify(xy, rows, cols, grid_rows=12, grid_cols=12, need_filter=1, after_filter=0, status=None):
    xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
    n = len(xy)
    st = np.ones(n, np.uint8) if status is None or len(status) != n else np.array(status, np.uint8)
    gm = np.zeros((grid_rows, grid_cols), np.int32)
    lib().orc_sparsify(_ptr(xy), n, rows, cols, grid_rows, grid_cols, need_filter, after_filter, _ptr(st), _ptr(gm))
    return st, gm


def lsd_map(img, min_norm=20.0):
    img = np.ascontiguousarray(img, np.uint8)
    R, C = img.shape
    norm = np.zeros((R - 1, C - 1), np.float32)
    ang = np.zeros((R - 1, C - 1), np.float32)
    val = np.zeros((R - 1, C - 1), np.uint8)
    cap = (R - 1) * (C - 1)
    idx = np.zeros(cap, np.int32)
    n = lib().orc_lsd_map(_ptr(img), R, C, min_norm, _ptr(norm), _ptr(ang), _ptr(val), _ptr(idx), cap)
    return norm, ang, val, idx[:n].copy()


def lsd_sort(norm, idx, sort_mode=0):
    norm = np.ascontiguousarray(norm, np.float32)
    idx = np.array(idx, np.int32)
    lib().orc_lsd_sort(_ptr(norm), _ptr(idx), len(idx), sort_mode)
    return idx


LSD_TOL_RAD = float(np.float32(22.5) * (np.float32(3.14159265358979323846) / np.float32(180.0)))


def lsd_lines(img, needed=1, min_norm=20.0, tol_rad=LSD_TOL_RAD, min_length=20.0, min_inlier=0.6, cap=4096):
    """FeatureLineDetector::DetectGoodFeatures (feature_line_detector.cpp:12-54) on one frame: [n, 12]
    float32 rectangles (start x, y, end x, y, center x, y, length, width, angle, dir x, y, inlier)."""
    img = np.ascontiguousarray(img, np.uint8)
    R, C = img.shape
    opts = np.array([min_norm, tol_rad, min_length, min_inlier], np.float32)
    out = np.zeros((max(cap, 1), 12), np.float32)
    n = lib().orc_lsd_lines(_ptr(img), R, C, _ptr(opts), needed, _ptr(out), cap)
    if n > cap:
        raise RuntimeError(f"cap {cap} < {n} lines")
    return out[:max(n, 0)].copy()


def lsd_min_region_size(rows, cols, tol_rad=22.5 * 3.14159265358979323846 / 180.0):
    return int(lib().orc_lsd_min_region_size(rows, cols, np.float32(tol_rad)))


# ------------------------------------------------------------------------------------- BRIEF (f1)
PATTERN_INC = os.path.join(HERE, "..", "feature_detector_amd", "csrc", "fd_brief_pattern.inc")


def brief_pattern() -> np.ndarray:
    """pattern_idx_ (descriptor_brief.cpp:52-309) as int16[1024], from the generated table
    (tools/gen_brief_pattern.py; tests/test_brief_host.py checks it against the reference source)."""
    import re

    words = [int(t, 16) for t in re.findall(r"0x[0-9a-fA-F]{8}", open(PATTERN_INC).read())]
    assert len(words) == 256
    b = np.array(words, np.uint32).view(np.uint8).reshape(256, 4).view(np.int8)
    return b.astype(np.int16).reshape(-1)


def brief(img, uv, length=256, half=8, sampler=0):
    """BriefDescriptor::ComputeForOneFeature (descriptor_brief.cpp:8-50) per keypoint.

    Returns (bits uint32 [n, ceil(length/32)], valid uint8 [n], moments float32 [n, 3] = m10, m01, m).
    sampler 0 = bilinear, 1 = truncation (the reference's float sampler is un-vendored: unpinned)."""
    img = np.ascontiguousarray(img, np.uint8)
    R, C = img.shape
    uv = np.ascontiguousarray(np.asarray(uv, np.float32).reshape(-1, 2))
    n = len(uv)
    nw = (length + 31) // 32
    bits = np.zeros((max(n, 1), nw), np.uint32)
    valid = np.zeros(max(n, 1), np.uint8)
    mom = np.zeros((max(n, 1), 3), np.float32)
    pat = brief_pattern()
    lib().orc_brief(_ptr(img), R, C, _ptr(uv), n, length, half, sampler, _ptr(pat), _ptr(bits), _ptr(valid),
                    _ptr(mom))
    return bits[:n], valid[:n], mom[:n]


# ------------------------------------------------------------------------------ SuperPoint (f3)
def nn_select(heat, border=3, dist=15, max_features=240, thr=0.1, prior=None):
    """CreateMask + SelectKeypointCandidatesFromHeatMap + SelectGoodFeaturesFromCandidates
    (nn_feature_point_detector.cpp:59-73, 128-155) on one heatmap; returns new features (n, 2) (x, y)."""
    heat = np.ascontiguousarray(heat, np.float32)
    R, C = heat.shape
    pr = np.zeros((1, 2), np.float32) if prior is None or len(prior) == 0 else np.ascontiguousarray(prior, np.float32)
    n_prior = 0 if prior is None else len(prior)
    cap = max(max_features, 1) + 1
    out = np.zeros((cap, 2), np.float32)
    n = lib().orc_nn_select(_ptr(heat), R, C, border, dist, max_features, np.float32(thr), _ptr(pr), n_prior,
                            _ptr(out), cap)
    return out[:min(n, cap)].copy()


def nn_select_list(kp, scores, rows, cols, border=3, dist=15, max_features=240, prior=None):
    """ArgSort + DirectlySelectGoodFeaturesWithDescriptors (nn_feature_point_detector.cpp:204-230) on one
    frame's keypoint list (kp [n, 2] int64 (u, v), scores [n]); returns (new features (m, 2) (x, y),
    their list indices (m,)). Equal scores: see orc_nn_select_list (ArgSort unpinned)."""
    kp = np.ascontiguousarray(kp, np.int64).reshape(-1, 2)
    scores = np.ascontiguousarray(scores, np.float32)
    pr = np.zeros((1, 2), np.float32) if prior is None or len(prior) == 0 else np.ascontiguousarray(prior, np.float32)
    n_prior = 0 if prior is None else len(prior)
    cap = max(max_features, 1) + 1
    out = np.zeros((cap, 2), np.float32)
    idx = np.zeros(cap, np.int32)
    n = lib().orc_nn_select_list(_ptr(kp), _ptr(scores), len(scores), rows, cols, border, dist, max_features, _ptr(pr),
                                 n_prior, _ptr(out), _ptr(idx), cap)
    return out[:min(n, cap)].copy(), idx[:min(n, cap)].copy()


def nn_descriptors(desc_map, xy):
    """ExtractDescriptorsForSelectedFeatures (nn_feature_point_detector.cpp:163-193); desc_map [C, h, w]."""
    desc_map = np.ascontiguousarray(desc_map, np.float32)
    ch, h, w = desc_map.shape
    xy = np.ascontiguousarray(np.asarray(xy, np.float32).reshape(-1, 2))
    out = np.zeros((max(len(xy), 1), ch), np.float32)
    lib().orc_nn_descriptors(_ptr(desc_map), ch, h, w, _ptr(xy), len(xy), _ptr(out))
    return out[:len(xy)]
