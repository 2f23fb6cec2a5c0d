"""ctypes binding of the CPU oracle (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("JXO_LIB_PATH") or os.path.join(HERE, "liboracle.so")  # ASan runs


def build(force: bool = False):
    if os.environ.get("JXO_LIB_PATH"):
        return  # a prebuilt variant (tools/asan_suite.sh)
    if force or not os.path.exists(LIB) or any(
            os.path.getmtime(os.path.join(HERE, f)) > os.path.getmtime(LIB)
            for f in os.listdir(HERE) if f.endswith((".c", ".h"))):
        subprocess.check_call(["make", "-s", "-C", HERE])


class _Params(ctypes.Structure):
    _fields_ = [("distance", ctypes.c_float), ("effort", ctypes.c_int),
                ("proposals", ctypes.c_uint32), ("coder", ctypes.c_int),
                ("filters", ctypes.c_uint32)]

FILTER_GAB = 1  # jxo.h JXO_FILTER_GAB
FILTER_EPF = 2  # jxo.h JXO_FILTER_EPF


class _Result(ctypes.Structure):
    _fields_ = [("xsize", ctypes.c_uint32), ("ysize", ctypes.c_uint32),
                ("bxs", ctypes.c_uint32), ("bys", ctypes.c_uint32),
                ("acs", ctypes.POINTER(ctypes.c_uint8)), ("qf", ctypes.POINTER(ctypes.c_uint8)),
                ("dc", ctypes.POINTER(ctypes.c_int32)), ("ac", ctypes.POINTER(ctypes.c_int32)),
                ("ac_tokens", ctypes.POINTER(ctypes.c_uint32)), ("homog", ctypes.POINTER(ctypes.c_float)),
                ("cmap", ctypes.POINTER(ctypes.c_int8)), ("tiles_x", ctypes.c_uint32),
                ("tiles_y", ctypes.c_uint32),
                ("global_scale", ctypes.c_uint32), ("quant_dc", ctypes.c_uint32),
                ("bytes", ctypes.POINTER(ctypes.c_uint8)), ("nbytes", ctypes.c_size_t)]


class _Xyb(ctypes.Structure):
    _fields_ = [("plane", ctypes.c_void_p * 3), ("xsize", ctypes.c_size_t),
                ("ysize", ctypes.c_size_t), ("stride", ctypes.c_size_t)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
        _lib.jxo_encode_rgb8.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_size_t, ctypes.POINTER(_Params), ctypes.POINTER(_Result)]
        _lib.jxo_result_free.argtypes = [ctypes.POINTER(_Result)]
        _lib.jxo_homog_map.argtypes = [ctypes.POINTER(_Xyb), ctypes.c_float, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_void_p]
        _lib.jxo_homogeneity.argtypes = [ctypes.POINTER(_Xyb), ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.c_size_t, ctypes.c_float, ctypes.c_int]
        _lib.jxo_homogeneity.restype = ctypes.c_float
        _lib.jxo_hook_f.argtypes = [ctypes.c_float] * 4
        _lib.jxo_hook_f.restype = ctypes.c_float
        _lib.jxo_srgb8_to_xyb.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
        _lib.jxo_cbrtf.argtypes = [ctypes.c_float]
        _lib.jxo_cbrtf.restype = ctypes.c_float
        _lib.jxo_export_kind.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        _lib.jxo_export_kind.restype = ctypes.c_int
        _lib.jxo_export_dct.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _lib.jxo_set_debug_big_cost.argtypes = [ctypes.c_void_p]
        _lib.jxo_set_debug_big_cost.restype = None
        _lib.jxo_set_debug_group_bins.argtypes = [ctypes.c_void_p]
        _lib.jxo_set_debug_group_bins.restype = None
        _lib.jxo_synth_rgb8.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                        ctypes.c_void_p]
        _lib.jxo_set_threads.argtypes = [ctypes.c_int]
        _lib.jxo_set_threads.restype = ctypes.c_int
    return _lib


def synth_rgb8(w: int, h: int, seed: int) -> np.ndarray:
    """C restatement of jxg.synth.synth_rgb8 (same bytes, OpenMP)."""
    out = np.empty((h, w, 3), dtype=np.uint8)
    lib().jxo_synth_rgb8(w, h, seed & 0xFFFFFFFFFFFFFFFF, out.ctypes.data)
    return out


def set_threads(n: int) -> int:
    """OpenMP threads of the oracle encode (n <= 0: query); returns the count."""
    return lib().jxo_set_threads(n)


class OracleResult:
    pass


def encode(rgb: np.ndarray, distance=1.0, effort=7, proposals=0, coder=0,
           filters=0) -> OracleResult:
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w, _ = rgb.shape
    p = _Params(distance, effort, proposals, coder, filters)
    r = _Result()
    st = lib().jxo_encode_rgb8(rgb.ctypes.data, w, h, w * 3, ctypes.byref(p), ctypes.byref(r))
    if st != 0:
        raise RuntimeError("oracle encode failed: %d" % st)
    try:
        o = OracleResult()
        nb = r.bxs * r.bys
        o.bxs, o.bys = r.bxs, r.bys
        o.acs = np.ctypeslib.as_array(r.acs, (nb,)).copy().reshape(r.bys, r.bxs)
        o.qf = np.ctypeslib.as_array(r.qf, (nb,)).copy().reshape(r.bys, r.bxs)
        o.dc = np.ctypeslib.as_array(r.dc, (3 * nb,)).copy().reshape(3, r.bys, r.bxs)
        o.ac = np.ctypeslib.as_array(r.ac, (nb * 192,)).copy().reshape(r.bys, r.bxs, 3, 64)
        ng = ((w + 255) // 256) * ((h + 255) // 256)
        o.ac_tokens = np.ctypeslib.as_array(r.ac_tokens, (ng * 3,)).copy().reshape(ng, 3)
        o.homog = (np.ctypeslib.as_array(r.homog, (nb * 3,)).copy().reshape(r.bys, r.bxs, 3)
                   if r.homog else None)
        nt = r.tiles_x * r.tiles_y
        o.cmap = np.ctypeslib.as_array(r.cmap, (2 * nt,)).copy().reshape(2, r.tiles_y, r.tiles_x)
        o.global_scale, o.quant_dc = r.global_scale, r.quant_dc
        o.bytes = bytes(np.ctypeslib.as_array(r.bytes, (r.nbytes,)))
        return o
    finally:
        lib().jxo_result_free(ctypes.byref(r))


def _xyb_struct(planes: np.ndarray):
    planes = np.ascontiguousarray(planes, dtype=np.float32)
    _, ys, xs = planes.shape
    s = _Xyb()
    for c in range(3):
        s.plane[c] = planes[c].ctypes.data
    s.xsize, s.ysize, s.stride = xs, ys, xs
    return s, planes


def homog_map(planes: np.ndarray, distance: float, h1_mode: int = 0):
    """planes: (3, Hp, Wp) float32 XYB.  Returns (r3 (bys,bxs,3), type (bys,bxs))."""
    s, planes = _xyb_struct(planes)
    _, ys, xs = planes.shape
    r3 = np.zeros((ys // 8, xs // 8, 3), dtype=np.float32)
    t = np.zeros((ys // 8, xs // 8), dtype=np.uint8)
    lib().jxo_homog_map(ctypes.byref(s), distance, h1_mode, r3.ctypes.data, t.ctypes.data)
    return r3, t


def homogeneity(planes, x, y, xs, ys, bx, by, distance, h1_mode=0):
    s, planes = _xyb_struct(planes)
    return lib().jxo_homogeneity(ctypes.byref(s), x, y, xs, ys, bx, by, distance, h1_mode)


def hook_f(ret, rh, rv, rd):
    return lib().jxo_hook_f(ret, rh, rv, rd)


def srgb8_to_xyb(rgb: np.ndarray) -> np.ndarray:
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w, _ = rgb.shape
    xp, yp = (w + 7) // 8 * 8, (h + 7) // 8 * 8
    out = np.zeros((3, yp, xp), dtype=np.float32)
    lib().jxo_srgb8_to_xyb(rgb.ctypes.data, w, h, w * 3, xp, yp, out.ctypes.data)
    return out


KIND_DIMS = [(8, 16), (16, 16), (16, 32), (32, 32), (32, 64), (64, 64), (64, 128), (128, 128),
             (128, 256), (256, 256)]


def kind_tables(kind: int):
    """(weights (3, rows*cols) float32, natural position of each stored index)"""
    r, c = KIND_DIMS[kind]
    w = np.zeros(3 * r * c, dtype=np.float32)
    nat = np.zeros(r * c, dtype=np.uint16)
    n = lib().jxo_export_kind(kind, w.ctypes.data, nat.ctypes.data)
    assert n == r * c
    return w.reshape(3, r * c), nat


def dct(x: np.ndarray) -> np.ndarray:
    """the oracle's normalized 1-D DCT (Lee) of a float32 vector"""
    v = np.ascontiguousarray(x, dtype=np.float32).copy()
    lib().jxo_export_dct(v.ctypes.data, len(v))
    return v


def debug_big_costs(rgb: np.ndarray, distance=1.0, effort=8, proposals=0, coder=0, filters=0):
    """(result, [groups][25] candidate estimates of the 128 / 256 px levels)
    -- the layout of the product's JXG_DEBUG_BIGCOST dump (test hook)"""
    h, w, _ = rgb.shape
    ng = ((w + 255) // 256) * ((h + 255) // 256)
    buf = np.full(ng * 25, np.nan, dtype=np.float32)
    lib().jxo_set_debug_big_cost(buf.ctypes.data)
    try:
        r = encode(rgb, distance, effort, proposals, coder, filters)
    finally:
        lib().jxo_set_debug_big_cost(None)
    return r, buf.reshape(ng, 25)


def max_group_bin(rgb: np.ndarray, distance=1.0, effort=7, proposals=0, coder=0, filters=0):
    """(result, the largest count of one (static cluster, token) bin inside one
    pass group) -- what the product's per-group LDS histogram must hold (test
    hook)"""
    buf = np.zeros(1, dtype=np.uint32)
    lib().jxo_set_debug_group_bins(buf.ctypes.data)
    try:
        r = encode(rgb, distance, effort, proposals, coder, filters)
    finally:
        lib().jxo_set_debug_group_bins(None)
    return r, int(buf[0])
