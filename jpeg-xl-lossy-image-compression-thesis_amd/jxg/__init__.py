"""jxg -- Python host mirror of the MI355X JPEG XL VarDCT encode path.

Thin ctypes layer over the C ABI in include/jxg.h (libjxg.so, built in-tree
for gfx950).  It mirrors the reference harness's encoder boundary:

* ``execute_cjxl(input, output, distance, effort)`` follows
  ``DockerManager::execute_cjxl`` (benchmark-jpegxl/src/docker_manager.rs:
  100-137): ``mkdir -p dirname(output)``, run the encoder with
  ``--distance=D --effort=E``, return ``(True, stdout)`` on exit 0 and
  ``(False, stderr-or-stdout)`` otherwise;
* ``comp_image_name`` is the ``{stem}-{distance}-{effort}.jxl`` naming of
  benchmark.rs:644-650 (Rust ``{}`` formatting of f64);
* ``calculate_mse`` / ``calculate_psnr`` restate image_reader.rs:555-606.

There is no CPU fallback: importing works anywhere, but every encode goes
through libjxg.so on a HIP device and raises if either is missing.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JXG_LIB_PATH") or os.path.join(HERE, "libjxg.so")  # override: experiments only
CLI_PATH = os.path.join(HERE, "jxg_cjxl")

PROPOSAL_P = 1
PROPOSAL_F = 2
FLAG_H1_INT_ABS = 1
FLAG_KEEP_MAPS = 2
FLAG_ANS = 4
FLAG_FORCE_ONE_STREAM = 8  # testing: the split assembly's one-stream fallback (same bytes)
FLAG_GABORISH = 16  # encoder inverse Gaborish + the decoder's Gaborish (cjxl --gaborish=1)
FLAG_EPF = 32  # the decoder's edge-preserving filter, iterations by distance (cjxl --epf=-1)
FLAG_AQ_MASKING = 64  # libjxl-shaped masking quant field (oracle/aq.c) instead of the activity AQ
# JXG_FLAGS_CJXL_DEFAULTS: what `cjxl IN OUT --distance=D --effort=E` encodes
# (docker_manager.rs:126-136) -- jxg_cjxl's defaults, bench.py's headline
FLAGS_CJXL_DEFAULTS = FLAG_ANS | FLAG_GABORISH | FLAG_EPF | FLAG_AQ_MASKING
# the same set as the oracle's filters mask (oracle/jxo.h: GAB 1 | EPF 2 | AQ_MASKING 4; coder 1)
ORACLE_FILTERS_CJXL_DEFAULTS = 7


class JxgError(RuntimeError):
    pass


class _Params(ctypes.Structure):
    _fields_ = [("distance", ctypes.c_float), ("effort", ctypes.c_int),
                ("proposals", ctypes.c_uint32), ("num_devices", ctypes.c_int),
                ("flags", ctypes.c_uint32), ("device", ctypes.c_int)]


class _Buffer(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_uint8)), ("size", ctypes.c_size_t)]


class _Stats(ctypes.Structure):
    _fields_ = [("xsize", ctypes.c_uint32), ("ysize", ctypes.c_uint32),
                ("xsize_blocks", ctypes.c_uint32), ("ysize_blocks", ctypes.c_uint32),
                ("num_groups", ctypes.c_uint32), ("num_lf_groups", ctypes.c_uint32),
                ("global_scale", ctypes.c_uint32), ("quant_dc", ctypes.c_uint32),
                ("bytes", ctypes.c_size_t),
                ("ac_strategy", ctypes.POINTER(ctypes.c_uint8)),
                ("quant_field", ctypes.POINTER(ctypes.c_uint8)),
                ("dc", ctypes.POINTER(ctypes.c_int32)),
                ("ac", ctypes.POINTER(ctypes.c_int32)),
                ("ac_tokens", ctypes.POINTER(ctypes.c_uint32)),
                ("homogeneity", ctypes.POINTER(ctypes.c_float)),
                ("ms_front", ctypes.c_float), ("ms_histogram", ctypes.c_float),
                ("ms_emit", ctypes.c_float), ("ms_assemble", ctypes.c_float),
                ("ms_total", ctypes.c_float), ("ms_host_call", ctypes.c_float),
                ("ms_host_codes", ctypes.c_float), ("ms_host_layout", ctypes.c_float),
                ("ms_front_kernel", ctypes.c_float), ("ms_aq", ctypes.c_float)]


class _Quality(ctypes.Structure):
    _fields_ = [("sse", ctypes.c_uint64), ("samples", ctypes.c_uint64), ("mse", ctypes.c_double),
                ("psnr", ctypes.c_double), ("ssim", ctypes.c_double)]


# every symbol declared in include/jxg.h
EXPORTS = ("jxg_status_str", "jxg_create", "jxg_destroy", "jxg_encode_rgb8",
           "jxg_encode_rgb8_device", "jxg_encode_batch_rgb8", "jxg_get_stats",
           "jxg_buffer_free", "jxg_homogeneity_map", "jxg_shard_sizes", "jxg_shard_begin",
           "jxg_shard_end", "jxg_shard_payload", "jxg_shard_assemble_device",
           "jxg_shard_assemble", "jxg_compare_rgb8", "jxg_compare_rgb8_device",
           "jxg_shard_head", "jxg_shard_write_host", "jxg_host_register", "jxg_host_unregister",
           "jxg_encode_batch_rgb8_device", "jxg_synth_rgb8_device", "jxg_shard_exchange",
           "jxg_submit_rgb8", "jxg_submit_rgb8_device", "jxg_receive", "jxg_pending",
           "jxg_set_input_stream", "jxg_pipeline_depth", "jxg_shard_plan",
           "jxg_shard_submit_device", "jxg_shard_next_head", "jxg_shard_write_next",
           "jxg_shard_write_flush", "jxg_set_pipeline_lanes", "jxg_warmup",
)

_lib = None


def load():
    """Load libjxg.so (raises JxgError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise JxgError("libjxg.so not built at %s (run __graft_entry__.build())" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    lib.jxg_status_str.restype = ctypes.c_char_p
    lib.jxg_status_str.argtypes = [ctypes.c_int]
    lib.jxg_create.argtypes = [ctypes.POINTER(_Params), ctypes.POINTER(vp)]
    lib.jxg_destroy.argtypes = [vp]
    lib.jxg_destroy.restype = None
    lib.jxg_encode_rgb8.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t,
                                    ctypes.POINTER(_Buffer)]
    lib.jxg_encode_rgb8_device.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_size_t, ctypes.POINTER(_Buffer)]
    lib.jxg_encode_batch_rgb8.argtypes = [vp, ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t,
                                          ctypes.POINTER(_Buffer)]
    lib.jxg_encode_batch_rgb8_device.argtypes = lib.jxg_encode_batch_rgb8.argtypes
    lib.jxg_submit_rgb8.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t]
    lib.jxg_submit_rgb8_device.argtypes = lib.jxg_submit_rgb8.argtypes
    lib.jxg_receive.argtypes = [vp, ctypes.POINTER(_Buffer)]
    lib.jxg_pending.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32)]
    lib.jxg_get_stats.argtypes = [vp, ctypes.POINTER(_Stats)]
    lib.jxg_buffer_free.argtypes = [ctypes.POINTER(_Buffer)]
    lib.jxg_buffer_free.restype = None
    lib.jxg_homogeneity_map.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_float,
                                        ctypes.c_uint32, vp, vp]
    sz = ctypes.c_size_t
    lib.jxg_shard_sizes.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.POINTER(sz), ctypes.POINTER(sz)]
    lib.jxg_shard_exchange.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.POINTER(sz), ctypes.POINTER(sz)]
    lib.jxg_shard_begin.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, sz, ctypes.c_uint32,
                                    ctypes.c_uint32, vp, vp]
    lib.jxg_shard_end.argtypes = [vp, vp, vp, ctypes.POINTER(sz)]
    lib.jxg_shard_payload.argtypes = [vp, vp, ctypes.c_int]
    lib.jxg_shard_assemble_device.argtypes = [vp, vp, ctypes.POINTER(sz), ctypes.POINTER(sz),
                                              ctypes.c_uint32, ctypes.POINTER(_Buffer)]
    lib.jxg_shard_assemble.argtypes = [ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                       ctypes.POINTER(sz), ctypes.c_uint32, ctypes.POINTER(_Buffer)]
    lib.jxg_shard_head.argtypes = [vp, vp, ctypes.POINTER(sz)]
    lib.jxg_shard_write_host.argtypes = [vp, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(sz),
                                         ctypes.c_uint32, vp, sz, ctypes.POINTER(sz)]
    lib.jxg_set_input_stream.argtypes = [vp, vp]
    lib.jxg_pipeline_depth.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    lib.jxg_shard_plan.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, vp, vp,
                                   ctypes.POINTER(ctypes.c_int)]
    lib.jxg_shard_submit_device.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, sz,
                                            ctypes.c_uint32, ctypes.c_uint32]
    lib.jxg_shard_next_head.argtypes = [vp, vp, ctypes.POINTER(sz)]
    lib.jxg_shard_write_next.argtypes = lib.jxg_shard_write_host.argtypes
    lib.jxg_shard_write_flush.argtypes = [vp]
    lib.jxg_set_pipeline_lanes.argtypes = [vp, ctypes.c_uint32]
    u32 = ctypes.c_uint32
    lib.jxg_host_register.argtypes = [vp, sz]
    lib.jxg_host_unregister.argtypes = [vp]
    cmp_args = [vp, vp, sz, vp, sz, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                ctypes.POINTER(_Quality)]
    lib.jxg_compare_rgb8.argtypes = cmp_args
    lib.jxg_compare_rgb8_device.argtypes = cmp_args
    lib.jxg_synth_rgb8_device.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint32, sz,
                                          ctypes.c_uint64]
    lib.jxg_warmup.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32]
    _lib = lib
    return lib


def _check(st):
    if st != 0:
        raise JxgError("jxg: %s (%d)" % (load().jxg_status_str(st).decode(), st))


class Codestream:
    """Zero-copy view of a jxg_buffer; released with jxg_buffer_free."""

    def __init__(self, buf):
        self._buf = buf
        self.size = buf.size

    def memoryview(self):
        return memoryview((ctypes.c_uint8 * self.size).from_address(self._buf.data)).cast("B")

    def tobytes(self) -> bytes:
        return ctypes.string_at(self._buf.data, self.size)

    def __len__(self):
        return self.size

    def release(self):
        if self._buf is not None and self._buf.data:
            load().jxg_buffer_free(ctypes.byref(self._buf))
        self._buf = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class Encoder:
    """One encoder context (= one HIP stream + device buffers) on one GPU."""

    def __init__(self, distance=1.0, effort=7, proposals=0, device=0, flags=0, num_devices=1):
        lib = load()
        self.params = _Params(distance, effort, proposals, num_devices, flags, device)
        self._ctx = ctypes.c_void_p()
        _check(lib.jxg_create(ctypes.byref(self.params), ctypes.byref(self._ctx)))

    def close(self):
        if self._ctx:
            load().jxg_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _take(buf):
        try:
            return ctypes.string_at(buf.data, buf.size)
        finally:
            load().jxg_buffer_free(ctypes.byref(buf))

    def encode(self, rgb: np.ndarray) -> bytes:
        """Host (H, W, 3) uint8 -> codestream bytes."""
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        h, w, c = rgb.shape
        if c != 3:
            raise ValueError("expected (H, W, 3) uint8")
        buf = _Buffer()
        _check(load().jxg_encode_rgb8(self._ctx, rgb.ctypes.data, w, h, w * 3, ctypes.byref(buf)))
        return self._take(buf)

    def encode_batch(self, frames) -> list:
        """Host frames of equal size, each (H, W, 3) uint8 -> list of codestream
        bytes (jxg_encode_batch_rgb8, BASELINE config 3)."""
        frames = [np.ascontiguousarray(f, dtype=np.uint8) for f in frames]
        if not frames:
            return []
        h, w, c = frames[0].shape
        if c != 3 or any(f.shape != frames[0].shape for f in frames):
            raise ValueError("expected equal-size (H, W, 3) uint8 frames")
        n = len(frames)
        ptrs = (ctypes.c_void_p * n)(*[f.ctypes.data for f in frames])
        outs = (_Buffer * n)()
        _check(load().jxg_encode_batch_rgb8(self._ctx, ptrs, n, w, h, w * 3, outs))
        return [self._take(outs[i]) for i in range(n)]

    def encode_batch_device(self, ptrs, width: int, height: int, row_stride: int | None = None,
                            copy: bool = True) -> list:
        """Device-resident frames of equal size (pointers) -> list of
        codestreams (jxg_encode_batch_rgb8_device); copy=False returns
        :class:`Codestream` views of the library's pinned buffers."""
        n = len(ptrs)
        if n == 0:
            return []
        arr = (ctypes.c_void_p * n)(*ptrs)
        outs = (_Buffer * n)()
        _check(load().jxg_encode_batch_rgb8_device(self._ctx, arr, n, width, height,
                                                   row_stride or width * 3, outs))
        return [self._take(outs[i]) if copy else Codestream(outs[i]) for i in range(n)]

    def encode_device(self, ptr: int, width: int, height: int, row_stride: int | None = None,
                      copy: bool = True):
        """Device-resident RGB8 (e.g. ``tensor.data_ptr()`` of a uint8 CUDA tensor).

        copy=False returns a :class:`Codestream` that owns the library's
        (pinned) output buffer instead of copying it into ``bytes``."""
        buf = _Buffer()
        _check(load().jxg_encode_rgb8_device(self._ctx, ctypes.c_void_p(ptr), width, height,
                                             row_stride or width * 3, ctypes.byref(buf)))
        return self._take(buf) if copy else Codestream(buf)

    # streaming encode (jxg_submit_rgb8[_device] / jxg_receive): a software
    # pipeline inside the library, driven by this thread
    def submit(self, rgb: np.ndarray):
        """Queue a host (H, W, 3) uint8 frame (copied before returning)."""
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        h, w, c = rgb.shape
        if c != 3:
            raise ValueError("expected (H, W, 3) uint8")
        _check(load().jxg_submit_rgb8(self._ctx, rgb.ctypes.data, w, h, w * 3))

    def submit_device(self, ptr: int, width: int, height: int, row_stride: int | None = None):
        """Queue a device-resident RGB8 frame; it must stay unchanged until its
        codestream has been received."""
        _check(load().jxg_submit_rgb8_device(self._ctx, ctypes.c_void_p(ptr), width, height,
                                             row_stride or width * 3))

    def receive(self, copy: bool = True):
        """Codestream of the oldest submitted frame (blocks until complete)."""
        buf = _Buffer()
        _check(load().jxg_receive(self._ctx, ctypes.byref(buf)))
        return self._take(buf) if copy else Codestream(buf)

    def pending(self) -> int:
        n = ctypes.c_uint32()
        _check(load().jxg_pending(self._ctx, ctypes.byref(n)))
        return n.value

    def pipeline_depth(self, width: int, height: int, rank: int = 0, world: int = 1) -> int:
        """Lanes of the streaming pipeline for these frames (or this rank's shard)."""
        n = ctypes.c_uint32()
        _check(load().jxg_pipeline_depth(self._ctx, width, height, rank, world, ctypes.byref(n)))
        return n.value

    def set_pipeline_lanes(self, lanes: int) -> None:
        """Cap this context's pipeline lanes (0: default) -- several contexts
        streaming on one GPU share its hardware queues (include/jxg.h)."""
        _check(load().jxg_set_pipeline_lanes(self._ctx, lanes))

    def set_input_stream(self, stream) -> None:
        """Order every later device-input call after the work submitted so far
        to `stream` (a hipStream_t handle, e.g. ``torch.cuda.current_stream()
        .cuda_stream``; None: the caller's writes are complete before each
        call) -- include/jxg.h."""
        _check(load().jxg_set_input_stream(self._ctx, ctypes.c_void_p(stream or None)))

    # streaming sharded encode (jxg_shard_submit_device / jxg_shard_next_head /
    # jxg_shard_write_next): see jxg.dist.ShardStream
    def shard_submit_device(self, ptr: int, width: int, height: int, rank: int, world: int,
                            row_stride: int | None = None):
        _check(load().jxg_shard_submit_device(self._ctx, ctypes.c_void_p(ptr), width, height,
                                              row_stride or width * 3, rank, world))

    def shard_next_head(self) -> np.ndarray:
        """Payload head of the oldest pending shard frame (waits for its sections)."""
        n = ctypes.c_size_t(0)
        _check(load().jxg_shard_next_head(self._ctx, None, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint32)
        _check(load().jxg_shard_next_head(self._ctx, out.ctypes.data, ctypes.byref(n)))
        return out

    def shard_write_next(self, heads, dst_ptr: int, dst_size: int):
        """jxg_shard_write_host for the oldest pending shard frame, which is then
        released; returns (ok, total) -- ok False when dst_size < total (the
        frame stays pending, nothing written).  The copies are enqueued: the
        PREVIOUS frame's are complete on return (:meth:`shard_write_flush`:
        the last one's)."""
        return self._write(load().jxg_shard_write_next, heads, dst_ptr, dst_size)

    def shard_write_flush(self):
        """Wait for the last shard_write_next's copies."""
        _check(load().jxg_shard_write_flush(self._ctx))

    def timings(self) -> tuple:
        """(ms_front_kernel, ms_host_call, ms_host_codes, ms_host_layout, ms_aq)
        of the last encode -- the per-frame subset of :meth:`stats` without its
        copies."""
        s = _Stats()
        _check(load().jxg_get_stats(self._ctx, ctypes.byref(s)))
        return s.ms_front_kernel, s.ms_host_call, s.ms_host_codes, s.ms_host_layout, s.ms_aq

    def stats(self) -> dict:
        s = _Stats()
        _check(load().jxg_get_stats(self._ctx, ctypes.byref(s)))
        nb = s.xsize_blocks * s.ysize_blocks
        out = {k: getattr(s, k) for k in ("xsize", "ysize", "xsize_blocks", "ysize_blocks",
                                          "num_groups", "num_lf_groups", "global_scale",
                                          "quant_dc", "bytes", "ms_front", "ms_histogram",
                                          "ms_emit", "ms_assemble", "ms_total",
                                          "ms_host_call", "ms_host_codes",
                                          "ms_host_layout", "ms_front_kernel", "ms_aq")}
        if s.ac_tokens:
            out["ac_tokens"] = np.ctypeslib.as_array(s.ac_tokens, (s.num_groups * 3,)).reshape(-1, 3).copy()
        if s.ac_strategy:
            shp = (s.ysize_blocks, s.xsize_blocks)
            out["acs"] = np.ctypeslib.as_array(s.ac_strategy, (nb,)).reshape(shp).copy()
            out["qf"] = np.ctypeslib.as_array(s.quant_field, (nb,)).reshape(shp).copy()
            out["dc"] = np.ctypeslib.as_array(s.dc, (3 * nb,)).reshape((3,) + shp).copy()
            out["ac"] = np.ctypeslib.as_array(s.ac, (nb * 192,)).reshape(shp + (3, 64)).copy()
            if s.homogeneity:
                out["homog"] = np.ctypeslib.as_array(s.homogeneity, (nb * 3,)).reshape(shp + (3,)).copy()
        return out

    # ---- sharded encode (one context per rank; see jxg.dist) ----
    def shard_begin(self, ptr: int, width: int, height: int, rank: int, world: int,
                    d_hist: int, d_xbuf: int, row_stride: int | None = None):
        """Front end + merge + AC statistics of this rank's pass groups;
        d_hist / d_xbuf are device pointers (sizes: :func:`shard_sizes`)."""
        _check(load().jxg_shard_begin(self._ctx, ctypes.c_void_p(ptr), width, height,
                                      row_stride or width * 3, rank, world,
                                      ctypes.c_void_p(d_hist), ctypes.c_void_p(d_xbuf)))

    def shard_end(self, d_hist: int, d_xbuf: int) -> int:
        """After all-reduce(d_hist) and all-gather(d_xbuf): emit this rank's
        sections; returns the payload size (kept on the device, see
        :meth:`shard_payload`)."""
        n = ctypes.c_size_t()
        _check(load().jxg_shard_end(self._ctx, ctypes.c_void_p(d_hist), ctypes.c_void_p(d_xbuf),
                                    ctypes.byref(n)))
        return n.value

    def shard_payload(self, dst: int, on_device: bool = True):
        """Copy the last payload to `dst` (device or host pointer)."""
        _check(load().jxg_shard_payload(self._ctx, ctypes.c_void_p(dst), 1 if on_device else 0))

    def shard_payload_bytes(self, size: int) -> bytes:
        buf = (ctypes.c_uint8 * size)()
        self.shard_payload(ctypes.addressof(buf), on_device=False)
        return bytes(buf)

    def shard_assemble_device(self, d_base: int, offsets, sizes, copy: bool = True):
        """Payloads gathered in device memory (d_base + offsets[i]) -> codestream."""
        n = len(sizes)
        offs = (ctypes.c_size_t * n)(*offsets)
        szs = (ctypes.c_size_t * n)(*sizes)
        buf = _Buffer()
        _check(load().jxg_shard_assemble_device(self._ctx, ctypes.c_void_p(d_base), offs, szs, n,
                                                ctypes.byref(buf)))
        return self._take(buf) if copy else Codestream(buf)

    def shard_head(self) -> np.ndarray:
        """This rank's payload head (u32 words) after shard_end."""
        n = ctypes.c_size_t(0)
        _check(load().jxg_shard_head(self._ctx, None, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint32)
        _check(load().jxg_shard_head(self._ctx, out.ctypes.data, ctypes.byref(n)))
        return out

    def shard_write_host(self, heads, dst_ptr: int, dst_size: int):
        """Write this rank's sections (and, on rank 0, headers + TOC) into the
        shared host buffer at dst_ptr; returns (ok, total codestream bytes) --
        ok False when dst_size < total (nothing written)."""
        return self._write(load().jxg_shard_write_host, heads, dst_ptr, dst_size)

    def _write(self, fn, heads, dst_ptr: int, dst_size: int):
        heads = [np.ascontiguousarray(h, dtype=np.uint32) for h in heads]
        n = len(heads)
        ptrs = (ctypes.c_void_p * n)(*[h.ctypes.data for h in heads])
        words = (ctypes.c_size_t * n)(*[h.size for h in heads])
        total = ctypes.c_size_t(0)
        st = fn(self._ctx, ptrs, words, n, ctypes.c_void_p(dst_ptr), dst_size, ctypes.byref(total))
        if st == -1 and total.value > dst_size:
            return False, total.value
        _check(st)
        return True, total.value

    def homogeneity_map(self, xyb: np.ndarray, distance: float, flags: int = 0):
        """Thesis selector over a (3, H, W) float32 XYB frame (H, W multiples of 8)."""
        xyb = np.ascontiguousarray(xyb, dtype=np.float32)
        _, ys, xs = xyb.shape
        r3 = np.zeros((ys // 8, xs // 8, 3), dtype=np.float32)
        t = np.zeros((ys // 8, xs // 8), dtype=np.uint8)
        _check(load().jxg_homogeneity_map(self._ctx, xyb.ctypes.data, xs, ys, distance, flags,
                                          r3.ctypes.data, t.ctypes.data))
        return r3, t

    def warmup(self, width: int, height: int):
        """jxg_warmup: allocate this context's buffers for width x height and
        load every kernel (one synthetic frame, result discarded)."""
        _check(load().jxg_warmup(self._ctx, width, height))

    def synth_device(self, ptr: int, width: int, height: int, seed: int,
                     row_stride: int | None = None):
        """Fill device memory with the benchmark's synthetic RGB8 frame
        (jxg.synth.synth_rgb8 bytes) on this context's stream."""
        _check(load().jxg_synth_rgb8_device(self._ctx, ctypes.c_void_p(ptr), width, height,
                                            row_stride or width * 3,
                                            seed & 0xFFFFFFFFFFFFFFFF))

    def compare(self, orig: np.ndarray, comp: np.ndarray, ssim: bool = True) -> dict:
        """Decode-side quality on the GPU (jxg_compare_rgb8): orig / comp are
        (H, W, 3) uint8 (comp = the decoded image).  Returns sse, samples, mse,
        psnr (image_reader.rs:555-606) and ssim (metrics.rs:55-84 counterpart)."""
        o = np.asarray(orig)
        c = np.asarray(comp)
        if o.shape != c.shape or o.ndim != 3 or o.shape[2] != 3:
            raise ValueError("orig / comp must both be (H, W, 3) uint8")
        o = np.ascontiguousarray(o, dtype=np.uint8)
        c = np.ascontiguousarray(c, dtype=np.uint8)
        h, w = o.shape[:2]
        q = _Quality()
        _check(load().jxg_compare_rgb8(self._ctx, o.ctypes.data, w * 3, c.ctypes.data, w * 3, w, h,
                                       1 if ssim else 0, ctypes.byref(q)))
        return {"sse": q.sse, "samples": q.samples, "mse": q.mse, "psnr": q.psnr, "ssim": q.ssim}

    def compare_device(self, d_orig: int, d_comp: int, width: int, height: int,
                       orig_stride: int | None = None, comp_stride: int | None = None,
                       ssim: bool = True) -> dict:
        """Same on device-resident RGB8 (e.g. torch tensors' data_ptr())."""
        q = _Quality()
        _check(load().jxg_compare_rgb8_device(
            self._ctx, ctypes.c_void_p(d_orig), orig_stride or width * 3, ctypes.c_void_p(d_comp),
            comp_stride or width * 3, width, height, 1 if ssim else 0, ctypes.byref(q)))
        return {"sse": q.sse, "samples": q.samples, "mse": q.mse, "psnr": q.psnr, "ssim": q.ssim}


# ---------------------------------------------------------------------------
# sharding helpers (host side; no device needed)
# ---------------------------------------------------------------------------
def shard_sizes(width: int, height: int, world: int):
    """(AC histogram words, record buffer bytes) of a sharded encode: the
    capacity of the send and of the receive buffer (largest of any rank)."""
    hw, sb = ctypes.c_size_t(), ctypes.c_size_t()
    _check(load().jxg_shard_sizes(width, height, world, ctypes.byref(hw), ctypes.byref(sb)))
    return hw.value, sb.value


def shard_exchange(width: int, height: int, world: int, rank: int):
    """(send bytes per peer, receive bytes per peer) of this rank's record
    exchange (an all_to_all with these splits)."""
    snd = (ctypes.c_size_t * world)()
    rcv = (ctypes.c_size_t * world)()
    _check(load().jxg_shard_exchange(width, height, world, rank, snd, rcv))
    return [int(x) for x in snd], [int(x) for x in rcv]


def shard_assemble(payloads) -> bytes:
    """Payloads of ranks 0..world-1 -> codestream (host only)."""
    n = len(payloads)
    keep = [np.frombuffer(bytes(p), dtype=np.uint8) for p in payloads]
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * n)(
        *[k.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) for k in keep])
    sizes = (ctypes.c_size_t * n)(*[k.size for k in keep])
    buf = _Buffer()
    _check(load().jxg_shard_assemble(ptrs, sizes, n, ctypes.byref(buf)))
    return Encoder._take(buf)


def group_count(width: int, height: int) -> int:
    return ((width + 255) // 256) * ((height + 255) // 256)


def lf_group_count(width: int, height: int) -> int:
    return ((width + 2047) // 2048) * ((height + 2047) // 2048)


def shard_plan(width: int, height: int, world: int):
    """The partition of a sharded encode (jxg_shard_plan; include/jxg.h):
    (owner rank of every pass group, owner rank of every LF group, kind) --
    kind 0 contiguous ranges, 1 whole LF groups per rank, 2 ranges with the
    per-block record exchange."""
    ng, nlf = group_count(width, height), lf_group_count(width, height)
    go = np.zeros(ng, dtype=np.uint32)
    lo = np.zeros(nlf, dtype=np.uint32)
    kind = ctypes.c_int(0)
    _check(load().jxg_shard_plan(width, height, world, go.ctypes.data, lo.ctypes.data,
                                 ctypes.byref(kind)))
    return go.tolist(), lo.tolist(), kind.value


def lf_owners(width: int, height: int, world: int) -> list:
    """Owner rank of every LF group in a sharded encode (jxg_shard_plan)."""
    return shard_plan(width, height, world)[1]


def shard_sections(width: int, height: int, rank: int, world: int, ans: bool = False):
    """TOC indices of the sections rank `rank` of `world` produces: LfGlobal on
    rank 0, the LF groups it owns, its pass groups (jxg_shard_plan), and on
    rank 0 HfGlobal -- except with ANS over several ranks, where HfGlobal is
    written at assembly from the ranks' HF presets (version-2 payload heads)."""
    go, lo, _ = shard_plan(width, height, world)
    nlf = len(lo)
    ids = [0] if rank == 0 else []
    ids += [1 + lg for lg in range(nlf) if lo[lg] == rank]
    if rank == 0 and not (ans and world > 1):
        ids.append(1 + nlf)
    ids += [2 + nlf + g for g in range(len(go)) if go[g] == rank]
    return ids


def make_payload(rank: int, world: int, width: int, height: int, sections) -> bytes:
    """The shard payload format of jxg_host.cpp (``JXGS`` v1) for a list of
    (TOC index, bytes) -- used by tests to feed jxg_shard_assemble."""
    head = np.array([0x5347584A, 1, rank, world, width, height, len(sections)] +
                    [v for i, b in sections for v in (i, len(b))], dtype="<u4").tobytes()
    return head + b"".join(b for _, b in sections)


# ---------------------------------------------------------------------------
# harness mirror (benchmark-jpegxl)
# ---------------------------------------------------------------------------
def _rust_plain(digits_repr: str) -> str:
    """Shortest round-trip digits (Python repr) -> Rust's exponent-free form."""
    s = digits_repr
    neg = s.startswith("-")
    if neg:
        s = s[1:]
    if "e" in s or "E" in s:
        mant, exp = s.lower().split("e")
        e = int(exp)
        if "." in mant:
            ip, fp = mant.split(".")
        else:
            ip, fp = mant, ""
        point = len(ip) + e  # position of the decimal point within ip + fp
        allds = ip + fp
        if point <= 0:
            s = "0." + "0" * (-point) + allds.lstrip("0")
        elif point >= len(allds):
            s = allds + "0" * (point - len(allds))
        else:
            s = allds[:point] + "." + allds[point:]
    if s.endswith(".0"):
        s = s[:-2]
    return ("-" if neg else "") + s


def rust_f64(v: float) -> str:
    """Rust ``format!("{}", f64)`` / ``f64::to_string``: shortest round-trip
    digits, never an exponent (1.0 -> "1", 1e-7 -> "0.0000001", 1e20 ->
    "100000000000000000000"), "NaN", "inf", "-inf"."""
    v = float(v)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "inf" if v > 0 else "-inf"
    if v == 0.0:
        return "-0" if math.copysign(1.0, v) < 0 else "0"
    return _rust_plain(repr(v))


def rust_f32(v: float) -> str:
    """Rust ``f32::to_string`` (the CSV's Distance column, csv_writer.rs:27):
    the shortest digits that round-trip through f32."""
    f = np.float32(v)
    if np.isnan(f):
        return "NaN"
    if np.isinf(f):
        return "inf" if f > 0 else "-inf"
    if f == 0:
        return "-0" if np.signbit(f) else "0"
    return _rust_plain(np.format_float_positional(f, unique=True, trim="-"))


def comp_image_name(stem: str, distance: float, effort: int) -> str:
    """benchmark.rs:644-650: ``{stem}-{distance}-{effort}.jxl``."""
    return "%s-%s-%d.jxl" % (stem, rust_f64(distance), effort)


def execute_cjxl(input_file: str, output_file: str, distance: float, effort: int,
                 proposals: str = "none", device: int = 0):
    """DockerManager::execute_cjxl (docker_manager.rs:100-137) with the GPU
    encoder in place of ``/libjxl/build/tools/cjxl``."""
    d = os.path.dirname(output_file)
    if d:
        os.makedirs(d, exist_ok=True)
    if not os.path.exists(CLI_PATH):
        raise JxgError("jxg_cjxl not built at %s" % CLI_PATH)
    args = [CLI_PATH, input_file, output_file, "--distance=%s" % rust_f64(distance),
            "--effort=%d" % effort, "--proposals=%s" % proposals, "--device=%d" % device]
    p = subprocess.run(args, capture_output=True, text=True)
    if p.returncode == 0:
        return True, p.stdout
    return False, p.stderr or p.stdout


def calculate_mse(orig: np.ndarray, comp: np.ndarray) -> float:
    """image_reader.rs:569-593: f64 sum of squared sample differences / count."""
    o = np.asarray(orig, dtype=np.float64).ravel()
    c = np.asarray(comp, dtype=np.float64).ravel()
    if o.size != c.size:
        raise ValueError("sample count mismatch")
    return float(np.sum((o - c) ** 2) / o.size)


def calculate_psnr(mse: float, max_value: float = 255.0) -> float:
    """image_reader.rs:604-606."""
    return 10.0 * math.log10((max_value * max_value) / mse) if mse > 0 else float("inf")
