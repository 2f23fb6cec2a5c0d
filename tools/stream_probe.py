"""Throughput of the streamed paths in ONE process, for rocprofv3 (no
torch.distributed launcher in between):
  host   `world` contexts on one GPU play the ranks of the streamed-shard
         protocol (jxg_shard_submit_device / next_head / write_next), e.g. a
         1/8 slice: --world 1 --h 544
  plain  whole frames through jxg_submit_rgb8_device / jxg_receive, e.g.
         config 3's frames: --w 1920 --h 1080
  python tools/stream_probe.py --mode host --world 2 --frames 40"""
import argparse
import ctypes
import mmap
import os
import sys
import time

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("JXG_BENCH_HW_QUEUES", "16")
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..",
                                "jpeg-xl-lossy-image-compression-thesis_amd"))
import jxg  # noqa: E402
from jxg.synth import synth_rgb8_device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", choices=("plain", "host"), default="host")
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--frames", type=int, default=40)
ap.add_argument("--warmup", type=int, default=16)
ap.add_argument("--w", type=int, default=7680)
ap.add_argument("--h", type=int, default=4320)
ap.add_argument("--lanes", type=int, default=-1,
                help="lane cap per context (-1: jxg.dist.shared_gpu_lanes(world), 0: none)")
a = ap.parse_args()
w, h, W = a.w, a.h, a.world
ts = [synth_rgb8_device(w, h, 0x4A584C02 + 100 * k) for k in range(2)]
torch.cuda.synchronize()
encs = [jxg.Encoder(flags=jxg.FLAG_ANS) for _ in range(W)]
if a.lanes < 0:
    from jxg.dist import shared_gpu_lanes
    a.lanes = shared_gpu_lanes(W, int(os.environ["GPU_MAX_HW_QUEUES"])) or 0
for e in encs:
    e.set_pipeline_lanes(a.lanes)
depth = min(e.pipeline_depth(w, h, r, W) for r, e in enumerate(encs)) if a.mode == "host" \
    else encs[0].pipeline_depth(w, h)
stamps = []
sizes = []
tsub = [0.0]  # main thread: seconds inside submit calls


def timed_submit(fn, *args):
    t = time.perf_counter()
    fn(*args)
    tsub[0] += time.perf_counter() - t

if a.mode == "plain":
    # whole frames through the one-context streaming pipeline (config 3 shape
    # with --w 1920 --h 1080): the per-frame kernel sequence under rocprofv3
    e0 = encs[0]

    def take():
        cs = e0.receive(copy=False)
        sizes.append(len(cs))
        cs.release()
        stamps.append(time.perf_counter())

    def run(n):
        for k in range(n):
            timed_submit(e0.submit_device, ts[k % 2].data_ptr(), w, h)
            while e0.pending() > max(16, depth):  # bench.py's replica loop
                take()
        while e0.pending():
            take()
else:
    buf = np.zeros(w * h * 2 + (1 << 20), dtype=np.uint8)
    # page-locked like ShardStream's shared buffer (the writes are DMA)
    assert jxg.load().jxg_host_register(ctypes.c_void_p(buf.ctypes.data), buf.nbytes) == 0

    ttake = [0.0, 0.0]  # seconds in next_head, in write_next

    def take():
        t = time.perf_counter()
        heads = [e.shard_next_head() for e in encs]
        t1 = time.perf_counter()
        for e in encs:
            ok, tot = e.shard_write_next(heads, buf.ctypes.data, buf.size)
        t2 = time.perf_counter()
        ttake[0] += t1 - t
        ttake[1] += t2 - t1
        sizes.append(tot)
        stamps.append(t2)

    def run(n):
        for k in range(n):
            for r, e in enumerate(encs):
                timed_submit(e.shard_submit_device, ts[k % 2].data_ptr(), w, h, r, W)
            if encs[0].pending() >= depth:
                take()
        while encs[0].pending():
            take()

run(a.warmup)
torch.cuda.synchronize()
stamps.clear()
tsub[0] = 0.0
if a.mode == "host":
    ttake[0] = ttake[1] = 0.0
t0 = time.perf_counter()
run(a.frames)
if a.mode == "host":
    for e in encs:
        e.shard_write_flush()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
gaps = np.diff(np.array([t0] + stamps)) * 1e3
print("mode %s %dx%d world %d lanes cap %d depth %d: %.3f ms/frame, %.1f MPix/s, bytes %d; in submit "
      "%.3f ms/frame; receive gaps ms p50 %.3f p90 %.3f max %.3f"
      % (a.mode, w, h, W, a.lanes, depth, dt * 1e3 / a.frames, w * h * a.frames / dt / 1e6, sizes[-1],
         tsub[0] * 1e3 / a.frames, np.median(gaps), np.percentile(gaps, 90), gaps.max()),
      flush=True)
if a.mode == "host":
    print("  in next_head %.3f ms/frame, in write_next %.3f ms/frame"
          % (ttake[0] * 1e3 / a.frames, ttake[1] * 1e3 / a.frames), flush=True)
for e in encs:
    e.close()
