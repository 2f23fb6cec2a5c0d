#!/usr/bin/env python3
"""Benchmark: MPix/s of VarDCT encode at d1.0 on synthetic 8K RGB (BASELINE.json
metric), device-resident RGB8 in HBM -> complete .jxl bytes in host memory.

  python bench.py --gpus N --steps K --warmup W [--mode shard|replica]
                  [--scaling strong|weak] [--coder prefix|ans] [--config C]

One step = one full encode (front end + merge stage, token statistics, entropy
codes, bit emission, assembly, D2H of the codestream).  The AC stream is
ANS-coded by default (libjxl's e7 entropy coder; --coder prefix for prefix
codes).  Single-GPU and replica steps go through the library's streaming entry
points (jxg_submit_rgb8_device / jxg_receive: a one-thread software pipeline
inside the library in which the rANS chains of earlier frames run under the
transform kernels of later ones); the timed region ends when the last
codestream of the K steps is in host memory.

N = 1: one 7680x4320 frame per step (BASELINE config 2's frame on one GPU).
N > 1 (launched by torch.distributed.run, backend nccl = RCCL):
  shard   (default) -- group sharding with the real exchange
          (jxg/dist.py) and assembly (--assembly host: every rank DMAs its
          sections into one /dev/shm codestream buffer of the node, rank 0
          writes headers + TOC; --assembly device: payload gather to rank 0):
            --scaling strong (default): ONE 7680x4320 frame per step split
              over the N ranks -- BASELINE config 2 as written;
            --scaling weak: one frame of N stacked 8K frames (every rank owns
              one 8K frame's worth of groups).
          The codestream is byte-identical to a single-GPU encode of the same
          frame (tests/test_gpu_shard.py).
  replica -- every rank encodes its own 8K frame (frame-level data
          parallelism, no data-path collective).
Timing: barrier + synchronize on both sides of the K steps, max over ranks.
--streams S (non-shard modes) runs S concurrent encoders per GPU (one host
thread, context and HIP stream each; the K frames split between them) through
the one-at-a-time entry point instead (--no-pipeline: S = 1 of those).

The JSON line also carries:
  roofline     -- the fused front kernel (XYB + homogeneity + AQ + 8x8 ACS +
                  DCT + quant): SURVEY.md §8(d)'s algorithmic bytes (15.078
                  B/px) per launch / its HIP-event duration (its own events, on
                  the encoder's stream) vs 8.0 TB/s; the design's own bytes
                  and the PMC-measured HBM traffic (profiles/) beside it;
  alt_coder    -- the same workload with the other AC entropy coder;
  quality      -- decoded PSNR / bpp of a 1920x1080 crop of the bench frame and
                  of a 1920x1080 photographic-like frame (untimed);
  cpu_baseline -- the oracle/ C restatement with OpenMP on the host's cores
                  (libjxl absent on the box) on the same frame, and whether
                  its bytes equal the GPU's.
"""
import argparse
import json
import os
import sys
import time

# The library's streaming pipeline runs up to 12 encoder lanes (7 at 8K, 12
# for 4K and smaller), one HIP stream each; HIP maps streams onto
# GPU_MAX_HW_QUEUES hardware queues per process (the box exports 4, one of them
# taken by torch's stream), and two lanes sharing a queue serialise their
# kernels.  Must be set before HIP initialises (JXG_BENCH_HW_QUEUES overrides
# it for experiments; at most 32).
os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, int(os.environ.get("JXG_BENCH_HW_QUEUES", "16"))))

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before libjxg: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import jxg  # noqa: E402
from jxg.synth import CONFIGS, SEED_BASE, synth_rgb8_device  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


SURVEY_BYTES_PER_PX = 15.078  # RGB8 3 + quant field/ACS 5/64 + 3 x int32 12


def front_bytes_survey(w, h):
    """SURVEY.md §8(d)'s algorithmic bytes of the fused XYB + DCT + quant
    kernel: read RGB8 (3 B/px), read the per-block quant field and ACS
    (5/64 B/px), write 3 x int32 coefficients (12 B/px) = 15.078 B/px.  The
    roofline fraction is priced on these bytes."""
    return SURVEY_BYTES_PER_PX * w * h


def front_bytes_design(w, h, effort):
    """The bytes this design's front kernel moves per launch (reported beside
    the §8(d) figure, not used for the fraction): RGB8 read (3 B/px), int16
    coefficients (6 B/px), per 8x8 block 3 x int32 DC + strategy + quant field
    + 3 x u16 non-zero counts (20 B); with the merge stage (effort >= 5) the
    XYB tile copy for merge_eval (12 B/px) and the per-block estimate (4 B)."""
    bxs, bys = (w + 7) // 8, (h + 7) // 8
    px = (bxs * 8) * (bys * 8)
    b = 3 * w * h + 6 * px + 20 * bxs * bys
    if effort >= 5:
        b += 12 * px + 4 * bxs * bys
    return b


def load_pmc_traffic(workload):
    p = os.path.join(ROOT, "profiles", "front_pmc_%s.json" % workload)
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except Exception:
        return None


def load_front_valu(workload):
    """PMC VALU-issue fraction of the front kernel (profiles/front_pmc_*.json)"""
    p = os.path.join(ROOT, "profiles", "front_pmc_%s.json" % workload)
    try:
        with open(p) as f:
            return json.load(f).get("valu_issue_frac")
    except Exception:
        return None


def load_merge_pmc(workload):
    p = os.path.join(ROOT, "profiles", "merge_pmc_%s.json" % workload)
    try:
        with open(p) as f:
            return json.load(f).get("valu_issue_frac")
    except Exception:
        return None


def cpu_threads():
    """host threads for the CPU baseline: the process's CPU affinity, capped at
    16 (the GPU box's CPU share per GPU; its nproc shows the whole host)"""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(img, distance, effort, proposals, coder, gpu_bytes):
    """The oracle/ C restatement (libjxl/cjxl are absent on the box: probe in
    profiles/r02a/probe.txt) timed on the host with OpenMP over
    cpu_threads() threads, on the same frame and settings as the GPU line.
    Its codestream is also compared with the GPU's (byte-exact parity)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi  # the checker, timed here only as the reported baseline

    oracle_ffi.build()
    n = oracle_ffi.set_threads(cpu_threads())
    t = time.perf_counter()
    r = oracle_ffi.encode(img, distance, effort, proposals, coder)
    dt = time.perf_counter() - t
    h, w, _ = img.shape
    return {"value": round(w * h / 1e6 / dt, 3), "unit": "MPix/s", "cores": n, "kind": "port",
            "sample": "one full %dx%d frame (the bench frame), oracle/ C restatement with OpenMP "
                      "(libjxl/cjxl absent on the box), %.2f s" % (w, h, dt),
            "bytes_equal_gpu": gpu_bytes is not None and r.bytes == gpu_bytes}


def quality_probe(enc, img, distance, effort):
    """Decoded quality at the bench settings (untimed): the top-left 1920x1080
    crop of the bench frame, encoded on the GPU, decoded by oracle/jxl_decode.py
    (no djxl on the box), PSNR by the reference formula (image_reader.rs:
    569-606); the full 8K frame takes minutes in the Python decoder."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import jxl_decode

    crop = np.ascontiguousarray(img[:1080, :1920])
    data = enc.encode(crop)
    dec = jxl_decode.decode(data).rgb
    mse = jxg.calculate_mse(crop, dec)
    pc = [round(jxg.calculate_psnr(jxg.calculate_mse(crop[..., c:c + 1], dec[..., c:c + 1])), 3)
          for c in range(3)]
    res = {"frame": "top-left 1920x1080 crop of the bench frame, d%g e%d" % (distance, effort),
           "psnr_db": round(jxg.calculate_psnr(mse), 3), "psnr_rgb_db": pc,
           "bpp": round(len(data) * 8.0 / (1920 * 1080), 4),
           "decoder": "oracle/jxl_decode.py (djxl absent)"}
    # the same settings on photographic-like content (smooth fields, soft
    # edges, band-limited texture: jxg.synth.natural_rgb8), where the rate-
    # distortion behaviour of a d1 encoder is meaningful; the bench frame is a
    # throughput workload with noise-heavy regions
    from jxg.synth import natural_rgb8
    nat = natural_rgb8(1920, 1080, 3)
    nd = enc.encode(nat)
    ndec = jxl_decode.decode(nd).rgb
    res["natural"] = {"frame": "natural_rgb8(1920, 1080, seed 3)",
                      "psnr_db": round(jxg.calculate_psnr(jxg.calculate_mse(nat, ndec)), 3),
                      "bpp": round(len(nd) * 8.0 / (1920 * 1080), 4)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 frames by default: the timed region of a streaming run includes one
    # pipeline fill + drain (about one frame's latency, ~22 ms at 8K ANS), which
    # costs 16 % of a 20-frame run and 3 % of a 100-frame one
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, help="BASELINE config index (2 = 8K)")
    ap.add_argument("--distance", type=float, default=1.0)
    ap.add_argument("--effort", type=int, default=7)
    ap.add_argument("--proposals", type=int, default=0)
    ap.add_argument("--mode", choices=("shard", "replica"), default="replica",
                    help="N > 1: replica = every rank streams its own frames through the "
                         "pipelined entry points (frame-level data parallelism, no data-path "
                         "collective); shard = one frame's pass groups split over the ranks")
    ap.add_argument("--alt-shard", type=int, default=1,
                    help="replica mode, N > 1: also time the sharded strong-scaling encode of "
                         "one frame over the N ranks (reported under 'sharded')")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="shard mode: strong = ONE frame of the config split over the N ranks "
                         "(BASELINE config 2 as written); weak = a frame of N stacked config "
                         "frames (every rank owns one frame's worth of groups)")
    ap.add_argument("--assembly", choices=("host", "device"), default="host",
                    help="shard mode: host = every rank DMAs its sections into one /dev/shm "
                         "buffer (rank 0 adds headers + TOC); device = payload gather to rank 0, "
                         "device assembly, one D2H")
    ap.add_argument("--coder", choices=("prefix", "ans"), default="ans",
                    help="AC entropy coder (libjxl codes with ANS at e7)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one-at-a-time jxg_encode_rgb8_device calls instead of the streaming "
                         "entry points")
    ap.add_argument("--streams", type=int, default=1,
                    help="concurrent encoders per GPU (replica / N=1 mode): one host thread, "
                         "context and HIP stream each; a step is still one frame")
    ap.add_argument("--alt-coder", type=int, default=1,
                    help="also time the other AC coder (reported under 'alt_coder'; 0 = off)")
    ap.add_argument("--alt-thesis", type=int, default=1,
                    help="also time the workload with the thesis proposals P+F "
                         "(reported under 'thesis_proposals'; 0 = off)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-quality", action="store_true",
                    help="skip the untimed decode-PSNR probe")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # JXG_DIST_BACKEND=gloo rehearses the multi-rank path with host-staged
    # collectives (several ranks may then share one device)
    backend = os.environ.get("JXG_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local)
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    name, w, h, nframes = CONFIGS[args.config]
    shard0 = world > 1 and args.mode == "shard"
    shard = shard0
    strong = shard and args.scaling == "strong"
    # inputs generated on the device (jxg_synth_rgb8_device: the bytes of
    # jxg.synth.synth_rgb8, without minutes of numpy at 8K / 16K)
    d_img = synth_rgb8_device(w, h, SEED_BASE + args.config + (0 if shard else rank), local)
    img = d_img.cpu().numpy() if world == 1 else None  # quality probe / CPU baseline
    # batch configs (64 x 1080p): a step is the whole batch of distinct frames,
    # device-resident
    frames = 1 if shard else nframes
    d_imgs = [d_img] + [synth_rgb8_device(w, h, SEED_BASE + args.config + f, local)
                        for f in range(1, frames)]
    pipeline = not shard and not args.no_pipeline
    ptrs = [t.data_ptr() for t in d_imgs]
    fh = h
    if shard and not strong:
        # one frame of N stacked config frames: every rank owns 1/N of its groups
        fh = h * world
        d_img = d_img.repeat(world, 1, 1).contiguous()
    torch.cuda.synchronize()

    def run(coder, nstreams, proposals=None, as_shard=None, pipe=None):
        """Warm up, then time args.steps frames over `nstreams` concurrent
        encoders (one host thread, context and HIP stream each)."""
        nonlocal shard, pipeline, frames, d_img
        pipe_saved = pipeline
        if pipe is not None:
            pipeline = pipe
        if as_shard is not None:  # the sharded strong-scaling line of a replica run
            shard, pipeline, frames = as_shard, False, 1
            d_img = synth_rgb8_device(w, h, SEED_BASE + args.config, local)
        flags = jxg.FLAG_ANS if coder == "ans" else 0
        props = args.proposals if proposals is None else proposals
        encs = [jxg.Encoder(distance=args.distance, effort=args.effort,
                            proposals=props, device=local, flags=flags)
                for _ in range(nstreams)]
        bufs = {}
        host = None
        if shard and args.assembly == "host":
            from jxg.dist import SharedHostBuffer
            if SharedHostBuffer.single_node():
                host = SharedHostBuffer(rank, world)
            # else: ranks on several nodes -> device assembly (payload gather)

        def step(e, k=0):
            if shard:
                from jxg.dist import encode_sharded
                return encode_sharded(e, d_img, w, fh, rank, world, bufs=bufs, copy=False,
                                      host=host)
            return e.encode_device(d_imgs[k % frames].data_ptr(), w, fh, copy=False)

        rec = {"front_ms": [], "host_ms": [], "sizes": [], "last": None}

        def took(e, k, out):
            t = e.timings()
            rec["front_ms"].append(t[0])
            rec["host_ms"].append(t[1:])
            rec["sizes"].append(len(out) if out is not None else 0)
            if k % frames == 0:
                rec["last"] = out

        def worker(e, ks):
            # the codestream ends in (pinned) host memory; ctypes calls release
            # the GIL, so the encoders' host work and HIP streams overlap
            if pipeline:
                # streaming entry points: submit every frame, receive each
                # codestream as soon as it is done (more than the library's
                # pipeline depth pending => the oldest is complete)
                got = 0
                for k in ks:
                    e.submit_device(d_imgs[k % frames].data_ptr(), w, fh)
                    while e.pending() > 16:
                        took(e, got, e.receive(copy=False))
                        got += 1
                while e.pending():
                    took(e, got, e.receive(copy=False))
                    got += 1
                return
            for k in ks:
                took(e, k, step(e, k))

        for e in encs:  # contexts warmed one after another
            if pipeline:
                # at least 16 frames: every lane of the library's pipeline (up
                # to 12) allocates its buffers on its first frame, which must
                # not land in the timed region
                worker(e, range(max(max(args.warmup, 1) * frames, 16)))
            else:
                for _ in range(args.warmup):
                    step(e)
        for key in ("front_ms", "host_ms", "sizes"):
            rec[key] = []

        total = args.steps * frames
        share = [list(range(i, total, nstreams)) for i in range(nstreams)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if nstreams == 1:
            worker(encs[0], range(total))
        else:
            import threading
            ths = [threading.Thread(target=worker, args=(e, n)) for e, n in zip(encs, share)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        rec["dt"] = dt
        rec["st"] = encs[0].stats()
        last = rec["last"]
        rec["last"] = last.tobytes() if hasattr(last, "tobytes") else last
        for e in encs[1:]:
            e.close()
        rec["enc"] = encs[0]
        if host is not None:
            dist.barrier()
            host.close()
        pipeline = pipe_saved
        return rec

    nstreams = 1 if shard else max(1, args.streams)
    R = run(args.coder, nstreams)
    dt, front_ms, host_ms, st = R["dt"], R["front_ms"], R["host_ms"], R["st"]
    nbytes = R["sizes"][-1] if R["sizes"] else 0
    px_step = w * fh * (1 if shard else world) * frames
    alt = None
    other = "prefix" if args.coder == "ans" else "ans"
    if not shard and args.alt_coder > 0:
        # the same workload with the other AC entropy coder
        A = run(other, nstreams)
        A["enc"].close()
        alt = {"coder": other, "streams_per_gpu": nstreams, "pipeline": pipeline,
               "value": round(px_step * args.steps / A["dt"] / 1e6, 2),
               "ms_per_step": round(A["dt"] * 1e3 / args.steps, 3),
               "ms_latency": round(sum(x[0] for x in A["host_ms"]) / len(A["host_ms"]), 3),
               "bytes_per_frame": A["sizes"][-1],
               "bpp": round(A["sizes"][-1] * 8.0 / (w * fh), 4)}
    sharded = None
    if world > 1 and not shard and args.alt_shard:
        # the same frame's groups split over the N ranks (strong scaling,
        # one frame per step, SURVEY §8e exchange + host assembly)
        S = run(args.coder, 1, as_shard=True)
        if rank == 0:
            sharded = {"mode": "shard", "scaling": "strong", "coder": args.coder,
                       "value": round(w * h * args.steps / S["dt"] / 1e6, 2),
                       "ms_per_step": round(S["dt"] * 1e3 / args.steps, 3),
                       "bytes_per_frame": S["sizes"][-1]}
        S["enc"].close()
        shard, pipeline, frames = False, not args.no_pipeline, nframes
    iso = None
    if pipeline:
        # the kernels alone on the GPU (one-at-a-time encodes, same coder): the
        # front kernel's roofline, the rANS chain kernel's duration
        iso = run(args.coder, 1, pipe=False)
        iso["enc"].close()
    thesis = None
    if not shard and args.alt_thesis and args.proposals != 3:
        # the thesis proposals P + F (combined.diff) on the same workload:
        # the homogeneity selector in the front kernel, hook F on every
        # 8x8 and merge candidate
        T = run(args.coder, nstreams, proposals=3)
        T["enc"].close()
        thesis = {"proposals": "P+F (combined.diff)",
                  "value": round(px_step * args.steps / T["dt"] / 1e6, 2),
                  "ms_per_step": round(T["dt"] * 1e3 / args.steps, 3),
                  "ms_front_kernel": round(sum(T["front_ms"]) / len(T["front_ms"]), 4),
                  "bytes_per_frame": T["sizes"][-1],
                  "bpp": round(T["sizes"][-1] * 8.0 / (w * fh), 4)}
    if rank == 0:
        ms_step = dt * 1e3 / args.steps
        frame_px = w * fh
        value = px_step * args.steps / dt / 1e6
        # roofline of the front kernel over this rank's launch (its tiles)
        fw, fhh = (w, fh // world) if shard else (w, fh)
        fb = front_bytes_survey(fw, fhh)
        fms_pipe = sum(front_ms) / len(front_ms)
        fms = sum(iso["front_ms"]) / len(iso["front_ms"]) if iso else fms_pipe
        achieved = fb / (fms * 1e-3) / 1e9 if fms > 0 else 0.0
        coder_desc = "%s-coded" % args.coder
        if shard:
            workload = ("%s: %dx%d RGB8 (synth_rgb8%s), VarDCT d%g e%d, proposals=%d, %s, "
                        "256x256 groups sharded over %d ranks (%s scaling), %s assembly"
                        % (name, w, fh, "" if strong else ", config frame stacked %d times" % world,
                           args.distance, args.effort, args.proposals, coder_desc, world,
                           args.scaling, args.assembly))
            par = "group-shard%d" % world
        else:
            workload = ("%s %dx%d RGB8 (synth_rgb8), VarDCT d%g e%d, proposals=%d, %s, "
                        "%d distinct frame(s) per step, %s"
                        % (name, w, h, args.distance, args.effort, args.proposals, coder_desc,
                           frames, "streaming entry points (jxg_submit_rgb8_device / "
                           "jxg_receive, one host thread)" if pipeline else
                           "%d concurrent encoder stream(s) per rank" % nstreams))
            par = "frame-dp%d" % world
        label = {"8k": "8K", "4k": "4K", "16k": "16384x16384", "cpu512": "512x512",
                 "1080p_x64": "64 x 1080p"}.get(name, name)
        res = {
            "metric": "MPix/s VarDCT encode @ d%s, %s RGB" % (
                "1.0" if args.distance == 1.0 else "%g" % args.distance, label),
            "value": round(value, 2),
            "unit": "MPix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": workload, "global_batch": 1 if shard else world * frames,
                       "parallelism": par},
            "streams_per_gpu": nstreams,
            "pipeline": pipeline,
            "ms_latency": round(sum(x[0] for x in host_ms) / len(host_ms), 3),
            "bytes_per_frame": nbytes,
            "bpp": round(nbytes * 8.0 / frame_px, 4),
            "stages_ms": {k: round(st[k], 4) for k in ("ms_front_kernel", "ms_front",
                                                       "ms_histogram", "ms_emit",
                                                       "ms_assemble", "ms_total")},
            "host_ms": {k: round(sum(x[i] for x in host_ms) / len(host_ms), 4)
                        for i, k in enumerate(("call", "codes", "layout"))},
            "roofline": {"kernel": "front_kernel", "bound": "hbm",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_pmc_traffic(name) if world == 1 else None,
                         "algorithmic_bytes": int(fb),
                         "bytes_per_px": SURVEY_BYTES_PER_PX,
                         "design_bytes": front_bytes_design(fw, fhh, args.effort),
                         "avg_ms": round(fms, 4),
                         # the kernel is VALU-bound (the six-candidate 8x8 search):
                         # its PMC VALU issue rate beside the HBM fraction
                         "valu_issue_frac_pmc": load_front_valu(name) if world == 1 else None,
                         "measured": ("one-at-a-time encodes (the kernel alone on the GPU); "
                                      "under the pipeline, sharing the GPU with rANS chains: "
                                      "%.4f ms" % fms_pipe) if iso else "timed region"},
            # the merge stage is latency-bound (VALU issue 35 %, waves waiting
            # on memory / LDS 41 % of their lifetime): its live time and the
            # PMC-measured VALU issue rate
            "merge_stage": {"kernels": "merge_eval + merge_resolve + merge_write",
                            "bound": "latency",
                            "avg_ms": round((iso["st"] if iso else st)["ms_front"] -
                                            (iso["st"] if iso else st)["ms_front_kernel"], 4),
                            "valu_issue_frac_pmc": load_merge_pmc(name) if world == 1 else None},
        }
        if iso is not None and args.coder == "ans":
            # the rANS chain: one serial state recurrence per pass group (the
            # format's), so its kernel time is set by the group with the most
            # tokens x the per-step latency (latency-bound, not HBM / MFMA)
            tok = np.asarray(iso["st"]["ac_tokens"]).reshape(-1, 3).sum(axis=1)
            ms_emit = iso["st"]["ms_emit"]
            res["ans_chain"] = {"kernel": "ans_encode_kernel (+ LF emission in the same span)",
                                "bound": "latency (dependent LDS lookups)",
                                "ms_emit_isolated": round(ms_emit, 4),
                                "tokens_max_group": int(tok.max()),
                                "tokens_mean_group": round(float(tok.mean()), 1),
                                "ns_per_token_max_group": round(ms_emit * 1e6 / max(1, tok.max()), 2)}
        if alt is not None:
            res["alt_coder"] = alt
        if thesis is not None:
            res["thesis_proposals"] = thesis
        if sharded is not None:
            res["sharded"] = sharded
        if world == 1 and not args.no_quality:
            res["quality"] = quality_probe(R["enc"], img, args.distance, args.effort)
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(img, args.distance, args.effort, args.proposals,
                                               1 if args.coder == "ans" else 0,
                                               R["last"])
        print(json.dumps(res), flush=True)
    R["enc"].close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
