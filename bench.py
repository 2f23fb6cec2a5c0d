#!/usr/bin/env python3
"""Benchmark: MPix/s of VarDCT encode at d1.0 on synthetic 8K RGB (BASELINE.json
metric), device-resident RGB8 in HBM -> complete .jxl bytes in host memory.

  python bench.py --gpus N --steps K --warmup W [--mode shard|replica]

One step = one full encode (front end + merge stage, token statistics, prefix
codes, bit emission, assembly, D2H of the codestream).

N = 1: one 7680x4320 frame per step (BASELINE config 2's frame on one GPU).
N > 1 (launched by torch.distributed.run, backend nccl = RCCL):
  shard   (default) -- group sharding: ONE frame of 7680 x
          (4320 N) pixels per step -- every rank owns 1/N of its 256x256 pass
          groups, i.e. one 8K frame's worth of work (weak scaling) -- with
          the real exchange: all-reduce of the AC histogram, all-gather of the
          per-block DC/strategy records, then (--assembly host, default)
          all-gather of the payload heads and every rank's D2H of its own
          sections into one /dev/shm codestream buffer of the node (rank 0
          writes headers + TOC), or (--assembly device) gather of the section
          payloads and assembly on rank 0.  The codestream is byte-identical to a
          single-GPU encode of the same frame (tests/test_gpu_shard.py).
  replica -- every rank encodes its own 8K frame (frame-level data
          parallelism, no data-path collective).
Timing: barrier + synchronize on both sides of the K steps, max over ranks.
--streams S (non-shard modes) runs S concurrent encoders per GPU (one host
thread, context and HIP stream each; the K frames split between them).

The line's value is the prefix-coded encode (default --coder prefix, S = 1);
'ans_coder' reports the same workload with the ANS coder (libjxl's e7 entropy
coder) timed with --alt-ans-streams concurrent encoders, because each pass
group's rANS state chain is serial and latency-bound.

The JSON line also carries:
  roofline     -- the fused front kernel (XYB + homogeneity + AQ + 8x8 ACS +
                  DCT + quant): algorithmic bytes per launch / its HIP-event
                  duration (its own events, on the encoder's stream) vs 8.0
                  TB/s, plus PMC-measured HBM traffic from profiles/ when present;
  cpu_baseline -- the CPU oracle (scalar C port, 1 core) on the same frame.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd"))

import torch  # noqa: E402  (import before libjxg: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import jxg  # noqa: E402
from jxg.synth import CONFIGS, SEED_BASE, synth_rgb8  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def front_bytes_per_launch(w, h, effort):
    """Algorithmic HBM bytes of one front-kernel launch: RGB8 read (3 B/px),
    int16 coefficients written (3 ch x 2 B = 6 B/px), per 8x8 block 3 x int32
    DC + strategy + quant field + 2 B x 3 non-zero counts (20 B / 64 px); with
    the merge stage (effort >= 5) also the XYB tile copy (12 B/px) and the
    per-block estimate (4 B / 64 px)."""
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


def load_merge_pmc(workload):
    p = os.path.join(ROOT, "profiles", "merge_pmc_%s.json" % workload)
    try:
        with open(p) as f:
            return json.load(f).get("valu_issue_frac")
    except Exception:
        return None


def cpu_baseline(img, distance, effort):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi  # the checker, timed here only as the reported baseline

    oracle_ffi.build()
    t = time.perf_counter()
    oracle_ffi.encode(img, distance, effort, 0)
    dt = time.perf_counter() - t
    h, w, _ = img.shape
    return {"value": round(w * h / 1e6 / dt, 3), "unit": "MPix/s", "cores": 1, "kind": "port",
            "sample": "one full %dx%d frame, oracle/ C restatement (libjxl unavailable), %.1f s"
                      % (w, h, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, help="BASELINE config index (2 = 8K)")
    ap.add_argument("--distance", type=float, default=1.0)
    ap.add_argument("--effort", type=int, default=7)
    ap.add_argument("--proposals", type=int, default=0)
    ap.add_argument("--mode", choices=("shard", "replica"), default="shard")
    ap.add_argument("--assembly", choices=("host", "device"), default="host",
                    help="shard mode: host = every rank DMAs its sections into one /dev/shm "
                         "buffer (rank 0 adds headers + TOC); device = payload gather to rank 0, "
                         "device assembly, one D2H")
    ap.add_argument("--coder", choices=("prefix", "ans"), default="prefix",
                    help="AC entropy coder (libjxl codes with ANS at e7)")
    ap.add_argument("--streams", type=int, default=1,
                    help="concurrent encoders per GPU (replica / N=1 mode): one host thread, "
                         "context and HIP stream each; a step is still one frame")
    ap.add_argument("--alt-ans-streams", type=int, default=3,
                    help="also time the ANS coder with this many concurrent encoders "
                         "(reported under 'ans_coder'; 0 = off)")
    ap.add_argument("--alt-thesis", type=int, default=1,
                    help="also time the workload with the thesis proposals P+F "
                         "(reported under 'thesis_proposals'; 0 = off)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
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
    shard = world > 1 and args.mode == "shard"
    img = synth_rgb8(w, h, SEED_BASE + args.config + (0 if shard else rank))
    d_img = torch.from_numpy(img).to(dev)
    # batch configs (64 x 1080p): a step is the whole batch of distinct frames,
    # device-resident, split over the concurrent encoders
    frames = 1 if shard else nframes
    d_imgs = [d_img] + [torch.from_numpy(synth_rgb8(w, h, SEED_BASE + args.config + f)).to(dev)
                        for f in range(1, frames)]
    fh = h
    if shard:
        # one frame of N stacked 8K frames: every rank owns 1/N of its groups
        fh = h * world
        d_img = d_img.repeat(world, 1, 1).contiguous()
    torch.cuda.synchronize()

    def run(coder, nstreams, proposals=None):
        """Warm up, then time args.steps frames over `nstreams` concurrent
        encoders (one host thread, context and HIP stream each)."""
        flags = jxg.FLAG_ANS if coder == "ans" else 0
        props = args.proposals if proposals is None else proposals
        encs = [jxg.Encoder(distance=args.distance, effort=args.effort,
                            proposals=props, device=local, flags=flags)
                for _ in range(nstreams)]
        bufs = {}
        host = None
        if shard and args.assembly == "host":
            from jxg.dist import SharedHostBuffer
            host = SharedHostBuffer(rank, world)

        def step(e, k=0):
            if shard:
                from jxg.dist import encode_sharded
                return encode_sharded(e, d_img, w, fh, rank, world, bufs=bufs, copy=False,
                                      host=host)
            return e.encode_device(d_imgs[k % frames].data_ptr(), w, fh, copy=False)

        for e in encs:  # contexts warmed one after another
            for _ in range(args.warmup):
                step(e)
        rec = {"front_ms": [], "host_ms": [], "sizes": []}

        def worker(e, ks):
            # the codestream ends in (pinned) host memory; ctypes calls release
            # the GIL, so the encoders' host work and HIP streams overlap
            for k in ks:
                out = step(e, k)
                t = e.timings()
                rec["front_ms"].append(t[0])
                rec["host_ms"].append(t[1:])
                rec["sizes"].append(len(out) if out is not None else 0)

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
        for e in encs:
            e.close()
        if host is not None:
            dist.barrier()
            host.close()
        return rec

    nstreams = 1 if shard else max(1, args.streams)
    R = run(args.coder, nstreams)
    dt, front_ms, host_ms, st = R["dt"], R["front_ms"], R["host_ms"], R["st"]
    nbytes = R["sizes"][-1] if R["sizes"] else 0
    alt = None
    if not shard and args.alt_ans_streams > 0 and args.coder != "ans":
        # the same workload with the ANS coder (libjxl's e7 entropy coder):
        # its per-group rANS chain is latency-bound, so concurrent encoders
        # overlap it with the other frames' kernels
        A = run("ans", args.alt_ans_streams)
        alt = {"coder": "ans", "streams_per_gpu": args.alt_ans_streams,
               "value": round(w * fh * world * frames * args.steps / A["dt"] / 1e6, 2),
               "ms_per_step": round(A["dt"] * 1e3 / args.steps, 3),
               "ms_latency": round(sum(x[0] for x in A["host_ms"]) / len(A["host_ms"]), 3),
               "bytes_per_frame": A["sizes"][-1],
               "bpp": round(A["sizes"][-1] * 8.0 / (w * fh), 4)}
    thesis = None
    if not shard and args.alt_thesis and args.proposals != 3:
        # the thesis proposals P + F (combined.diff) on the same workload:
        # the homogeneity selector in the front kernel, hook F on every
        # 8x8 and merge candidate
        T = run(args.coder, 1, proposals=3)
        thesis = {"proposals": "P+F (combined.diff)",
                  "value": round(w * fh * world * frames * args.steps / T["dt"] / 1e6, 2),
                  "ms_per_step": round(T["dt"] * 1e3 / args.steps, 3),
                  "ms_front_kernel": round(sum(T["front_ms"]) / len(T["front_ms"]), 4),
                  "bytes_per_frame": T["sizes"][-1],
                  "bpp": round(T["sizes"][-1] * 8.0 / (w * fh), 4)}
    if rank == 0:
        ms_step = dt * 1e3 / args.steps
        frame_px = w * fh
        value = frame_px * (1 if shard else world) * frames * args.steps / dt / 1e6
        # roofline of the front kernel over this rank's launch (its tiles)
        fw, fhh = (w, fh // world) if shard else (w, fh)
        fb = front_bytes_per_launch(fw, fhh, args.effort)
        fms = sum(front_ms) / len(front_ms)
        achieved = fb / (fms * 1e-3) / 1e9 if fms > 0 else 0.0
        if shard:
            workload = ("%s x%d: %dx%d RGB8 (synth_rgb8 8K frame stacked %d times), VarDCT d%g "
                        "e%d, proposals=%d, %s-coded, 256x256 groups sharded over %d ranks, "
                        "%s assembly"
                        % (name, world, w, fh, world, args.distance, args.effort,
                           args.proposals, args.coder, world, args.assembly))
            par = "group-shard%d" % world
        else:
            workload = ("%s %dx%d RGB8 (synth_rgb8), VarDCT d%g e%d, proposals=%d, %s-coded, "
                        "%d distinct frame(s) per step, %d concurrent encoder stream(s) per rank"
                        % (name, w, h, args.distance, args.effort, args.proposals, args.coder,
                           frames, nstreams))
            par = "frame-dp%d" % world
        res = {
            "metric": "MPix/s VarDCT encode @ d1.0, 8K RGB",
            "value": round(value, 2),
            "unit": "MPix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": workload, "global_batch": 1 if shard else world * frames,
                       "parallelism": par},
            "streams_per_gpu": nstreams,
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
                         "algorithmic_bytes": fb, "avg_ms": round(fms, 4)},
            # the dominant kernels (merge stage) are VALU-issue-bound, not
            # HBM-bound: their live time and the PMC-measured VALU issue rate
            "merge_stage": {"kernels": "merge_eval + merge_resolve + merge_write",
                            "bound": "valu",
                            "avg_ms": round(st["ms_front"] - st["ms_front_kernel"], 4),
                            "valu_issue_frac_pmc": load_merge_pmc(name) if world == 1 else None},
        }
        if alt is not None:
            res["ans_coder"] = alt
        if thesis is not None:
            res["thesis_proposals"] = thesis
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(img, args.distance, args.effort)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
