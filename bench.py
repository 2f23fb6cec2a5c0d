#!/usr/bin/env python3
"""Benchmark: MPix/s of VarDCT encode at d1.0 on synthetic 8K RGB (BASELINE.json
metric), device-resident RGB8 in HBM -> complete .jxl bytes in host memory.

  python bench.py --gpus N --steps K --warmup W

One step = one full encode of one 7680x4320 frame per rank (front end, token
statistics, prefix codes, bit emission, assembly, D2H of the codestream).
Multi-GPU (launched by torch.distributed.run): every rank encodes its own frame
(frame-level data parallelism, no data-path collective), so scaling is weak;
the barrier + max-over-ranks timing follows the driver contract.

The JSON line also carries:
  roofline     -- the fused front kernel (XYB + ACS + DCT + quant): algorithmic
                  bytes per launch / its HIP-event duration vs 8.0 TB/s, plus
                  PMC-measured HBM traffic from profiles/ when present;
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


def front_bytes_per_launch(w, h):
    """Algorithmic HBM bytes of one front launch: RGB8 read (3 B/px), int16
    coefficients written (3 ch x 2 B = 6 B/px), per 8x8 block 3 x int32 DC +
    strategy + quant field (14 B / 64 px)."""
    bxs, bys = (w + 7) // 8, (h + 7) // 8
    return 3 * w * h + 6 * (bxs * 8) * (bys * 8) + 14 * bxs * bys


def load_pmc_traffic(workload):
    p = os.path.join(ROOT, "profiles", "front_pmc_%s.json" % workload)
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch")
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, help="BASELINE config index (2 = 8K)")
    ap.add_argument("--distance", type=float, default=1.0)
    ap.add_argument("--effort", type=int, default=7)
    ap.add_argument("--proposals", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    name, w, h, _ = CONFIGS[args.config]
    img = synth_rgb8(w, h, SEED_BASE + args.config + rank)
    d_img = torch.from_numpy(img).to("cuda:%d" % local)
    torch.cuda.synchronize()

    enc = jxg.Encoder(distance=args.distance, effort=args.effort, proposals=args.proposals,
                      device=local)
    for _ in range(args.warmup):
        out = enc.encode_device(d_img.data_ptr(), w, h, copy=False)
    # front-kernel duration over the timed region (HIP events on the encoder's
    # own stream, bracketing exactly the front launch)
    front_ms = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nbytes = 0
    host_ms = []
    for _ in range(args.steps):
        # the codestream ends in (pinned) host memory; copy=False keeps it there
        out = enc.encode_device(d_img.data_ptr(), w, h, copy=False)
        st = enc.stats()
        front_ms.append(st["ms_front"])
        host_ms.append((st["ms_host_call"], st["ms_host_codes"], st["ms_host_layout"]))
        nbytes = len(out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device="cuda:%d" % local, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    enc.close()
    if rank == 0:
        ms_step = dt * 1e3 / args.steps
        value = w * h * world * args.steps / dt / 1e6
        fb = front_bytes_per_launch(w, h)
        fms = sum(front_ms) / len(front_ms)
        achieved = fb / (fms * 1e-3) / 1e9
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
            "config": {"workload": "%s %dx%d RGB8 (synth_rgb8), VarDCT d%g e%d, proposals=%d, "
                                   "prefix-coded, one frame per rank" % (
                                       name, w, h, args.distance, args.effort, args.proposals),
                       "global_batch": world, "parallelism": "frame-dp%d" % world},
            "bytes_per_frame": nbytes,
            "bpp": round(nbytes * 8.0 / (w * h), 4),
            "stages_ms": {k: round(st[k], 4) for k in ("ms_front", "ms_histogram", "ms_emit",
                                                       "ms_assemble", "ms_total")},
            "host_ms": {k: round(sum(x[i] for x in host_ms) / len(host_ms), 4)
                        for i, k in enumerate(("call", "codes", "layout"))},
            "roofline": {"kernel": "front_kernel", "bound": "hbm",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_pmc_traffic(name),
                         "algorithmic_bytes": fb, "avg_ms": round(fms, 4)},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(img, args.distance, args.effort)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
