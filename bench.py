#!/usr/bin/env python3
"""Benchmark: MPix/s of VarDCT encode at d1.0 on synthetic 8K RGB (BASELINE.json
metric), device-resident RGB8 in HBM -> complete .jxl bytes in host memory.

  python bench.py --gpus N --steps K --warmup W [--mode shard|replica]
                  [--scaling strong|weak] [--coder prefix|ans] [--config C]

One step = one full encode (front end + merge stage, token statistics, entropy
codes, bit emission, assembly, D2H of the codestream).  The encode is the one
the reference's harness gets from `cjxl IN OUT --distance=1 --effort=7`
(docker_manager.rs:126-136): JXG_FLAGS_CJXL_DEFAULTS -- ANS, inverse
Gaborish, EPF by distance, the masking quant field (--preset cjxl, the
default); --preset plain is the unfiltered activity-AQ encode of rounds 1-4
(reported beside it as `filters_off`).  --coder prefix swaps the AC coder.  Single-GPU and replica steps go through the library's streaming entry
points (jxg_submit_rgb8_device / jxg_receive: a one-thread software pipeline
inside the library in which the rANS chains of earlier frames run under the
transform kernels of later ones); the timed region ends when the last
codestream of the K steps is in host memory.

N = 1: one 7680x4320 frame per step (BASELINE config 2's frame on one GPU);
the steps cycle through two distinct synthetic frames.
N > 1: one process per GPU.  Launched by torch.distributed.run (RANK /
LOCAL_RANK / WORLD_SIZE from the environment; WORLD_SIZE must equal --gpus),
or, with WORLD_SIZE unset, bench.py starts the N ranks itself under
torch.distributed.run (a child process, before anything touches the GPU) and
exits with its status.  Backend nccl = RCCL.
  shard   (default) -- BASELINE config 2 as written, strong scaling: every
          step is ONE 7680x4320 frame whose 256x256 pass groups are split over
          the N ranks (whole LF groups per rank, jxg_shard_plan kind 1: no
          per-block records move; one HF preset per rank: no histogram
          collective), streamed through jxg.dist.ShardStream -- each rank
          keeps up to jxg_pipeline_depth frames' shards in flight in the
          library's lanes (jxg_shard_submit_device), swaps each frame's payload
          heads with the other ranks through a node-shared /dev/shm region and
          DMAs its sections into the frame's codestream there
          (jxg_shard_next_head / jxg_shard_write_next; rank 0 adds headers +
          TOC).  value = frames x 7680 x 4320 / time over all ranks.  The
          /dev/shm exchange replaces an RCCL gather on purpose: the
          codestream must end in host memory, and every rank DMAs its own
          sections there over its own PCIe link.
          --scaling weak: one frame of N stacked 8K frames per step instead.
  shard-sync -- the same split one frame at a time (jxg.dist.encode_sharded:
          record exchange + histogram all-reduce when the plan / coder needs
          them, --assembly host|device).
  replica -- every rank streams its own 8K frames (frame-level data
          parallelism, no data-path collective); also reported beside the
          shard line as `replicas`.
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
  filters_off  -- (--preset cjxl) the unfiltered activity-AQ encode (the
                  rounds 1-4 headline), same pipeline;
  roofline_e4  -- the front kernel at effort 4 (DCT8 only: the literal fused
                  XYB + DCT + quant of SURVEY §8(d)), a labelled secondary line;
  quality      -- decoded PSNR / bpp of a 1920x1080 crop of the bench frame and
                  of a 1920x1080 photographic-like frame (untimed);
  cpu_baseline -- the oracle/ C restatement with OpenMP on the host's cores
                  (libjxl absent on the box) on the same frame, and whether
                  its bytes equal the GPU's.
"""
import argparse
import json
import os
import resource
import sys
import time

# The library's streaming pipeline runs up to 12 encoder lanes (7 at 8K, 12
# for 4K and smaller), one HIP stream each; HIP maps streams onto
# GPU_MAX_HW_QUEUES hardware queues per process (the box exports 4, one of them
# taken by torch's stream), and two lanes sharing a queue serialise their
# kernels.  Must be set before HIP initialises (JXG_BENCH_HW_QUEUES overrides
# it for experiments; at most 32).
#
# Several ranks on ONE device (the JXG_DIST_BACKEND=gloo rehearsal of the
# multi-GPU path on a one-GPU box): every process has its own
# GPU_MAX_HW_QUEUES queues, so 4 ranks x 16 = 64 queues oversubscribe the
# device's hardware queue slots and the scheduler time-slices the processes
# (round 4's 4-rank rehearsal: 49 ms per frame, 367 ms latency,
# profiles/r04m/bench_gloo4.log).  The rehearsal splits the 16 queues between
# the ranks sharing the device instead (each rank's pipeline lanes follow:
# queues - 1).  A rank alone on its GPU (the driver's N-GPU run) keeps 16.
def _ranks_sharing_device():
    if os.environ.get("JXG_DIST_BACKEND", "nccl") != "gloo":
        return 1
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    ndev = len(vis.split(",")) if vis else int(os.environ.get("JXG_BENCH_DEVICES", "1"))
    return max(1, (lw + ndev - 1) // ndev)


RANKS_PER_DEVICE = _ranks_sharing_device()
HW_QUEUES = min(32, int(os.environ.get("JXG_BENCH_HW_QUEUES",
                                       str(max(3, 16 // RANKS_PER_DEVICE)))))
os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)

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


def load_front_valu_floor(workload, avg_ms):
    """The front kernel's VALU floor from its PMC counters: SQ_INSTS_VALU
    wave-instructions x 2 cycles each (wave64 on a 32-lane SIMD,
    MI355X_MICROARCH.md 'v_fma_f32 (wave64) 2 cyc') / (1024 SIMDs x 2.4 GHz, the
    guide's max clock: the lowest floor), against the measured kernel time."""
    p = os.path.join(ROOT, "profiles", "front_pmc_%s.json" % workload)
    try:
        with open(p) as f:
            insts = json.load(f)["SQ_INSTS_VALU"]
        clk = 2.4e9
        floor = insts * 2.0 / (1024 * clk) * 1e3
        return {"valu_insts": int(insts), "cycles_per_inst": 2, "simds": 1024,
                "clock_ghz": 2.4, "floor_ms": round(floor, 4),
                "frac": round(floor / avg_ms, 4) if avg_ms else None}
    except Exception:
        return None


def load_merge_pmc(workload):
    p = os.path.join(ROOT, "profiles", "merge_pmc_%s.json" % workload)
    try:
        with open(p) as f:
            return json.load(f).get("valu_issue_frac")
    except Exception:
        return None


def cpu_quota():
    """CPUs of this process's cgroup CPU quota (cgroup v2 cpu.max, or v1
    cfs_quota / cfs_period), None when unlimited.  On the GPU box nproc and the
    affinity mask show the whole machine (256 CPUs) while the quota is the
    box's share (16): OpenMP over 256 threads under a 16-CPU quota is
    throttled (round 3's 8.0 MPix/s on "256 cores" vs 21 on 16)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(q) // int(per))
        return None
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return max(1, q // per) if q > 0 else None
    except (OSError, ValueError):
        return None


def cpu_affinity():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_threads():
    """host threads for the CPU baseline: the CPUs this process may actually
    use -- its affinity, capped by its cgroup CPU quota"""
    n = cpu_affinity()
    q = cpu_quota()
    return max(1, min(n, q) if q else n)


def cpu_baseline(img, distance, effort, proposals, coder, filters, gpu_bytes, sweep=None):
    """The oracle/ C restatement (libjxl/cjxl are absent on the box: probe in
    profiles/r02a/probe.txt) timed on the host with OpenMP over
    cpu_threads() threads, on the same frame and settings as the GPU line.
    Its codestream is also compared with the GPU's (byte-exact parity)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi  # the checker, timed here only as the reported baseline

    oracle_ffi.build()
    h, w, _ = img.shape

    def timed(threads):
        n = oracle_ffi.set_threads(threads)
        t = time.perf_counter()
        r = oracle_ffi.encode(img, distance, effort, proposals, coder, filters)
        return n, time.perf_counter() - t, r

    n, dt, r = timed(cpu_threads())
    res = {"value": round(w * h / 1e6 / dt, 3), "unit": "MPix/s", "cores": n, "kind": "port",
           "nproc": os.cpu_count(), "affinity": cpu_affinity(), "cgroup_quota_cpus": cpu_quota(),
           "sample": "one full %dx%d frame (the bench frame), oracle/ C restatement with OpenMP "
                     "on %d threads = the process's CPU affinity (%d) capped by its cgroup CPU "
                     "quota (%s; nproc %s; libjxl/cjxl absent on the box), same flags as the GPU "
                     "line (oracle filters mask %d), %.2f s"
                     % (w, h, n, cpu_affinity(), cpu_quota(), os.cpu_count(), filters, dt),
           "bytes_equal_gpu": gpu_bytes is not None and r.bytes == gpu_bytes}
    if sweep:
        # threads vs throughput (one frame each, same bytes)
        res["sweep"] = {}
        for th in sweep:
            n2, dt2, r2 = timed(th)
            res["sweep"][str(n2)] = round(w * h / 1e6 / dt2, 3)
            assert r2.bytes == r.bytes
        oracle_ffi.set_threads(n)
    return res


def quality_natural(enc):
    """decoded PSNR / bpp of the photographic-like 1920x1080 frame (untimed)"""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import jxl_decode
    from jxg.synth import natural_rgb8

    nat = natural_rgb8(1920, 1080, 3)
    nd = enc.encode(nat)
    ndec = jxl_decode.decode(nd).rgb
    return {"frame": "natural_rgb8(1920, 1080, seed 3)",
            "psnr_db": round(jxg.calculate_psnr(jxg.calculate_mse(nat, ndec)), 3),
            "bpp": round(len(nd) * 8.0 / (1920 * 1080), 4)}


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


def write_png(path, img):
    """8-bit RGB PNG, filter 0, zlib level 1 (the harness's input format)"""
    import struct
    import zlib

    h, w, _ = img.shape
    raw = np.zeros((h, w * 3 + 1), dtype=np.uint8)
    raw[:, 1:] = img.reshape(h, w * 3)

    def chunk(t, b):
        return struct.pack(">I", len(b)) + t + b + struct.pack(">I", zlib.crc32(t + b) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
                chunk(b"IDAT", zlib.compress(raw.tobytes(), 1)) + chunk(b"IEND", b""))


def single_image_probe(img, distance, effort, headline_bytes, device, runs=3):
    """What one image costs a caller that encodes images one at a time -- the
    harness's pattern (execute_cjxl runs one encoder process per (image,
    distance, effort), docker_manager.rs:126-136, benchmark.rs:641-660):
    * cli: `jxg_cjxl IN.png OUT.jxl --distance=D --effort=E` wall time, process
      start to exit (HIP runtime init, PNG decode, jxg_create, encode, write,
      jxg_destroy), and the phases the tool reports (JXG_CJXL_TIMING);
    * encode_rgb8: one-at-a-time jxg_encode_rgb8 from host RGB8 on a warm
      context (H2D included);
    * create_destroy: jxg_create + jxg_destroy, and the first encode of a new
      context (its buffers and tables) against a warm one."""
    import subprocess
    import tempfile

    h, w, _ = img.shape
    out = {"image": "%dx%d synth_rgb8 frame (bench frame 0) as PNG" % (w, h)}
    flags = jxg.FLAGS_CJXL_DEFAULTS
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "frame.png")
        t0 = time.perf_counter()
        write_png(src, img)
        out["png_bytes"] = os.path.getsize(src)
        walls, phases, same = [], [], True
        env = dict(os.environ, JXG_CJXL_TIMING="1")
        for i in range(runs):
            dst = os.path.join(td, "frame-%g-%d.jxl" % (distance, effort))
            t0 = time.perf_counter()
            u0 = time.time() * 1e3
            p = subprocess.run([jxg.CLI_PATH, src, dst, "--distance=%g" % distance,
                                "--effort=%d" % effort, "--device=%d" % device],
                               capture_output=True, text=True, env=env)
            walls.append((time.perf_counter() - t0) * 1e3)
            u1 = time.time() * 1e3
            if p.returncode != 0:
                out["cli_error"] = p.stderr.strip()[-300:]
                break
            line = [l for l in p.stderr.splitlines() if l.startswith("{")]
            if line:
                ph = json.loads(line[-1])
                um = ph.pop("unix_ms_main", None)
                if um:  # process start (exec, dynamic loading) / exit (teardown)
                    ph["ms_before_main"] = um[0] - u0
                    ph["ms_after_main"] = u1 - um[1]
                phases.append(ph)
            with open(dst, "rb") as f:
                same = same and (headline_bytes is None or f.read() == headline_bytes)
        if walls:
            out["cli"] = {"argv": "jxg_cjxl IN.png OUT.jxl --distance=%g --effort=%d" % (distance, effort),
                          "ms_wall": [round(x, 1) for x in walls],
                          "ms_wall_best": round(min(walls), 1),
                          "mpix_s_wall_best": round(w * h / (min(walls) * 1e3), 1),
                          "bytes_equal_headline": same}
            if phases:
                best = min(range(len(phases)), key=lambda i: walls[i])
                ph = {k: round(v, 2) for k, v in phases[best].items()}
                # (ms_create_overlapped runs on a second thread beside the decode)
                ph["ms_unaccounted"] = round(walls[best] - sum(
                    v for k, v in phases[best].items() if k != "ms_create_overlapped"), 1)
                out["cli"]["phases_best_run"] = ph
    # one-at-a-time jxg_encode_rgb8 from host memory, warm context
    host = np.ascontiguousarray(img)
    t0 = time.perf_counter()
    enc = jxg.Encoder(distance=distance, effort=effort, device=device, flags=flags)
    t_create = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    first = enc.encode(host)
    t_first = (time.perf_counter() - t0) * 1e3
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        enc.encode(host)
        ts.append((time.perf_counter() - t0) * 1e3)
    t0 = time.perf_counter()
    enc.close()
    t_destroy = (time.perf_counter() - t0) * 1e3
    cd = []
    for _ in range(5):
        t0 = time.perf_counter()
        jxg.Encoder(distance=distance, effort=effort, device=device, flags=flags).close()
        cd.append((time.perf_counter() - t0) * 1e3)
    out["encode_rgb8"] = {"ms": [round(x, 2) for x in ts], "ms_median": round(float(np.median(ts)), 2),
                          "mpix_s": round(w * h / (float(np.median(ts)) * 1e3), 1),
                          "bytes_equal_headline": headline_bytes is None or first == headline_bytes}
    out["create_destroy"] = {"ms_first_create": round(t_create, 2),
                             "ms_first_encode_new_context": round(t_first, 2),
                             "ms_destroy": round(t_destroy, 2),
                             "ms_create_destroy": [round(x, 2) for x in cd]}
    return out


def spawn_ranks(n, argv):
    """Run this script as n ranks under torch.distributed.run (one node,
    rendezvous on 127.0.0.1) in a child process; returns its exit status."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 300 frames by default: the timed region of a streaming run includes one
    # pipeline fill + drain (about one frame's latency, ~25 ms at 8K ANS), which
    # costs 16 % of a 20-frame run, 2-3 % of a 100-frame one and < 1 % of 300
    # (1.1 s of timed encodes at 8K)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, help="BASELINE config index (2 = 8K)")
    ap.add_argument("--distance", type=float, default=1.0)
    ap.add_argument("--effort", type=int, default=7)
    ap.add_argument("--proposals", type=int, default=0)
    ap.add_argument("--mode", choices=("shard", "shard-sync", "replica"),
                    default="shard",
                    help="N > 1: shard = every frame's pass groups split over the ranks, "
                         "streamed (jxg.dist.ShardStream; BASELINE config 2 as written); "
                         "shard-sync = the same one frame at a time (encode_sharded); "
                         "replica = every rank streams its own frames (frame-level data "
                         "parallelism)")
    ap.add_argument("--alt-replica", type=int, default=1,
                    help="shard mode, N > 1: also time frame replicas (reported under "
                         "'replicas')")
    ap.add_argument("--distinct", type=int, default=2,
                    help="distinct synthetic frames the steps cycle through")
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
    ap.add_argument("--preset", choices=("cjxl", "plain"), default="cjxl",
                    help="cjxl = JXG_FLAGS_CJXL_DEFAULTS (Gaborish + EPF + masking AQ: what "
                         "`cjxl IN OUT --distance=1 --effort=7` encodes, the headline); plain = "
                         "no restoration filters, activity AQ")
    ap.add_argument("--alt-preset", "--alt-cjxl", dest="alt_preset", type=int, default=1,
                    help="also time the other preset (reported under 'filters_off' or "
                         "'cjxl_defaults'; 0 = off)")
    ap.add_argument("--alt-e4", type=int, default=1,
                    help="also report the effort-4 (DCT8-only) front kernel's roofline "
                         "('roofline_e4'; 0 = off)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sweep", default="",
                    help="comma-separated OpenMP thread counts: also time the CPU baseline at "
                         "each (reported under cpu_baseline.sweep)")
    ap.add_argument("--no-quality", action="store_true",
                    help="skip the untimed decode-PSNR probe")
    ap.add_argument("--no-single", action="store_true",
                    help="skip the untimed one-image-at-a-time probe (single_image)")
    args = ap.parse_args()

    # one process per GPU: with WORLD_SIZE unset, --gpus N > 1 starts the N
    # ranks itself (before this process touches the GPU); a launcher's
    # WORLD_SIZE must agree with --gpus
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d" % (env_world, args.gpus), file=sys.stderr)
        sys.exit(2)
    world = int(env_world or "1")
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
    sharded_mode = world > 1 and args.mode in ("shard", "shard-sync")
    strong = sharded_mode and args.scaling == "strong"
    fh = h if strong or not sharded_mode else h * world
    # inputs generated on the device (jxg_synth_rgb8_device: the bytes of
    # jxg.synth.synth_rgb8, without minutes of numpy at 8K / 16K).  Every rank
    # of a sharded run holds the same frames; replicas get their own.  Batch
    # configs (64 x 1080p): a step is the whole batch of distinct frames.
    def make_frames(sharded):
        per_step = 1 if sharded else nframes
        n = per_step * max(1, args.distinct) if per_step == 1 else per_step
        seed0 = SEED_BASE + args.config + (0 if sharded else 1000 * rank)
        out = []
        for f in range(n):
            t = synth_rgb8_device(w, h, seed0 + (f if per_step > 1 else 100 * f), local)
            if sharded and not strong:
                # one frame of N stacked config frames: every rank owns 1/N of its groups
                t = t.repeat(world, 1, 1).contiguous()
            out.append(t)
        return per_step, out

    img = None
    if world == 1:  # quality probe / CPU baseline: the first frame
        img = synth_rgb8_device(w, h, SEED_BASE + args.config, local).cpu().numpy()
    torch.cuda.synchronize()

    preset_flags = {"cjxl": jxg.FLAGS_CJXL_DEFAULTS & ~jxg.FLAG_ANS, "plain": 0}
    pflags = preset_flags[args.preset]

    def run(mode, coder, nstreams=1, proposals=None, pipe=True, extra_flags=None, effort=None):
        """Warm up, then time args.steps steps of `mode` ("frames": each rank
        encodes whole frames -- N = 1 / replicas; "shard": ShardStream;
        "shard-sync": encode_sharded)."""
        sharded = mode != "frames"
        per_step, d_imgs = make_frames(sharded)
        nd = len(d_imgs)
        flags = (jxg.FLAG_ANS if coder == "ans" else 0) | (
            pflags if extra_flags is None else extra_flags)
        props = args.proposals if proposals is None else proposals
        encs = [jxg.Encoder(distance=args.distance, effort=args.effort if effort is None else effort,
                            proposals=props, device=local, flags=flags)
                for _ in range(nstreams)]
        rec = {"front_ms": [], "host_ms": [], "aq_ms": [], "sizes": [], "last": None}

        def took(e, k, out):
            t = e.timings()
            rec["front_ms"].append(t[0])
            rec["host_ms"].append(t[1:4])
            rec["aq_ms"].append(t[4])
            rec["sizes"].append(len(out) if out is not None else 0)
            if k % nd == 0:
                # shared-memory views (ShardStream) are recycled: keep a copy
                rec["last"] = out.tobytes() if isinstance(out, np.ndarray) else out

        ss = None
        host = None
        bufs = {}
        if mode == "shard":
            from jxg.dist import ShardStream
            # (each process has its own HW_QUEUES queues, split above when
            # ranks share a device: its lanes follow them, no cap needed)
            ss = ShardStream(encs[0], w, fh, rank, world)
        elif mode == "shard-sync" and args.assembly == "host":
            from jxg.dist import SharedHostBuffer
            if SharedHostBuffer.single_node():
                host = SharedHostBuffer(rank, world)
            # else: ranks on several nodes -> device assembly (payload gather)

        def worker(e, ks):
            # the codestream ends in (pinned / shared) host memory; ctypes
            # calls release the GIL, so several encoders' host work overlaps
            if ss is not None:
                # (a received view stays valid until the next receive: took()
                # keeps only its size, and copies the bytes of the frames it
                # keeps); frames are taken as soon as they are complete
                got = 0
                for k in ks:
                    ss.submit(d_imgs[k % nd].data_ptr())
                    while ss.pending() >= ss.max_pending or (ss.pending() and ss.ready()):
                        took(e, got, ss.receive())
                        got += 1
                while ss.pending():
                    took(e, got, ss.receive())
                    got += 1
            elif mode == "shard-sync":
                from jxg.dist import encode_sharded
                for k in ks:
                    took(e, k, encode_sharded(e, d_imgs[k % nd], w, fh, rank, world, bufs=bufs,
                                              copy=False, host=host))
            elif pipe:
                # streaming entry points: submit every frame, receive each
                # codestream as soon as it is done (more than the library's
                # pipeline depth pending => the oldest is complete)
                got = 0
                hold = max(16, e.pipeline_depth(w, h))
                for k in ks:
                    e.submit_device(d_imgs[k % nd].data_ptr(), w, h)
                    while e.pending() > hold:
                        took(e, got, e.receive(copy=False))
                        got += 1
                while e.pending():
                    took(e, got, e.receive(copy=False))
                    got += 1
            else:
                for k in ks:
                    took(e, k, e.encode_device(d_imgs[k % nd].data_ptr(), w, h, copy=False))

        for e in encs:  # contexts warmed one after another
            # at least 16 frames when streaming: every lane of the library's
            # pipeline (up to 12) allocates its buffers on its first frame,
            # which must not land in the timed region
            nw = max(args.warmup, 1) * per_step
            if ss is not None:
                # every lane slot of the rank's pipeline (up to 12 lanes x 4
                # frames) allocates its buffers on its first frames: all of
                # them run before the timed region
                nw = max(nw, 2 * ss.depth + 8)
            worker(e, range(max(nw, 16) if (pipe or ss is not None) else args.warmup * per_step))
        for key in ("front_ms", "host_ms", "aq_ms", "sizes"):
            rec[key] = []
        if ss is not None:
            ss.wait_s = 0.0

        total = args.steps * per_step
        share = [list(range(i, total, nstreams)) for i in range(nstreams)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ru0 = resource.getrusage(resource.RUSAGE_SELF)  # this process's CPU (all threads)
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
        dt_own = time.perf_counter() - t0  # this rank's own work, before the barrier
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu_own = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
        wait_own = ss.wait_s if ss is not None else 0.0
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([dt], dtype=torch.float64,
                              device="cpu" if backend == "gloo" else dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
            # per-rank time and the time it spent waiting for the other ranks
            # (ShardStream: heads, slots, frames) -> rank 0
            mine = torch.tensor([dt_own, wait_own, cpu_own], dtype=torch.float64,
                                device="cpu" if backend == "gloo" else dev)
            allr = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(allr, mine)
            rec["per_rank"] = [(float(x[0]), float(x[1])) for x in allr]
            rec["cpu_per_rank"] = [float(x[2]) for x in allr]
        rec["dt"] = dt
        rec["cpu_s"] = cpu_own
        rec["per_step"] = per_step
        rec["st"] = encs[0].stats()
        last = rec["last"]
        rec["last"] = last.tobytes() if hasattr(last, "tobytes") else last
        if ss is not None:
            ss.close()
        for e in encs[1:]:
            e.close()
        rec["enc"] = encs[0]
        if host is not None:
            dist.barrier()
            host.close()
        rec["depth"] = ss.depth if ss is not None else None
        return rec

    if world == 1 or args.mode == "replica":
        mode = "frames"
    else:
        mode = args.mode
    pipeline = mode == "frames" and not args.no_pipeline
    nstreams = 1 if mode != "frames" else max(1, args.streams)
    R = run(mode, args.coder, nstreams, pipe=pipeline)
    dt, front_ms, host_ms, st = R["dt"], R["front_ms"], R["host_ms"], R["st"]
    per_step = R["per_step"]
    nbytes = R["sizes"][-1] if R["sizes"] else 0
    # pixels of one step over the whole job
    px_step = w * fh * per_step * (1 if mode != "frames" else world)
    alt = None
    other = "prefix" if args.coder == "ans" else "ans"
    if mode == "frames" and args.alt_coder > 0:
        # the same workload with the other AC entropy coder
        A = run("frames", other, nstreams, pipe=pipeline)
        A["enc"].close()
        alt = {"coder": other, "streams_per_gpu": nstreams, "pipeline": pipeline,
               "value": round(px_step * args.steps / A["dt"] / 1e6, 2),
               "ms_per_step": round(A["dt"] * 1e3 / args.steps, 3),
               "ms_latency": round(sum(x[0] for x in A["host_ms"]) / len(A["host_ms"]), 3),
               "bytes_per_frame": A["sizes"][-1],
               "bpp": round(A["sizes"][-1] * 8.0 / (w * h), 4)}
    replicas = None
    if mode != "frames" and args.alt_replica:
        # every rank streams its own frames (frame-level data parallelism)
        P = run("frames", args.coder, 1, pipe=True)
        if rank == 0:
            replicas = {"mode": "replica", "scaling": "weak", "coder": args.coder,
                        "value": round(w * h * world * args.steps / P["dt"] / 1e6, 2),
                        "ms_per_step": round(P["dt"] * 1e3 / args.steps, 3),
                        "bytes_per_frame": P["sizes"][-1]}
        P["enc"].close()
    iso = None
    streamed = mode == "shard"
    if mode == "frames" and pipeline or streamed:
        # the kernels alone on the GPU (one-at-a-time encodes of this rank's
        # frame, same coder): the front kernel's roofline, the rANS chain
        # kernel's duration
        iso = run("frames", args.coder, 1, pipe=False)
        iso["enc"].close()
    thesis = None
    if mode == "frames" and args.alt_thesis and args.proposals != 3:
        # the thesis proposals P + F (combined.diff) on the same workload:
        # the homogeneity selector in the front kernel, hook F on every
        # 8x8 and merge candidate
        T = run("frames", args.coder, nstreams, proposals=3, pipe=pipeline)
        T["enc"].close()
        thesis = {"proposals": "P+F (combined.diff)",
                  "value": round(px_step * args.steps / T["dt"] / 1e6, 2),
                  "ms_per_step": round(T["dt"] * 1e3 / args.steps, 3),
                  "ms_front_kernel": round(sum(T["front_ms"]) / len(T["front_ms"]), 4),
                  "bytes_per_frame": T["sizes"][-1],
                  "bpp": round(T["sizes"][-1] * 8.0 / (w * h), 4)}
    alt_preset = None
    other_preset = "plain" if args.preset == "cjxl" else "cjxl"
    if mode == "frames" and args.alt_preset:
        # the other preset on the same workload and coder: with the cjxl
        # headline, the unfiltered activity-AQ encode of rounds 1-4
        C = run("frames", args.coder, nstreams, pipe=pipeline,
                extra_flags=preset_flags[other_preset])
        alt_preset = {"preset": other_preset,
                      "flags": ("gaborish + epf + masking AQ (JXG_FLAGS_CJXL_DEFAULTS)"
                                if other_preset == "cjxl" else
                                "no Gaborish, no EPF, activity AQ"),
                      "value": round(px_step * args.steps / C["dt"] / 1e6, 2),
                      "ms_per_step": round(C["dt"] * 1e3 / args.steps, 3),
                      "bytes_per_frame": C["sizes"][-1],
                      "bpp": round(C["sizes"][-1] * 8.0 / (w * h), 4)}
        if world == 1 and not args.no_quality:
            alt_preset["quality_natural"] = quality_natural(C["enc"])
        C["enc"].close()
    e4 = None
    if mode == "frames" and args.alt_e4 and world == 1:
        # the front kernel at effort 4 (DCT8 only, no merge stage): the fused
        # XYB + DCT + quant of SURVEY §8(d) taken literally, one frame at a time
        E = run("frames", args.coder, 1, pipe=False, effort=4)
        E["enc"].close()
        e4 = sum(E["front_ms"]) / len(E["front_ms"])
    if rank == 0:
        ms_step = dt * 1e3 / args.steps
        value = px_step * args.steps / dt / 1e6
        # roofline of the front kernel: the isolated one-at-a-time launch over
        # a whole frame (the kernel alone on the GPU)
        fw, fhh = w, h
        fb = front_bytes_survey(fw, fhh)
        fms_pipe = sum(front_ms) / len(front_ms)
        fms = sum(iso["front_ms"]) / len(iso["front_ms"]) if iso else fms_pipe
        if not iso and mode != "frames":
            fb = front_bytes_survey(w, fh) / world  # this rank's share of the frame
        achieved = fb / (fms * 1e-3) / 1e9 if fms > 0 else 0.0
        coder_desc = "%s-coded" % args.coder
        # PMC figures (profiles/front_pmc_<key>.json) are per preset
        pmc_key = name + ("_cjxl" if args.preset == "cjxl" else "")
        preset_desc = ("cjxl defaults (JXG_FLAGS_CJXL_DEFAULTS: Gaborish + EPF + masking AQ)"
                       if args.preset == "cjxl" else "no filters, activity AQ")
        distinct = max(1, args.distinct) if per_step == 1 else per_step
        if mode != "frames":
            workload = ("%s: %dx%d RGB8 (synth_rgb8, %d distinct frames cycled), VarDCT d%g e%d, "
                        "%s, proposals=%d, %s, 256x256 groups sharded over %d ranks (%s scaling; "
                        "partition kind %d), %s"
                        % (name, w, fh, distinct, args.distance, args.effort, preset_desc,
                           args.proposals,
                           coder_desc, world, args.scaling, jxg.shard_plan(w, fh, world)[2],
                           "streamed (jxg.dist.ShardStream, %d frames in flight per rank, heads "
                           "and sections through /dev/shm)" % R["depth"]
                           if streamed else
                           "one frame at a time (encode_sharded), %s assembly" % args.assembly))
            par = "group-shard%d" % world
        else:
            workload = ("%s %dx%d RGB8 (synth_rgb8), VarDCT d%g e%d, %s, proposals=%d, %s, "
                        "%d frame(s) per step, %d distinct frames cycled, %s"
                        % (name, w, h, args.distance, args.effort, preset_desc, args.proposals,
                           coder_desc,
                           per_step, distinct, "streaming entry points (jxg_submit_rgb8_device / "
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
            "scaling": "strong" if strong or world == 1 else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {"workload": workload,
                       "global_batch": per_step * (1 if mode != "frames" else world),
                       "parallelism": par},
            "streams_per_gpu": nstreams,
            "hw_queues_per_process": HW_QUEUES,
            "ranks_per_device": RANKS_PER_DEVICE,
            "pipeline": pipeline or streamed,
            "ms_latency": round(sum(x[0] for x in host_ms) / len(host_ms), 3),
            "bytes_per_frame": nbytes,
            "bpp": round(nbytes * 8.0 / (w * fh), 4) if mode == "frames" or rank == 0 else None,
            "stages_ms": {k: round(st[k], 4) for k in ("ms_front_kernel", "ms_front",
                                                       "ms_histogram", "ms_emit",
                                                       "ms_assemble", "ms_total")},
            "host_ms": {k: round(sum(x[i] for x in host_ms) / len(host_ms), 4)
                        for i, k in enumerate(("call", "codes", "layout"))},
            "roofline": {"kernel": "front_kernel", "bound": "hbm",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_pmc_traffic(pmc_key),
                         "algorithmic_bytes": int(fb),
                         "bytes_per_px": SURVEY_BYTES_PER_PX,
                         "design_bytes": front_bytes_design(fw, fhh, args.effort),
                         "avg_ms": round(fms, 4),
                         "aq_kernel_ms": round(sum(iso["aq_ms"]) / len(iso["aq_ms"]), 4)
                         if iso else None,
                         # the kernel is VALU-bound (the six-candidate 8x8 search):
                         # its PMC VALU issue rate beside the HBM fraction
                         "valu_issue_frac_pmc": load_front_valu(pmc_key),
                         # the bound that applies: VALU issue (the HBM fraction
                         # cannot pass ~0.17 while the kernel runs at this floor)
                         "valu_floor": load_front_valu_floor(pmc_key, fms),
                         "measured": ("one-at-a-time encodes of a whole frame (the kernel alone "
                                      "on the GPU, HIP events on its stream); in the timed run "
                                      "(sharing the GPU with rANS chains%s): %.4f ms"
                                      % ("" if mode == "frames" else
                                         ", this rank's 1/%d of the frame" % world, fms_pipe))
                         if iso else "timed region"},
            # the merge stage is latency-bound (VALU issue 35 %, waves waiting
            # on memory / LDS 41 % of their lifetime): its live time and the
            # PMC-measured VALU issue rate
            "merge_stage": {"kernels": "merge_eval + merge_resolve + merge_write",
                            "bound": "latency",
                            "avg_ms": round((iso["st"] if iso else st)["ms_front"] -
                                            (iso["st"] if iso else st)["ms_front_kernel"], 4),
                            "valu_issue_frac_pmc": load_merge_pmc(pmc_key)},
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
        if alt_preset is not None:
            res["filters_off" if other_preset == "plain" else "cjxl_defaults"] = alt_preset
        if e4 is not None:
            fb4 = front_bytes_survey(w, h)
            a4 = fb4 / (e4 * 1e-3) / 1e9
            res["roofline_e4"] = {"kernel": "front_kernel (effort 4: XYB + DC/AQ + DCT8 + quant, "
                                            "no 8x8 search, no merge stage)",
                                  "bound": "hbm", "achieved": round(a4, 1), "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": round(a4 / HBM_PEAK_GBS, 4),
                                  "algorithmic_bytes": int(fb4), "avg_ms": round(e4, 4),
                                  # PMC HBM bytes per launch (profiles/front_pmc_<cfg>_e4.json)
                                  "traffic": load_pmc_traffic(name + "_e4"),
                                  "valu_floor": load_front_valu_floor(name + "_e4", e4),
                                  "measured": "one-at-a-time encodes at effort 4, HIP events on "
                                              "the encoder's stream"}
        if replicas is not None:
            res["replicas"] = replicas
        if R.get("per_rank"):
            # every rank's own time per step (before the closing barrier) and the
            # time per step it waited for the other ranks (ShardStream: heads,
            # slots, frames), over the timed steps
            res["per_rank_ms_per_step"] = [round(a * 1e3 / args.steps, 3) for a, _ in R["per_rank"]]
            res["ms_wait_ranks"] = [round(b * 1e3 / args.steps, 3) for _, b in R["per_rank"]]
        # host CPU the ranks used over the timed region (getrusage of each rank's
        # process, every thread: submit / ShardStream thread + the library's
        # helper pool), as busy CPUs = CPU seconds / wall seconds, against the
        # cgroup quota the box grants (8 ranks on a 16-CPU share)
        cpus = R.get("cpu_per_rank") or [R["cpu_s"]]
        res["host_cpu"] = {"busy_cpus_per_rank": [round(c / dt, 2) for c in cpus],
                           "busy_cpus_total": round(sum(cpus) / dt, 2),
                           "cgroup_quota_cpus": cpu_quota()}
        if world == 1 and not args.no_quality:
            res["quality"] = quality_probe(R["enc"], img, args.distance, args.effort)
        if world == 1 and not args.no_single and args.preset == "cjxl" and args.coder == "ans":
            # the drop-in's per-call cost (untimed: after the timed region)
            res["single_image"] = single_image_probe(img, args.distance, args.effort,
                                                     R["last"] if args.proposals == 0 else None,
                                                     local)
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(img, args.distance, args.effort, args.proposals,
                                               1 if args.coder == "ans" else 0,
                                               jxg.ORACLE_FILTERS_CJXL_DEFAULTS
                                               if args.preset == "cjxl" else 0,
                                               R["last"],
                                               [int(x) for x in args.cpu_sweep.split(",") if x])
        print(json.dumps(res), flush=True)
    R["enc"].close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
