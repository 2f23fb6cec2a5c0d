"""Multi-GPU group-sharded encode over torch.distributed.

One process per GPU (backend "nccl" = RCCL over xGMI).  Each rank encodes a
balanced contiguous raster range of the frame's 256x256 pass groups and the
LF groups it owns (the rank holding most of an LF group's pass groups); the
only collectives are
  1. prefix codes only: all_reduce(sum) of the AC token histogram (132 x 128
     u32, 68 KB) so all ranks derive the same codes (one HF preset).  With ANS
     every rank codes its groups with its own histograms (one HF preset per
     rank; its clustered counts ride in its payload head and
     HfGlobal is written at assembly), so there is no histogram collective,
  2. all_to_all of per-block records (strategy, quant field, quantized DC;
     14 B per 8x8 block): a rank sends the records of its pass groups whose LF
     group another rank owns to that rank only (jxg_shard_exchange splits;
     8K over 8 ranks: ~0.7 MB per rank instead of an all-gather of 7.3 MB;
     16384^2 over 8 ranks: nothing),
  3. assembly, either
     host   (``host=SharedHostBuffer``): one all-gather of the payload heads
            (section ids and sizes, ~2 KB per rank; + ~13 KB of preset with
            ANS), then every rank DMAs its
            own sections into one /dev/shm buffer shared by the node's ranks
            at their codestream offsets (rank 0 adds headers + TOC) -- the
            node's PCIe links work in parallel and nothing crosses xGMI; or
     device (default): a gather of the per-rank section payloads on rank 0
            (device to device; staged through the host under gloo), which
            writes headers + TOC and moves every section with the concat
            kernel, then one D2H of the codestream.
With prefix codes the result is byte-identical to a single-GPU encode of the
same frame; with ANS it decodes to the same image (same coefficients, strategy,
quant field, DC and CfL maps) with per-rank histograms.

:class:`ShardStream` is the streaming form (the multi-GPU pipeline bench.py
--gpus N times): consecutive frames, each split over the ranks by a partition
that needs no record exchange (whole LF groups per rank, jxg_shard_plan kind
0 / 1) and coded with one HF preset per rank (ANS), so a rank's frames flow
through the library's lanes with no collective at all; per frame the ranks
only swap their payload heads through a node-shared /dev/shm region and DMA
their sections into it.  The /dev/shm exchange replaces an RCCL gather on
purpose: the codestream must end in host memory, so every rank DMAs its own
sections there over its own PCIe link (nothing crosses xGMI); RCCL is used by
the one-frame-at-a-time device assembly of :func:`encode_sharded`.
"""
from __future__ import annotations

import ctypes
import mmap
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from . import FLAG_ANS, Encoder, load, shard_assemble, shard_exchange, shard_sizes


class SharedHostBuffer:
    """One host buffer mapped by every rank of a node (/dev/shm file, MAP_SHARED),
    page-locked in each process (jxg_host_register) so the ranks' D2H copies
    are DMA.  Grown collectively: every rank sees the same required size (it
    follows from the all-gathered heads), so all re-map together."""

    def __init__(self, rank: int, world: int, group=None):
        self.rank, self.world, self.group = rank, world, group
        # every rank must map the same /dev/shm file: refuse (on every rank,
        # before any shared-memory use) unless all ranks run on one node
        if not self.single_node(group):
            raise RuntimeError("SharedHostBuffer needs all ranks on one node; use device assembly")
        tag = [os.getpid()] if rank == 0 else [None]
        dist.broadcast_object_list(tag, src=0, group=group)
        self.tag = tag[0]
        self.gen = 0
        self.cap = 0
        self.mm = None
        self.addr = 0
        self.path = None

    @staticmethod
    def single_node(group=None) -> bool:
        """True when every rank of `group` runs on this host (a collective)."""
        import socket

        names = [None] * dist.get_world_size(group)
        dist.all_gather_object(names, (socket.gethostname(), os.path.exists("/dev/shm")),
                               group=group)
        return len(set(names)) == 1 and names[0][1]

    def _release(self):
        if self.mm is not None:
            load().jxg_host_unregister(ctypes.c_void_p(self.addr))
            try:
                self.mm.close()
            except BufferError:  # a caller still holds a zero-copy view: GC unmaps later
                pass
            self.mm = None
            if self.rank == 0 and self.path and os.path.exists(self.path):
                os.unlink(self.path)

    def ensure(self, need: int):
        if need <= self.cap:
            return
        cap = max(need + (1 << 20), 2 * self.cap)
        cap = (cap + (1 << 21) - 1) & ~((1 << 21) - 1)
        dist.barrier(group=self.group)  # nobody still reads the old mapping
        self._release()
        self.gen += 1
        self.path = "/dev/shm/jxg_cs_%d_%d" % (self.tag, self.gen)
        if self.rank == 0:
            fd = os.open(self.path, os.O_CREAT | os.O_RDWR | os.O_TRUNC, 0o600)
            os.ftruncate(fd, cap)
            os.close(fd)
        dist.barrier(group=self.group)
        fd = os.open(self.path, os.O_RDWR)
        self.mm = mmap.mmap(fd, cap, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        os.close(fd)
        self.addr = ctypes.addressof(ctypes.c_char.from_buffer(self.mm))
        if load().jxg_host_register(ctypes.c_void_p(self.addr), cap) != 0:
            raise RuntimeError("jxg_host_register failed")
        self.cap = cap

    def view(self, n: int, offset: int = 0) -> np.ndarray:
        """zero-copy view of the codestream; valid until the next frame's
        write into the buffer (or close)"""
        return np.frombuffer(self.mm, dtype=np.uint8, count=n, offset=offset)

    def close(self):
        self._release()
        self.cap = 0


AC_CONTEXTS = 7425   # AC contexts of one HF preset (15 block contexts x 495)
ANS_MAX_HISTS = 8    # histograms per preset (csrc/jxg_bitstream.h kAnsMaxHists)
WRITE_LAG = 2        # include/jxg.h JXG_SHARD_WRITE_LAG
ALPHA = 128


def _head_cap(width: int, height: int) -> int:
    """Upper bound of a payload head in u32 words: 7 + 2 x sections, a rank
    holding at most LfGlobal, HfGlobal, every LF group and every pass group;
    plus, for version-2 heads (ANS, one HF preset per rank), the preset block
    [B][nhist][context map packed in words][counts nhist x 128]."""
    nlf = -(-width // 2048) * -(-height // 2048)
    ngroups = -(-width // 256) * -(-height // 256)
    preset = 2 + -(-AC_CONTEXTS // 4) + ANS_MAX_HISTS * ALPHA
    return 7 + 2 * (2 + nlf + ngroups) + preset


def _head_len(h) -> int:
    """Words of a payload head (version 1: 7 + 2 x sections; version 2: + the
    preset block, whose first word counts the words after it)."""
    base = 7 + 2 * int(h[6])
    return base if int(h[1]) == 1 else base + 1 + int(h[base])


def _all_gather_heads(head: np.ndarray, rank: int, world: int, width: int, height: int,
                      group=None):
    """Variable-length u32 payload heads of all ranks (rank order), on every
    rank, with ONE all-gather of fixed-capacity slots (no size exchange): a
    head's own length is 7 + 2 x its section count (word 6)."""
    dev = "cpu" if dist.get_backend(group) == "gloo" else torch.device("cuda", torch.cuda.current_device())
    cap = _head_cap(width, height)
    if head.size > cap or head.size < 7 or head.size != _head_len(head):
        raise RuntimeError("payload head of %d words outside [7, %d]" % (head.size, cap))
    mine = torch.zeros(cap, dtype=torch.int32, device=dev)
    mine[:head.size] = torch.from_numpy(head.view(np.int32).copy()).to(dev)
    parts = [torch.empty(cap, dtype=torch.int32, device=dev) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    allh = torch.stack(parts).cpu().numpy().view(np.uint32)  # one copy to the host
    return [allh[r, :_head_len(allh[r])].copy() for r in range(world)]


def gather_payloads(payload: bytes, rank: int, world: int, device, group=None):
    """Variable-size byte payloads of all ranks -> list on rank 0 (None
    elsewhere): all_gather of the sizes, then a gather of padded buffers."""
    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    cap = max(sizes)
    mine = torch.zeros(cap, dtype=torch.uint8, device=device)
    if payload:
        mine[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    bufs = [torch.empty(cap, dtype=torch.uint8, device=device) for _ in range(world)] \
        if rank == 0 else None
    dist.gather(mine, bufs, dst=0, group=group)
    if rank != 0:
        return None
    return [bytes(b[:s].cpu().numpy().tobytes()) for b, s in zip(bufs, sizes)]


def _comm_device(dev, group=None) -> torch.device:
    """where a collective's tensors live: HBM under nccl (RCCL), host memory
    under gloo"""
    return torch.device("cpu") if dist.get_backend(group) == "gloo" else torch.device(dev)


def _copy_back(dst: torch.Tensor, src: torch.Tensor):
    """dst <- src unless they are the same storage (nccl: the collective wrote
    dst itself)"""
    if src.data_ptr() != dst.data_ptr() or src.device != dst.device:
        dst.copy_(src)


def encode_sharded(enc: Encoder, d_rgb: torch.Tensor, width: int, height: int, rank: int,
                   world: int, group=None, bufs=None, copy: bool = True,
                   host: SharedHostBuffer | None = None):
    """Encode one frame (device-resident (H, W, 3) uint8 on every rank) with
    group sharding; returns the codestream on rank 0 (bytes, or a zero-copy
    view with copy=False: a :class:`jxg.Codestream` of pinned memory, or with
    ``host`` a numpy view of the shared buffer), None elsewhere.  `bufs`
    caches the exchange tensors across calls."""
    dev = d_rgb.device
    # the frame was produced on torch's stream: the library orders its reads
    # after it (include/jxg.h, device inputs)
    enc.set_input_stream(torch.cuda.current_stream(dev).cuda_stream)
    if bufs is None:
        bufs = {}
    key = (width, height, world, rank)
    if bufs.get("key") != key:
        hist_words, cap = shard_sizes(width, height, world)
        snd, rcv = shard_exchange(width, height, world, rank)
        bufs.clear()
        bufs["key"] = key
        bufs["hist"] = torch.zeros(hist_words, dtype=torch.int32, device=dev)
        bufs["send"] = torch.zeros(cap, dtype=torch.uint8, device=dev)
        bufs["recv"] = torch.zeros(cap, dtype=torch.uint8, device=dev)
        bufs["splits"] = (snd, rcv)
        # a collective is skipped only when NO rank exchanges (every rank
        # derives the same answer from the geometry)
        bufs["any"] = any(sum(shard_exchange(width, height, world, r)[0]) for r in range(world))
        # the zero fills run on torch's stream; the library writes these
        # buffers on its own stream -- without this wait a late fill could
        # clear the histogram shard_begin just wrote (seen: a rank's HF preset
        # with no histogram when the GPU was busy with earlier work)
        torch.cuda.synchronize(dev)
    hist, send, recv = bufs["hist"], bufs["send"], bufs["recv"]
    snd, rcv = bufs["splits"]
    enc.shard_begin(d_rgb.data_ptr(), width, height, rank, world, hist.data_ptr(),
                    send.data_ptr())
    ns, nr = sum(snd), sum(rcv)
    # one code path for both backends: under nccl (RCCL) the collectives run on
    # the HBM tensors themselves (`.to(comm)` returns the same tensor, the
    # copy-backs are skipped); gloo (the CPU rehearsal, e.g. several ranks on
    # one device) stages the same tensors through the host
    comm = _comm_device(dev, group)
    # ANS: one HF preset per rank -- every rank codes its groups
    # with its own histograms, no all-reduce; HfGlobal is built at assembly
    # from the presets in the payload heads.  Prefix codes: one preset from
    # the summed histogram.
    presets = bool(enc.params.flags & FLAG_ANS)
    if not presets:
        h = hist.to(comm)
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        _copy_back(hist, h)
    if bufs["any"]:
        r = recv[:nr] if comm == dev else torch.empty(nr, dtype=torch.uint8, device=comm)
        dist.all_to_all_single(r, send[:ns].to(comm), output_split_sizes=rcv,
                               input_split_sizes=snd, group=group)
        _copy_back(recv[:nr], r)
    torch.cuda.synchronize(dev)  # the library's stream reads what the collectives wrote
    size = enc.shard_end(hist.data_ptr(), recv.data_ptr())
    if host is not None:
        heads = _all_gather_heads(enc.shard_head(), rank, world, width, height, group)
        ok, total = enc.shard_write_host(heads, host.addr, host.cap)
        if not ok:  # same `total` on every rank: all grow together
            host.ensure(total)
            ok, total = enc.shard_write_host(heads, host.addr, host.cap)
        dist.barrier(group=group)  # every rank's sections are in place
        if rank != 0:
            return None
        v = host.view(total)
        return bytes(v) if copy else v
    # device assembly: payloads gathered into one buffer on rank 0 (RCCL,
    # device to device; the gloo rehearsal stages the same gather through the
    # host), which assembles them with the concat kernel
    n = torch.tensor([size], dtype=torch.int64, device=comm)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    # payload buffers under their own keys: "send" / "recv" are the record
    # exchange's (reused by the next frame's shard_begin / shard_end)
    cap = (max(sizes) + 15) // 16 * 16
    if bufs.get("pcap", 0) < cap:
        bufs["pcap"] = cap
        bufs["psend"] = torch.empty(cap, dtype=torch.uint8, device=dev)
        bufs["precv"] = torch.empty(world * cap + 64, dtype=torch.uint8, device=dev) \
            if rank == 0 else None
        torch.cuda.synchronize(dev)  # allocated on torch's stream, written on the library's
    psend = bufs["psend"][:cap]
    enc.shard_payload(psend.data_ptr(), on_device=True)  # returns with the copy complete
    precv = bufs["precv"]
    views = [precv[r * cap:(r + 1) * cap] for r in range(world)] if rank == 0 else None
    parts = None
    if rank == 0:
        parts = views if comm == dev else [torch.empty(cap, dtype=torch.uint8, device=comm)
                                           for _ in range(world)]
    dist.gather(psend.to(comm), parts, dst=0, group=group)
    if rank == 0:
        for v, part in zip(views, parts):
            _copy_back(v, part)
    if rank != 0:
        return None
    torch.cuda.synchronize(dev)
    return enc.shard_assemble_device(precv.data_ptr(), [r * cap for r in range(world)], sizes,
                                     copy=copy)


def shared_gpu_lanes(ranks_on_device: int, queues: int = 16) -> int | None:
    """Lane cap for each of `ranks_on_device` ranks streaming on one GPU: the
    process-wide hardware queues (GPU_MAX_HW_QUEUES, bench.py 16) less one,
    split between them, at least two (one lane per rank serialises its frames:
    8 contexts 0.69 GPix/s at 1 lane, 3.9 at 2, 4.0 at 3, profiles/r04q);
    None: a rank has its GPU to itself."""
    if ranks_on_device <= 1:
        return None
    return max(2, (queues - 1) // ranks_on_device)


class ShardStream:
    """Streaming group-sharded encode (jxg_shard_submit_device /
    jxg_shard_next_head / jxg_shard_write_next), the multi-GPU pipeline
    bench.py --gpus N times.  Every rank submits its shard
    of the same frames in the same order; frames flow through the library's
    pipeline lanes (front end, merge stage, statistics, codes and rANS chains
    of up to jxg_pipeline_depth frames overlap) with no collective inside a
    frame.  Per frame, in order, each rank
      1. takes its payload head (the oldest frame's sections emitted),
      2. publishes it in the node-shared /dev/shm region (slot k % S) and
         reads the other ranks' heads there (a sequence word per rank and
         slot: spin until every rank has published frame k),
      3. DMAs its sections into frame k's codestream slot (rank 0 adds headers
         + TOC) -- the copies run on while it goes on; it marks frame k done
         once write_next of frame k + WRITE_LAG (or a flush) has returned.
    Rank 0's :meth:`receive` returns a zero-copy view of frame k's codestream
    once every rank has marked it done; other ranks get None.  **The view is
    valid only until the next receive** (receive(k + 1) releases frame k's slot
    to the writers; round 5 changed this from "the next S - 1 receives"):
    keep a copy (``receive(copy=True)`` or ``bytes(view)``) to hold a frame
    longer.  A frame is written into slot k % S only once rank 0 has
    released frame k - S (called receive for a later frame), so at most
    depth + S - 2 frames may be pending: :meth:`submit` raises beyond.  All ranks must run on one node (the shared
    mapping); the partition must need no record exchange and the coder must
    be ANS when world > 1 (jxg_shard_submit_device refuses otherwise).
    `lanes` caps the rank's pipeline lanes (jxg_set_pipeline_lanes): for
    ranks sharing one GPU, :func:`shared_gpu_lanes`."""

    def __init__(self, enc: Encoder, width: int, height: int, rank: int, world: int,
                 group=None, slots: int = 6, slot_bytes: int | None = None,
                 lanes: int | None = None):
        self.enc, self.w, self.h, self.rank, self.world = enc, width, height, rank, world
        if slots <= WRITE_LAG:
            # a rank marks frame k done only after writing frame k + WRITE_LAG,
            # and writing frame k waits for slot k % slots (frame k - slots) to
            # be done on every rank, its own included
            raise ValueError("ShardStream needs slots > %d (got %d)" % (WRITE_LAG, slots))
        if lanes is not None:  # ranks sharing one GPU split its hardware queues
            enc.set_pipeline_lanes(lanes)
        self.depth = enc.pipeline_depth(width, height, rank, world)
        self.slots = slots
        self.hcap = _head_cap(width, height)
        # codestream slot: 12 bpp + 1 MiB (a d1 8K frame is ~2 bpp); a frame
        # over it raises (pass slot_bytes)
        self.slot_bytes = slot_bytes or ((width * height * 3 // 2 + (1 << 20) + 4095) & ~4095)
        # int64: published[S][W], done[S][W], released (frames rank 0 is done with)
        self.meta_words = 2 * slots * world + 1
        self.heads_off = 8 * self.meta_words
        self.data_off = (self.heads_off + 4 * slots * world * self.hcap + 4095) & ~4095
        self.host = SharedHostBuffer(rank, world, group)
        self.host.ensure(self.data_off + slots * self.slot_bytes)
        self.meta = np.frombuffer(self.host.mm, dtype=np.int64, count=self.meta_words)
        if rank == 0:
            self.meta[:] = -1
            self.meta[-1] = 0
        dist.barrier(group=group)
        self.published = self.meta[:slots * world].reshape(slots, world)
        self.done = self.meta[slots * world:2 * slots * world].reshape(slots, world)
        self.heads = np.frombuffer(self.host.mm, dtype=np.uint32,
                                   count=slots * world * self.hcap,
                                   offset=self.heads_off).reshape(slots, world, self.hcap)
        self.max_pending = self.depth  # (more pending: submit writes the oldest out)
        self.max_ahead = self.depth + slots - 2  # pending frames submit accepts
        self.submitted = 0   # frames submitted
        self.written = 0     # frames whose sections this rank has written
        self.received = 0    # frames returned by receive()
        self.unmarked = []   # frames written whose copies may be in flight (not done yet)
        self.totals = {}
        self.wait_s = 0.0    # seconds spent waiting for the other ranks (heads, slots, frames)

    def _wait(self, cond, what):
        t0 = time.perf_counter()
        spins, told = 0, False
        if cond():
            return
        while not cond():
            spins += 1
            if spins > 64:
                time.sleep(20e-6)
            dt = time.perf_counter() - t0
            if dt > 10 and not told:  # a rank is far behind (or gone): say so once
                import sys
                print("ShardStream rank %d: waiting %.0f s for %s" % (self.rank, dt, what),
                      file=sys.stderr, flush=True)
                told = True
            if dt > 120:
                raise RuntimeError("ShardStream: timed out waiting for " + what)
        self.wait_s += time.perf_counter() - t0

    def pending(self) -> int:
        return self.submitted - self.received

    def ready(self) -> int:
        """Frames already written by this rank (receive may still wait for
        the other ranks)."""
        return self.written - self.received

    def submit(self, ptr: int):
        """Queue this rank's shard of the next frame (device RGB8, unchanged
        until the frame is received).  When the library's lanes are all busy
        the oldest frame is written out first (its codestream is then taken by
        a later :meth:`receive`)."""
        if self.submitted - self.received >= self.max_ahead:
            raise RuntimeError("ShardStream: %d frames pending (at most depth + slots - 2 = "
                               "%d): receive first" % (self.pending(), self.max_ahead))
        if self.submitted - self.written >= self.depth:
            self._write_one()
        self.enc.shard_submit_device(ptr, self.w, self.h, self.rank, self.world)
        self.submitted += 1

    def _write_one(self):
        k = self.written
        s, r = k % self.slots, self.rank
        head = self.enc.shard_next_head()
        if head.size > self.hcap:
            raise RuntimeError("payload head of %d words over %d" % (head.size, self.hcap))
        # slot s was last used by frame k - S: every rank must be done with it
        # (this rank's own part: flushed here if it is still unmarked)
        if self.unmarked and self.unmarked[0] <= k - self.slots:
            self._mark()
        self._wait(lambda: bool((self.done[s] >= k - self.slots).all()), "slot %d" % s)
        # ... and rank 0 must have released the frame it held (receive of a
        # later frame): on rank 0 itself the submit bound guarantees it
        self._wait(lambda: int(self.meta[-1]) > k - self.slots, "release of frame %d" % (k - self.slots))
        self.heads[s, r, :head.size] = head
        self.published[s, r] = k          # (x86: the head's stores are visible first)
        self._wait(lambda: bool((self.published[s] >= k).all()), "heads of frame %d" % k)
        heads = [self.heads[s, q, :_head_len(self.heads[s, q])].copy() for q in range(self.world)]
        base = self.host.addr + self.data_off + s * self.slot_bytes
        ok, total = self.enc.shard_write_next(heads, base, self.slot_bytes)
        if not ok:
            raise RuntimeError("codestream of %d bytes over the %d-byte slot" % (total,
                                                                               self.slot_bytes))
        self.totals[k] = total
        # write_next returned once the copies of the frame WRITE_LAG writes
        # back had landed (include/jxg.h JXG_SHARD_WRITE_LAG)
        self.unmarked.append(k)
        while len(self.unmarked) > WRITE_LAG:
            j = self.unmarked.pop(0)
            self.done[j % self.slots, r] = j
        self.written += 1

    def _mark(self):
        """This rank's parts of the frames written are in place (flush)."""
        if self.unmarked:
            self.enc.shard_write_flush()
            for j in self.unmarked:
                self.done[j % self.slots, self.rank] = j
            self.unmarked = []

    def receive(self, copy: bool = False):
        """The oldest frame not yet received: rank 0 gets a numpy view of its
        codestream, valid until the next receive (which releases its slot), or
        with copy=True its bytes; other ranks None."""
        k = self.received
        if k >= self.submitted:
            raise RuntimeError("ShardStream: nothing pending")
        if self.rank == 0:
            self.meta[-1] = k  # frames < k released (the view of k - 1 ends here)
        while self.written <= k:
            self._write_one()
        if self.unmarked and self.unmarked[0] <= k:
            self._mark()
        self.received += 1
        total = self.totals.pop(k)
        if self.rank != 0:
            return None
        s = k % self.slots
        self._wait(lambda: bool((self.done[s] >= k).all()), "frame %d" % k)
        v = self.host.view(total, self.data_off + s * self.slot_bytes)
        return v.tobytes() if copy else v

    def close(self):
        while self.received < self.submitted:
            self.receive()
        dist.barrier(group=self.host.group)
        self.meta = self.published = self.done = self.heads = None
        self.host.close()
