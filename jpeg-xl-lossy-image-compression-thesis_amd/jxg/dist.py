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
            (device to device), which writes headers + TOC and moves every
            section with the concat kernel, then one D2H of the codestream.
With prefix codes the result is byte-identical to a single-GPU encode of the
same frame; with ANS it decodes to the same image (same coefficients, strategy,
quant field, DC and CfL maps) with per-rank histograms.
"""
from __future__ import annotations

import ctypes
import mmap
import os

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

    def view(self, n: int) -> np.ndarray:
        """zero-copy view of the codestream; valid until the next frame's
        write into the buffer (or close)"""
        return np.frombuffer(self.mm, dtype=np.uint8, count=n)

    def close(self):
        self._release()
        self.cap = 0


AC_CONTEXTS = 7425   # AC contexts of one HF preset (15 block contexts x 495)
ANS_MAX_HISTS = 8    # histograms per preset (csrc/jxg_bitstream.h kAnsMaxHists)
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


def encode_sharded(enc: Encoder, d_rgb: torch.Tensor, width: int, height: int, rank: int,
                   world: int, group=None, bufs=None, copy: bool = True,
                   host: SharedHostBuffer | None = None):
    """Encode one frame (device-resident (H, W, 3) uint8 on every rank) with
    group sharding; returns the codestream on rank 0 (bytes, or a zero-copy
    view with copy=False: a :class:`jxg.Codestream` of pinned memory, or with
    ``host`` a numpy view of the shared buffer), None elsewhere.  `bufs`
    caches the exchange tensors across calls."""
    dev = d_rgb.device
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
    gloo = dist.get_backend(group) == "gloo"
    # ANS: one HF preset per rank -- every rank codes its groups
    # with its own histograms, no all-reduce; HfGlobal is built at assembly
    # from the presets in the payload heads.  Prefix codes: one preset from
    # the summed histogram.
    presets = bool(enc.params.flags & FLAG_ANS)
    if gloo:
        # host staging (gloo: CPU rehearsal of the exchange, e.g. several ranks
        # on one device); the nccl (RCCL) path below keeps everything in HBM
        if not presets:
            h = hist.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            hist.copy_(h)
        if bufs["any"]:
            r_cpu = torch.empty(nr, dtype=torch.uint8)
            dist.all_to_all_single(r_cpu, send[:ns].cpu(), output_split_sizes=rcv,
                                   input_split_sizes=snd, group=group)
            recv[:nr].copy_(r_cpu)
    else:
        if not presets:
            dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
        if bufs["any"]:
            dist.all_to_all_single(recv[:nr], send[:ns], output_split_sizes=rcv,
                                   input_split_sizes=snd, group=group)
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
    if gloo:
        payloads = gather_payloads(enc.shard_payload_bytes(size), rank, world, "cpu", group)
        return shard_assemble(payloads) if rank == 0 else None
    # payloads gathered device to device into one buffer on rank 0
    n = torch.tensor([size], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    cap = (max(sizes) + 15) // 16 * 16
    if bufs.get("cap", 0) < cap:
        bufs["cap"] = cap
        bufs["send"] = torch.empty(cap, dtype=torch.uint8, device=dev)
        bufs["recv"] = torch.empty(world * cap + 64, dtype=torch.uint8, device=dev) \
            if rank == 0 else None
    cap_alloc = bufs["cap"]
    send = bufs["send"][:cap]
    enc.shard_payload(send.data_ptr(), on_device=True)
    recv = bufs["recv"]
    views = [recv[r * cap:(r + 1) * cap] for r in range(world)] if rank == 0 else None
    dist.gather(send, views, dst=0, group=group)
    del cap_alloc
    if rank != 0:
        return None
    torch.cuda.synchronize(dev)
    return enc.shard_assemble_device(recv.data_ptr(), [r * cap for r in range(world)], sizes,
                                     copy=copy)
