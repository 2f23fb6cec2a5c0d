"""Multi-GPU group-sharded encode over torch.distributed.

One process per GPU (backend "nccl" = RCCL over xGMI).  Each rank encodes a
balanced contiguous raster range of the frame's 256x256 pass groups; the only
collectives are
  1. all_reduce(sum) of the AC token histogram (132 x 128 u32, 68 KB) so all
     ranks derive the same prefix codes,
  2. all_gather of the per-block records (strategy, quant field, quantized DC;
     14 B per 8x8 block) that the LF-group streams of other ranks read,
  3. a gather of the per-rank section payloads on rank 0, which writes the
     headers and TOC (jxg_shard_assemble, host only).
The result is byte-identical to a single-GPU encode of the same frame.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import Encoder, shard_assemble, shard_sizes


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
                   world: int, group=None, bufs=None, copy: bool = True):
    """Encode one frame (device-resident (H, W, 3) uint8 on every rank) with
    group sharding; returns the codestream on rank 0 (bytes, or a
    :class:`jxg.Codestream` view of pinned memory with copy=False), None
    elsewhere.  `bufs` caches the exchange tensors across calls."""
    dev = d_rgb.device
    hist_words, slot = shard_sizes(width, height, world)
    if bufs is None:
        bufs = {}
    key = (width, height, world)
    if bufs.get("key") != key:
        bufs.clear()
        bufs["key"] = key
        bufs["hist"] = torch.zeros(hist_words, dtype=torch.int32, device=dev)
        bufs["xbuf"] = torch.zeros(world * slot, dtype=torch.uint8, device=dev)
    hist, xbuf = bufs["hist"], bufs["xbuf"]
    enc.shard_begin(d_rgb.data_ptr(), width, height, rank, world, hist.data_ptr(),
                    xbuf.data_ptr())
    mine = xbuf[rank * slot:(rank + 1) * slot]
    gloo = dist.get_backend(group) == "gloo"
    if gloo:
        # host staging (gloo: CPU rehearsal of the exchange, e.g. several ranks
        # on one device); the nccl (RCCL) path below keeps everything in HBM
        h = hist.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        hist.copy_(h)
        parts = [torch.empty(slot, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, mine.cpu(), group=group)
        xbuf.copy_(torch.cat(parts))
    else:
        dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
        dist.all_gather_into_tensor(xbuf, mine.clone(), group=group)
    torch.cuda.synchronize(dev)  # the library's stream reads what the collectives wrote
    size = enc.shard_end(hist.data_ptr(), xbuf.data_ptr())
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
