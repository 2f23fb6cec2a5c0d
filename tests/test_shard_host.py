"""Group sharding, host side (no GPU): the payload format, the section
ownership of jxg_host.cpp make_plan and the host-only jxg_shard_assemble,
pinned against the CPU oracle's codestream -- split into per-rank payloads
by the TOC, exchanged over torch.distributed (gloo, world size 2) and
re-assembled byte for byte.  The GPU side of the same path (jxg_shard_begin /
jxg_shard_end) is covered by tests/test_gpu_shard.py."""
import os

import numpy as np
import pytest


def oracle_sections(oracle, decoder, img, d=1.0, e=7, p=0):
    ref = oracle.encode(img, d, e, p)
    dec = decoder.decode(ref.bytes, want_pixels=False)
    secs = [ref.bytes[o:o + s] for o, s in zip(dec.section_offsets, dec.section_sizes)]
    return ref.bytes, secs


def payloads_for(jxg, w, h, world, secs):
    out = []
    for r in range(world):
        ids = jxg.shard_sections(w, h, r, world)
        out.append(jxg.make_payload(r, world, w, h, [(i, secs[i]) for i in ids]))
    return out


CASES = [(520, 300, 2), (777, 333, 3), (1000, 700, 4), (2100, 600, 8)]


@pytest.mark.parametrize("w,h,world", CASES)
def test_assemble_matches_oracle(jxg_mod, oracle, decoder, w, h, world):
    from jxg.synth import synth_rgb8

    full, secs = oracle_sections(oracle, decoder, synth_rgb8(w, h, w + h))
    assert len(secs) == 2 + jxg_mod.lf_group_count(w, h) + jxg_mod.group_count(w, h)
    # every section owned by exactly one rank
    owned = sorted(i for r in range(world) for i in jxg_mod.shard_sections(w, h, r, world))
    assert owned == list(range(len(secs)))
    assert jxg_mod.shard_assemble(payloads_for(jxg_mod, w, h, world, secs)) == full


def test_assemble_rejects_bad_payloads(jxg_mod, oracle, decoder):
    from jxg.synth import synth_rgb8

    w, h, world = 600, 300, 2
    _, secs = oracle_sections(oracle, decoder, synth_rgb8(w, h, 3))
    pl = payloads_for(jxg_mod, w, h, world, secs)
    with pytest.raises(jxg_mod.JxgError):
        jxg_mod.shard_assemble(pl[:1])            # a rank missing
    with pytest.raises(jxg_mod.JxgError):
        jxg_mod.shard_assemble([pl[0], pl[0]])    # sections twice
    with pytest.raises(jxg_mod.JxgError):
        jxg_mod.shard_assemble([pl[0][:20], pl[1]])  # truncated


def _gloo_worker(rank, world, port, w, h, secs, full, result):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import numpy as np

        import jxg
        from jxg.dist import _all_gather_heads, gather_payloads

        ids = jxg.shard_sections(w, h, rank, world)
        payload = jxg.make_payload(rank, world, w, h, [(i, secs[i]) for i in ids])
        got = gather_payloads(payload, rank, world, "cpu")
        # payload heads (7 + 2 x sections words) in one fixed-capacity all-gather
        head = np.frombuffer(payload[:4 * (7 + 2 * len(ids))], dtype=np.uint32)
        heads = _all_gather_heads(head, rank, world, w, h)
        heads_ok = (len(heads) == world and np.array_equal(heads[rank], head) and
                    all(int(hd[2]) == r and hd.size == 7 + 2 * int(hd[6])
                        for r, hd in enumerate(heads)))
        if rank == 0:
            result.put((jxg.shard_assemble(got) == full, heads_ok))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gather_and_assemble(jxg_mod, oracle, decoder):
    import socket

    import torch.multiprocessing as mp
    from jxg.synth import synth_rgb8

    w, h, world = 1000, 520, 2
    full, secs = oracle_sections(oracle, decoder, synth_rgb8(w, h, 11))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, w, h, secs, full, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) == (True, True)


def partition_py(w, h, world):
    """Restatement of jxg_host.cpp make_partition (include/jxg.h): kind 0
    contiguous raster ranges when no LF group is split over ranks; else kind 1
    whole LF groups (largest pixel area first, ties by index, to the
    least-loaded rank, ties to the lower rank) when the largest load is within
    5 % of the mean; else kind 2 (ranges + the record exchange)."""
    gxs, gys = -(-w // 256), -(-h // 256)
    lfxs, lfys = -(-w // 2048), -(-h // 2048)
    ng, nlf = gxs * gys, lfxs * lfys
    if world == 1:
        return [0] * ng, [0] * nlf, 0

    def shard_of(g):
        r = g * world // ng
        while r + 1 < world and ng * (r + 1) // world <= g:
            r += 1
        while r > 0 and ng * r // world > g:
            r -= 1
        return r

    def lf_of(g):
        return (g // gxs) // 8 * lfxs + (g % gxs) // 8

    grp = [shard_of(g) for g in range(ng)]
    own, nas = [], [0] * world
    for lg in range(nlf):
        lx, ly = lg % lfxs, lg // lfxs
        cnt = [0] * world
        for gy in range(ly * 8, min(ly * 8 + 8, gys)):
            for gx in range(lx * 8, min(lx * 8 + 8, gxs)):
                cnt[shard_of(gy * gxs + gx)] += 1
        best, bs = -1, 0
        for r in range(world):
            if cnt[r] and (best < 0 or cnt[r] - 16 * nas[r] > bs):
                best, bs = r, cnt[r] - 16 * nas[r]
        own.append(best)
        nas[best] += 1
    if all(own[lf_of(g)] == grp[g] for g in range(ng)):
        return grp, own, 0
    if nlf >= world:
        area = [min(2048, w - (lg % lfxs) * 2048) * min(2048, h - (lg // lfxs) * 2048)
                for lg in range(nlf)]
        load, lfo = [0] * world, [0] * nlf
        for lg in sorted(range(nlf), key=lambda i: -area[i]):
            r = min(range(world), key=lambda q: (load[q], q))
            lfo[lg] = r
            load[r] += area[lg]
        if min(load) > 0 and max(load) * 100 * world <= sum(area) * 105:
            return [lfo[lf_of(g)] for g in range(ng)], lfo, 1
    return grp, own, 2


SHAPES = [(7680, 4320, 2), (7680, 4320, 4), (7680, 4320, 8), (16384, 16384, 8),
          (3840, 2160, 2), (3840, 2160, 4), (2100, 600, 8), (4100, 5000, 3), (4096, 512, 2),
          (8192, 512, 4), (1920, 1080, 1)]


@pytest.mark.parametrize("w,h,world", SHAPES)
def test_partition_matches_restatement(jxg_mod, w, h, world):
    assert jxg_mod.shard_plan(w, h, world) == partition_py(w, h, world)


def test_partition_kinds(jxg_mod):
    """BASELINE config 2 (8K) over 2 / 4 / 8 ranks: whole LF groups, balanced
    to a few percent, no record exchange; config 4 (16384^2 over 8): aligned
    ranges."""
    for world in (2, 4, 8):
        go, lo, kind = jxg_mod.shard_plan(7680, 4320, world)
        assert kind == 1
        cnt = [go.count(r) for r in range(world)]
        assert max(cnt) <= 1.05 * 510 / world
        assert all(sum(jxg_mod.shard_exchange(7680, 4320, world, r)[0]) == 0 for r in range(world))
    go, lo, kind = jxg_mod.shard_plan(16384, 16384, 8)
    assert kind == 0 and go == [g * 8 // 4096 for g in range(4096)]


@pytest.mark.parametrize("w,h,world", SHAPES)
def test_record_exchange_plan(jxg_mod, w, h, world):
    """jxg_shard_exchange (C++) against the partition: a rank sends each of its
    pass groups' records to the owner of the group's LF group (if another
    rank), receives the other ranks' groups inside its own LF groups; sends
    and receives pair up across ranks."""
    rec = 1024 * 2 + 1024 * 4 * 3 + 32  # acs, qf, DC, and the 16 colour tiles ytox / ytob
    go, owners, kind = jxg_mod.shard_plan(w, h, world)
    gxs = -(-w // 256)
    lfxs = -(-w // 2048)
    ng = len(go)
    plan = [jxg_mod.shard_exchange(w, h, world, r) for r in range(world)]
    for r in range(world):
        snd, rcv = plan[r]
        for p in range(world):
            want = sum(1 for g in range(ng)
                       if go[g] == r and p != r and owners[(g // gxs) // 8 * lfxs + (g % gxs) // 8] == p)
            assert snd[p] == want * rec
            assert rcv[p] == plan[p][0][r]  # what p sends to r
    assert all(0 <= o < world for o in owners)
    _, cap = jxg_mod.shard_sizes(w, h, world)
    assert all(max(sum(s), sum(rv)) <= cap for s, rv in plan)
    assert (kind == 2) == any(sum(s) for s, _ in plan)


def _v2_payload(rank, world, w, h, sections, nh=1, cm=None, counts=None, fix_b=None):
    """A version-2 payload (one HF preset per rank, jxg_host.cpp shard_finish):
    head, [B][nhist][context map bytes in words][counts nhist x 128], body."""
    cw = (7425 + 3) // 4
    cm = np.zeros(7425, dtype=np.uint8) if cm is None else cm
    counts = np.full((nh, 128), 0, dtype=np.uint32) if counts is None else counts
    if counts.size:
        counts[:, 0] = 1000
        counts[:, 1] = 24
    cmw = np.zeros(cw * 4, dtype=np.uint8)
    cmw[:7425] = cm
    B = 1 + cw + counts.size if fix_b is None else fix_b
    head = np.array([0x5347584A, 2, rank, world, w, h, len(sections)] +
                    [v for i, b in sections for v in (i, len(b))] + [B, nh], dtype="<u4")
    body = head.tobytes() + cmw.tobytes() + counts.astype("<u4").tobytes()
    return body + b"".join(b for _, b in sections)


def test_assemble_v2_presets(jxg_mod):
    """Host-only assembly of version-2 payload heads (ANS, one HF preset per
    rank): HfGlobal is generated from the presets (num_hf_presets = ranks);
    malformed preset blocks are refused."""
    w, h, world = 4096, 512, 2
    ids = [jxg_mod.shard_sections(w, h, r, world, ans=True) for r in range(world)]
    nlf = jxg_mod.lf_group_count(w, h)
    assert 1 + nlf not in ids[0] + ids[1]  # HfGlobal comes from the presets
    secs = {i: bytes([(i * 7 + k) & 255 for k in range(5 + i % 3)]) for r in ids for i in r}
    good = [_v2_payload(r, world, w, h, [(i, secs[i]) for i in ids[r]]) for r in range(world)]
    out = jxg_mod.shard_assemble(good)
    body = sum(len(b) for b in secs.values())
    assert len(out) > body
    for r in range(world):  # every section's bytes appear in the codestream
        for i in ids[r]:
            assert secs[i] in out
    bad = []
    bad.append([_v2_payload(0, world, w, h, [(i, secs[i]) for i in ids[0]], nh=0), good[1]])
    bad.append([_v2_payload(0, world, w, h, [(i, secs[i]) for i in ids[0]], nh=9,
                            counts=np.zeros((9, 128), dtype=np.uint32)), good[1]])
    cm = np.zeros(7425, dtype=np.uint8)
    cm[100] = 1  # context mapped past the preset's one histogram
    bad.append([_v2_payload(0, world, w, h, [(i, secs[i]) for i in ids[0]], cm=cm), good[1]])
    bad.append([_v2_payload(0, world, w, h, [(i, secs[i]) for i in ids[0]], fix_b=5), good[1]])
    # a version-1 rank among version-2 ranks
    bad.append([jxg_mod.make_payload(0, world, w, h, [(i, secs[i]) for i in ids[0]]), good[1]])
    for pl in bad:
        with pytest.raises(jxg_mod.JxgError):
            jxg_mod.shard_assemble(pl)


def test_shared_gpu_lanes_split():
    """Ranks rehearsed on one GPU split its hardware queues (GPU_MAX_HW_QUEUES
    - 1), at least two lanes each; a rank alone on its GPU is not capped."""
    from jxg.dist import shared_gpu_lanes

    assert shared_gpu_lanes(1) is None and shared_gpu_lanes(0) is None
    assert [shared_gpu_lanes(k) for k in (2, 3, 4, 5, 8, 16)] == [7, 5, 3, 3, 2, 2]
    assert shared_gpu_lanes(2, queues=32) == 15


def test_shard_stream_rejects_too_few_slots(jxg_mod):
    """a rank marks frame k done after writing frame
    k + WRITE_LAG and writing frame k waits for frame k - slots on every rank,
    so slots <= WRITE_LAG would wait on itself; the constructor refuses it
    before touching the encoder or the shared region."""
    import pytest

    from jxg import dist as jd

    for slots in range(0, jd.WRITE_LAG + 1):
        with pytest.raises(ValueError):
            jd.ShardStream(None, 64, 64, 0, 1, slots=slots)


class _FakeShardEnc:
    """Stands in for jxg.Encoder in ShardStream's protocol tests (no GPU):
    frame k's codestream is 100 bytes of value k & 255, written synchronously
    into the slot; the head is an empty version-1 head."""

    def __init__(self, depth):
        self.depth, self.sub, self.wrote = depth, 0, 0

    def pipeline_depth(self, w, h, rank=0, world=1):
        return self.depth

    def shard_submit_device(self, ptr, w, h, rank, world):
        assert self.sub - self.wrote < self.depth, "the library's lanes are full"
        self.sub += 1

    def shard_next_head(self):
        h = np.zeros(7, dtype=np.uint32)
        h[1] = 1
        return h

    def shard_write_next(self, heads, base, size):
        import ctypes

        ctypes.memmove(base, bytes([self.wrote & 255]) * 100, 100)
        self.wrote += 1
        return True, 100

    def shard_write_flush(self):
        pass


def test_shard_stream_slot_release(jxg_mod, monkeypatch):
    """Writing ahead of receive (submit past the library's depth): a frame
    goes into slot k % slots only once rank 0 released frame k - slots, and
    submit refuses more than depth + slots - 2 pending frames -- so a frame
    whose codestream has not been received is never overwritten.  slots = 3
    (the smallest accepted), depth 2, world 1 (gloo)."""
    import socket

    import pytest
    import torch.distributed as dist

    from jxg import dist as jd

    class _NoPin:  # page-locking needs a HIP device: not part of the protocol
        @staticmethod
        def jxg_host_register(addr, size):
            return 0

        @staticmethod
        def jxg_host_unregister(addr):
            return 0

    monkeypatch.setattr(jd, "load", lambda: _NoPin)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    try:
        enc = _FakeShardEnc(depth=2)
        ss = jd.ShardStream(enc, 64, 64, 0, 1, slots=3)
        assert ss.max_ahead == 3
        got = []
        for k in range(3):  # frame 0 is written from submit (lanes full at 2)
            ss.submit(0)
        assert ss.written == 1 and ss.pending() == 3
        with pytest.raises(RuntimeError, match="receive first"):
            ss.submit(0)
        for k in range(3, 12):
            got.append(bytes(ss.receive()))
            ss.submit(0)  # writes ahead: frame k - 1 while k - 2 is received
        while ss.pending():
            got.append(bytes(ss.receive()))
        assert got == [bytes([k]) * 100 for k in range(12)]
        ss.close()
    finally:
        dist.destroy_process_group()
