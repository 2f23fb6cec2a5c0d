"""GPU group sharding on one device: `world` contexts play the
ranks, the collectives are done with torch ops (sum of the histograms; the
all_to_all of the per-block records by the jxg_shard_exchange splits), and the
assembled codestream must equal the single-context
encode byte for byte (one AC histogram -> one HF preset, so sharding does not
change a bit).  The multi-process RCCL version of the same exchange is
jxg.dist.encode_sharded (bench.py --gpus N)."""
import ctypes
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def sharded_encode(jxg_mod, img, world, d=1.0, e=7, p=0, flags=0, t=None):
    import torch

    if t is None:
        h, w, _ = img.shape
        t = torch.from_numpy(np.ascontiguousarray(img)).cuda()
    else:
        h, w, _ = t.shape
    hist_words, cap = jxg_mod.shard_sizes(w, h, world)
    plan = [jxg_mod.shard_exchange(w, h, world, r) for r in range(world)]
    encs = [jxg_mod.Encoder(distance=d, effort=e, proposals=p, flags=flags) for _ in range(world)]
    hists = [torch.zeros(hist_words, dtype=torch.int32, device="cuda") for _ in range(world)]
    sends = [torch.zeros(cap, dtype=torch.uint8, device="cuda") for _ in range(world)]
    # the contexts' streams are not ordered after torch's: the frame and the
    # zero-filled buffers must be complete first (include/jxg.h)
    torch.cuda.synchronize()
    for r in range(world):
        encs[r].shard_begin(t.data_ptr(), w, h, r, world, hists[r].data_ptr(), sends[r].data_ptr())
    # prefix codes: one HF preset from the summed histogram; ANS: one preset
    # per rank (its own histogram, no all-reduce)
    presets = bool(flags & jxg_mod.FLAG_ANS) and world > 1
    hist = torch.stack(hists).sum(0).to(torch.int32).contiguous()

    def segment(src, dst):  # src's records for dst (send order: by destination)
        snd = plan[src][0]
        o = sum(snd[:dst])
        return sends[src][o:o + snd[dst]]

    recvs = []
    for r in range(world):
        parts = [segment(q, r) for q in range(world) if q != r]
        rb = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        if parts:
            cat = torch.cat(parts)
            assert cat.numel() == sum(plan[r][1])
            rb[:cat.numel()] = cat
        recvs.append(rb)
    torch.cuda.synchronize()
    payloads = []
    for r in range(world):
        size = encs[r].shard_end((hists[r] if presets else hist).data_ptr(),
                                 recvs[r].data_ptr())
        payloads.append(encs[r].shard_payload_bytes(size))
    # distributed host assembly: every "rank" writes its sections into one
    # host buffer (first call with a too-small buffer reports the size)
    heads = [e.shard_head() for e in encs]
    ok, total = encs[0].shard_write_host(heads, 0, 0)
    assert not ok and total > 0
    hbuf = np.full(total + 7, 0xAB, dtype=np.uint8)
    for r in range(world):
        ok, t2 = encs[r].shard_write_host(heads, hbuf.ctypes.data, hbuf.size)
        assert ok and t2 == total
    host_written = hbuf[:total].tobytes()
    assert (hbuf[total:] == 0xAB).all()
    # device assembly on "rank 0" from one buffer (word-aligned offsets)
    cap = (max(len(p) for p in payloads) + 15) // 16 * 16
    blob = np.zeros(world * cap + 64, dtype=np.uint8)
    for r, p in enumerate(payloads):
        blob[r * cap:r * cap + len(p)] = np.frombuffer(p, dtype=np.uint8)
    d_blob = torch.from_numpy(blob).cuda()
    dev_out = encs[0].shard_assemble_device(d_blob.data_ptr(), [r * cap for r in range(world)],
                                            [len(p) for p in payloads])
    for enc in encs:
        enc.close()
    host_out = jxg_mod.shard_assemble(payloads)
    assert dev_out == host_out
    assert host_written == host_out
    return dev_out


CASES = [(520, 300, 2, 1.0, 7, 0), (777, 333, 3, 2.0, 5, 3), (1000, 700, 4, 1.0, 7, 2),
         (2100, 600, 8, 0.5, 4, 0), (1920, 1080, 5, 1.0, 7, 1)]


@pytest.mark.parametrize("w,h,world,d,e,p", CASES)
def test_sharded_equals_single(jxg_mod, w, h, world, d, e, p):
    from jxg.synth import synth_rgb8

    img = synth_rgb8(w, h, w * 3 + h)
    with jxg_mod.Encoder(distance=d, effort=e, proposals=p) as enc:
        ref = enc.encode(img)
    assert sharded_encode(jxg_mod, img, world, d, e, p) == ref


def test_sharded_8k_equals_single(jxg_mod):
    from jxg.synth import config_image

    img = config_image(2)
    with jxg_mod.Encoder(distance=1.0, effort=7) as enc:
        ref = enc.encode(img)
    assert sharded_encode(jxg_mod, img, 8) == ref


def _gloo_rank(rank, world, port, w, h, result, shm=False, flags=0):
    import os

    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import jxg
        from jxg.dist import SharedHostBuffer, encode_sharded
        from jxg.synth import synth_rgb8

        img = synth_rgb8(w, h, 5)
        t = torch.from_numpy(img).cuda()
        host = SharedHostBuffer(rank, world) if shm else None
        with jxg.Encoder(distance=1.0, effort=7, flags=flags) as enc:
            out = encode_sharded(enc, t, w, h, rank, world, host=host)
            out2 = encode_sharded(enc, t, w, h, rank, world, host=host)  # buffer reuse
            if rank == 0:
                ref = enc.encode(img)
                result.put((bytes(out), bytes(out2), ref))
        if host is not None:
            dist.barrier()
            host.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shm,ans", [(False, False), (True, False), (True, True), (False, True)])
def test_multiprocess_encode_sharded(jxg_mod, decoder, shm, ans):
    """jxg.dist.encode_sharded in 2 processes (gloo, both ranks on cuda:0):
    the multi-process orchestration bench.py --gpus N runs over RCCL; shm:
    the distributed host assembly into a /dev/shm buffer.  Prefix codes: the
    single-GPU bytes; ANS (one HF preset per rank, no histogram all-reduce):
    the single-GPU image."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    flags = jxg_mod.FLAG_ANS if ans else 0
    procs = [ctx.Process(target=_gloo_rank, args=(r, 2, port, 1100, 700, q, shm, flags))
             for r in range(2)]
    for p in procs:
        p.start()
    # read before joining: a child holding queued data does not exit until it
    # has been consumed
    got = q.get(timeout=280)
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    out, out2, ref = got
    assert out == out2
    if not ans:
        assert out == ref
    else:
        dr, dg = decoder.decode(ref), decoder.decode(out)
        assert dg.npresets == 2
        _same_image(dr, dg)


def _same_image(a, b):
    for k in ("acs", "qf", "dc", "ac", "cmap"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert np.array_equal(a.rgb, b.rgb)


@pytest.mark.parametrize("world", [2, 3, 5])
def test_sharded_ans_per_rank_presets(jxg_mod, decoder, world):
    """ANS sharding with one HF preset per rank (no histogram
    all-reduce): the codestream carries `world` presets, every pass group
    selects its rank's, and it decodes to exactly the single-GPU image."""
    from jxg.synth import synth_rgb8

    img = synth_rgb8(1500, 900, 17)
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS) as enc:
        ref = enc.encode(img)
    got = sharded_encode(jxg_mod, img, world, flags=jxg_mod.FLAG_ANS)
    dr, dg = decoder.decode(ref), decoder.decode(got)
    assert dr.npresets == 1 and dg.npresets == world
    go, _, _ = jxg_mod.shard_plan(1500, 900, world)
    assert list(dg.group_presets) == go  # every pass group selects its rank's preset
    _same_image(dr, dg)


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_8k_strong(jxg_mod, world):
    """BASELINE config 2 as written: one 8K frame split over `world` ranks
    (strong scaling), records exchanged only to the LF-group owners"""
    from jxg.synth import synth_rgb8_device

    t = synth_rgb8_device(7680, 4320, 0x4A584C02)
    with jxg_mod.Encoder(distance=1.0, effort=7) as enc:
        ref = enc.encode_device(t.data_ptr(), 7680, 4320)
    assert sharded_encode(jxg_mod, None, world, t=t) == ref


# ---------------------------------------------------------------------------
# streaming shards (jxg_shard_submit_device / next_head / write_next): the
# multi-GPU pipeline, `world` contexts of one process playing the ranks
# ---------------------------------------------------------------------------
def streamed_shards(jxg_mod, ts, w, h, world, d=1.0, e=7, p=0, flags=None, lanes=None):
    """Frames ts (device tensors) through `world` contexts' streaming shard
    pipelines; heads swapped in-process, sections written into one host
    buffer per frame.  Returns the codestreams in order.  lanes: each
    context's lane cap (jxg_set_pipeline_lanes)."""
    import torch

    flags = jxg_mod.FLAG_ANS if flags is None else flags
    torch.cuda.synchronize()  # the frames are written (no input stream set)
    encs = [jxg_mod.Encoder(distance=d, effort=e, proposals=p, flags=flags) for _ in range(world)]
    if lanes is not None:
        for enc in encs:
            enc.set_pipeline_lanes(lanes)
    depth = min(enc.pipeline_depth(w, h, r, world) for r, enc in enumerate(encs))
    outs = []
    buf = np.zeros(w * h * 2 + (1 << 20), dtype=np.uint8)

    def take():
        heads = [enc.shard_next_head() for enc in encs]
        buf[:] = 0xCD
        total = None
        for enc in encs:
            ok, t = enc.shard_write_next(heads, buf.ctypes.data, buf.size)
            assert ok and (total is None or t == total)
            total = t
        for enc in encs:  # write_next enqueues the copies: wait for them
            enc.shard_write_flush()
        outs.append(buf[:total].tobytes())

    for t in ts:
        for r, enc in enumerate(encs):
            enc.shard_submit_device(t.data_ptr(), w, h, r, world)
        if encs[0].pending() >= depth:
            take()
    while encs[0].pending():
        take()
    for enc in encs:
        assert enc.pending() == 0
        enc.close()
    return outs


def test_stream_shards_write_lag(jxg_mod):
    """the JXG_SHARD_WRITE_LAG promise with no flush -- each
    frame has its own host buffer, nothing is flushed until the end, and
    frame k's buffer is checked as soon as write_next of frame k + LAG has
    returned on every context (two contexts, two lanes each, so lane slots
    and their write events are re-used)."""
    import torch

    from jxg.synth import synth_rgb8_device

    w, h, world, n = 4096, 512, 2, 9
    lag = 2  # include/jxg.h JXG_SHARD_WRITE_LAG
    ts = [synth_rgb8_device(w, h, 0x1A6 + k) for k in range(n)]
    ref = streamed_shards(jxg_mod, ts, w, h, world, lanes=2)
    torch.cuda.synchronize()
    encs = [jxg_mod.Encoder(flags=jxg_mod.FLAG_ANS) for _ in range(world)]
    for enc in encs:
        enc.set_pipeline_lanes(2)
    depth = min(enc.pipeline_depth(w, h, r, world) for r, enc in enumerate(encs))
    bufs, totals, checked = [], [], []

    def take():
        k = len(bufs)
        heads = [enc.shard_next_head() for enc in encs]
        buf = np.full(w * h * 2 + (1 << 20), 0xCD, dtype=np.uint8)
        total = None
        for enc in encs:
            ok, t = enc.shard_write_next(heads, buf.ctypes.data, buf.size)
            assert ok and (total is None or t == total)
            total = t
        bufs.append(buf)
        totals.append(total)
        if k >= lag:  # frame k - lag has landed on every context
            j = k - lag
            assert bufs[j][:totals[j]].tobytes() == ref[j], "frame %d not in place" % j
            checked.append(j)

    for t in ts:
        for r, enc in enumerate(encs):
            enc.shard_submit_device(t.data_ptr(), w, h, r, world)
        if encs[0].pending() >= depth:
            take()
    while encs[0].pending():
        take()
    for enc in encs:
        enc.shard_write_flush()
        enc.close()
    assert checked == list(range(n - lag))
    assert [b[:t].tobytes() for b, t in zip(bufs, totals)] == ref


@pytest.mark.parametrize("w,h,world,nframes", [(4096, 512, 2, 9), (8192, 512, 4, 5), (1100, 700, 1, 14)])
def test_stream_shards_equal_one_at_a_time(jxg_mod, decoder, w, h, world, nframes):
    """Streamed shards (several frames in flight per rank, more than the
    pipeline depth for the 1-rank case) give the bytes of the one-frame-at-a-
    time sharded encode of every frame; they decode to the single-GPU image
    (ANS: one HF preset per rank)."""
    from jxg.synth import synth_rgb8_device

    ts = [synth_rgb8_device(w, h, 0x4A58 + 31 * k) for k in range(nframes)]
    got = streamed_shards(jxg_mod, ts, w, h, world)
    assert len(got) == nframes
    for k in (0, nframes // 2, nframes - 1):
        if world > 1:
            assert got[k] == sharded_encode(jxg_mod, None, world, flags=jxg_mod.FLAG_ANS, t=ts[k])
        else:  # world 1: the whole frame, == the single-GPU bytes
            with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS) as enc:
                assert got[k] == enc.encode_device(ts[k].data_ptr(), w, h)
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS) as enc:
        ref = enc.encode_device(ts[1].data_ptr(), w, h)
    dr, dg = decoder.decode(ref), decoder.decode(got[1])
    assert dg.npresets == world
    _same_image(dr, dg)


def test_stream_8k_over_8(jxg_mod):
    """The 8K ANS frame over 8 streamed shards (the driver's 8-GPU bench shape,
    here 8 contexts on one GPU) == the one-at-a-time sharded bytes."""
    from jxg.synth import synth_rgb8_device

    ts = [synth_rgb8_device(7680, 4320, 0x4A584C02 + k) for k in range(3)]
    got = streamed_shards(jxg_mod, ts, 7680, 4320, 8, lanes=2)
    for k in (0, 2):
        assert got[k] == sharded_encode(jxg_mod, None, 8, flags=jxg_mod.FLAG_ANS, t=ts[k])


def test_stream_shards_lane_cap(jxg_mod):
    """jxg_set_pipeline_lanes (ranks sharing one GPU): the depth follows the
    cap, (lanes - 1) x batch + 1; the bytes do not change with it; the cap
    is refused while frames are pending and above 12 lanes."""
    from jxg.dist import shared_gpu_lanes
    from jxg.synth import synth_rgb8_device

    assert shared_gpu_lanes(1) is None and shared_gpu_lanes(8) == 2 and shared_gpu_lanes(4) == 3
    w, h, world = 4096, 512, 2
    ts = [synth_rgb8_device(w, h, 0x4A60 + 7 * k) for k in range(7)]
    ref = streamed_shards(jxg_mod, ts, w, h, world)
    with jxg_mod.Encoder(flags=jxg_mod.FLAG_ANS) as enc:
        full = enc.pipeline_depth(w, h, 0, world)
        batch = (full - 1) // 11  # 12 lanes at the default 16 queues
        for cap in (1, 2, 3):
            enc.set_pipeline_lanes(cap)
            assert enc.pipeline_depth(w, h, 0, world) == (cap - 1) * batch + 1
        enc.set_pipeline_lanes(0)
        assert enc.pipeline_depth(w, h, 0, world) == full
        with pytest.raises(jxg_mod.JxgError, match="invalid"):
            enc.set_pipeline_lanes(13)
        enc.set_pipeline_lanes(2)
        enc.shard_submit_device(ts[0].data_ptr(), w, h, 0, world)
        with pytest.raises(jxg_mod.JxgError, match="invalid"):  # a frame is pending
            enc.set_pipeline_lanes(3)
        enc.shard_next_head()
    for cap in (1, 2):
        assert streamed_shards(jxg_mod, ts, w, h, world, lanes=cap) == ref


def test_stream_shards_refusals(jxg_mod):
    """No collective inside the streaming pipeline: a plan that needs the
    record exchange, or prefix codes over several ranks, is refused; a full
    pipeline refuses another frame; one-at-a-time calls wait for the
    pending frames."""
    import torch

    t = torch.zeros((2160, 3840, 3), dtype=torch.uint8, device="cuda")
    with jxg_mod.Encoder(flags=jxg_mod.FLAG_ANS) as enc:
        assert jxg_mod.shard_plan(3840, 2160, 8)[2] == 2
        with pytest.raises(jxg_mod.JxgError, match="unsupported"):
            enc.shard_submit_device(t.data_ptr(), 3840, 2160, 0, 8)
    with jxg_mod.Encoder() as enc:  # prefix codes: the histogram all-reduce
        with pytest.raises(jxg_mod.JxgError, match="unsupported"):
            enc.shard_submit_device(t.data_ptr(), 4096, 512, 0, 2)
    small = torch.zeros((512, 4096, 3), dtype=torch.uint8, device="cuda")
    with jxg_mod.Encoder(flags=jxg_mod.FLAG_ANS) as enc:
        depth = enc.pipeline_depth(4096, 512, 0, 2)
        for _ in range(depth):
            enc.shard_submit_device(small.data_ptr(), 4096, 512, 0, 2)
        with pytest.raises(jxg_mod.JxgError, match="invalid"):  # every lane holds a frame
            enc.shard_submit_device(small.data_ptr(), 4096, 512, 0, 2)
        with pytest.raises(jxg_mod.JxgError, match="invalid"):  # lanes busy
            enc.encode_device(small.data_ptr(), 4096, 512)
        with pytest.raises(jxg_mod.JxgError, match="invalid"):  # shard frames, not whole ones
            enc.receive()
        assert enc.pending() == depth
        enc.shard_next_head()
        assert enc.pending() == depth


def test_stream_pending_refuses_one_at_a_time(jxg_mod):
    """a context with streamed frames in flight is a pipeline lane;
    encode / encode_device / compare refuse until they are received."""
    from jxg.synth import synth_rgb8

    img = synth_rgb8(640, 480, 3)
    with jxg_mod.Encoder(flags=jxg_mod.FLAG_ANS) as enc:
        ref = enc.encode(img)
        enc.submit(img)
        enc.submit(img)
        for call in (lambda: enc.encode(img), lambda: enc.compare(img, img),
                     lambda: enc.encode_batch([img])):
            with pytest.raises(jxg_mod.JxgError, match="invalid"):
                call()
        assert enc.receive() == ref and enc.receive() == ref
        assert enc.encode(img) == ref  # drained: one-at-a-time again


def test_input_stream_ordering(jxg_mod):
    """jxg_set_input_stream: the library's reads of a device frame are ordered
    after the caller's stream, without a host synchronisation -- the frame is
    written by a long chain of torch kernels on a side stream right before
    the submit."""
    import torch

    from jxg.synth import synth_rgb8

    img = synth_rgb8(1024, 768, 9)
    side = torch.cuda.Stream()
    with jxg_mod.Encoder(flags=jxg_mod.FLAG_ANS) as enc:
        ref = enc.encode(img)
        enc.set_input_stream(side.cuda_stream)
        src = torch.from_numpy(img).cuda()
        torch.cuda.synchronize()
        outs = []
        for _ in range(3):
            dst = torch.zeros_like(src)
            side.wait_stream(torch.cuda.current_stream())  # dst's zero fill first
            with torch.cuda.stream(side):
                x = src.to(torch.float32)
                for _ in range(200):  # keep the side stream busy
                    x = x * 1.0
                dst.copy_(x.to(torch.uint8))
            enc.submit_device(dst.data_ptr(), 1024, 768)
            outs.append(dst)
        got = [enc.receive() for _ in range(3)]
        assert all(g == ref for g in got)
        dst2 = torch.zeros_like(src)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            x = src.to(torch.float32)
            for _ in range(200):
                x = x * 1.0
            dst2.copy_(x.to(torch.uint8))
        assert enc.encode_device(dst2.data_ptr(), 1024, 768) == ref


def test_sharded_8k_ans_over_8(jxg_mod, decoder):
    """BASELINE config 2 with the north-star coder: an 8K frame, ANS, over 8
    contexts (whole LF groups per rank, one HF preset per rank).  LfGlobal and
    every LF-group section equal the single-GPU encode's; the pass groups of
    the bottom group row (ranks 6 and 7, with all 8 presets in HfGlobal)
    decode to the single-GPU coefficients; each group selects its rank's
    preset; the streamed shards give the same bytes."""
    from jxg.synth import synth_rgb8_device

    w, h, world = 7680, 4320, 8
    t = synth_rgb8_device(w, h, 0x4A584C02)
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS | jxg_mod.FLAG_KEEP_MAPS) as enc:
        ref = enc.encode_device(t.data_ptr(), w, h)
        st = enc.stats()
    got = sharded_encode(jxg_mod, None, world, flags=jxg_mod.FLAG_ANS, t=t)
    go, lo, kind = jxg_mod.shard_plan(w, h, world)
    assert kind == 1
    nlf = len(lo)
    dr = decoder.decode(ref, groups=[])
    gxs = -(-w // 256)
    bottom = [16 * gxs + gx for gx in range(gxs)]
    dg = decoder.decode(got, groups=bottom)
    for i in range(1 + nlf):  # LfGlobal + LF groups: byte-identical sections
        a = ref[dr.section_offsets[i]:dr.section_offsets[i] + dr.section_sizes[i]]
        b = got[dg.section_offsets[i]:dg.section_offsets[i] + dg.section_sizes[i]]
        assert a == b, i
    assert dg.npresets == world
    assert [int(dg.group_presets[g]) for g in bottom] == [go[g] for g in bottom]
    rows = slice(16 * 32, dg.bys)
    assert np.array_equal(dg.ac[rows], st["ac"][rows])
    assert np.array_equal(dg.acs[rows], st["acs"][rows].astype(np.int32))
    assert np.array_equal(dg.ac_tokens[bottom], st["ac_tokens"][bottom])
    assert streamed_shards(jxg_mod, [t], w, h, world)[0] == got


def _sharded_ans_matches_single(jxg_mod, decoder, w, h, seed, world, p, flags, rows):
    """ANS over `world` contexts (one HF preset per rank) against the
    one-context encode: LfGlobal and every LF-group section byte-identical, the
    pass groups of block-group rows `rows` decoded to the single encode's
    coefficients, strategies and token counts, each group on its rank's preset"""
    from jxg.synth import synth_rgb8_device

    t = synth_rgb8_device(w, h, seed)
    keep = jxg_mod.FLAG_KEEP_MAPS
    with jxg_mod.Encoder(distance=1.0, effort=7, proposals=p, flags=flags | keep) as enc:
        ref = enc.encode_device(t.data_ptr(), w, h)
        st = enc.stats()
    got = sharded_encode(jxg_mod, None, world, p=p, flags=flags, t=t)
    del t
    go, lo, kind = jxg_mod.shard_plan(w, h, world)
    nlf = len(lo)
    dr = decoder.decode(ref, groups=[])
    gxs = -(-w // 256)
    sel = [gy * gxs + gx for gy in rows for gx in range(gxs)]
    dg = decoder.decode(got, groups=sel)
    assert (dg.gab, dg.epf_iters) == (dr.gab, dr.epf_iters)  # filters signalled alike
    for i in range(1 + nlf):  # LfGlobal + LF groups: byte-identical sections
        a = ref[dr.section_offsets[i]:dr.section_offsets[i] + dr.section_sizes[i]]
        b = got[dg.section_offsets[i]:dg.section_offsets[i] + dg.section_sizes[i]]
        assert a == b, i
    assert dg.npresets == world
    assert [int(dg.group_presets[g]) for g in sel] == [go[g] for g in sel]
    for gy in rows:
        r = slice(32 * gy, min(32 * gy + 32, dg.bys))
        assert np.array_equal(dg.ac[r], st["ac"][r])
        assert np.array_equal(dg.acs[r], st["acs"][r].astype(np.int32))
    assert np.array_equal(dg.ac_tokens[sel], st["ac_tokens"][sel])
    return kind


def test_sharded_8k_cjxl_over_8(jxg_mod, decoder):
    """config 2 at the headline preset (JXG_FLAGS_CJXL_DEFAULTS: Gaborish,
    EPF, masking AQ, ANS) over 8 contexts.  The inverse Gaborish and the AQ
    neighbourhood read across shard edges; every rank reads its halo from the
    whole frame, so the LF sections (quant field, strategies, DC) equal the
    single-GPU encode's and the decoded group rows at rank seams (block-group
    rows 7, 8, 16) hold the single-GPU coefficients."""
    kind = _sharded_ans_matches_single(jxg_mod, decoder, 7680, 4320, 0x4A584C02, 8, 0,
                                       jxg_mod.FLAGS_CJXL_DEFAULTS, [7, 8, 16])
    assert kind == 1


def test_sharded_16k_cjxl_pf_over_8(jxg_mod, decoder):
    """config 4 at the headline preset: 16384^2, P+F, cjxl defaults, over 8
    contexts (the single-context encode equals the oracle fingerprint
    16k_d1_cjxl_pf in test_gpu_configs).  LfGlobal and all 64 LF-group sections
    (DC, quant field, strategies, CfL: everything the AQ halo and the inverse
    Gaborish decide across rank seams) equal the single encode's byte for
    byte; the frame signals the same filters and one HF preset per rank."""
    from jxg.synth import synth_rgb8_device

    w = h = 16384
    t = synth_rgb8_device(w, h, 0x4A584C04)
    flags = jxg_mod.FLAGS_CJXL_DEFAULTS
    with jxg_mod.Encoder(distance=1.0, effort=7, proposals=3, flags=flags) as enc:
        ref = enc.encode_device(t.data_ptr(), w, h)
    got = sharded_encode(jxg_mod, None, 8, p=3, flags=flags, t=t)
    del t
    go, lo, kind = jxg_mod.shard_plan(w, h, 8)
    assert kind == 0 and len(lo) == 64
    dr = decoder.decode(ref, toc_only=True)
    dg = decoder.decode(got, toc_only=True)
    assert (dg.gab, dg.epf_iters) == (dr.gab, dr.epf_iters) == (True, 1)
    for i in range(1 + len(lo)):
        a = ref[dr.section_offsets[i]:dr.section_offsets[i] + dr.section_sizes[i]]
        b = got[dg.section_offsets[i]:dg.section_offsets[i] + dg.section_sizes[i]]
        assert a == b, i


def test_sharded_16k_pf_over_8(jxg_mod):
    """BASELINE config 4 as written: 16384^2, proposals P+F, over 8 contexts
    (LF-group rows aligned with the ranks: no record moves); prefix codes ->
    the codestream equals the oracle fingerprint of the whole frame."""
    import hashlib

    import json
    import os

    from jxg.synth import synth_rgb8_device

    g = {e["name"]: e for e in json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                                           "config_golden.json")))}["16k_d1_pf"]
    t = synth_rgb8_device(16384, 16384, g["seed"])
    assert jxg_mod.shard_plan(16384, 16384, 8)[2] == 0
    assert all(sum(jxg_mod.shard_exchange(16384, 16384, 8, r)[0]) == 0 for r in range(8))
    out = sharded_encode(jxg_mod, None, 8, p=3, t=t)
    assert len(out) == g["bytes"]
    assert hashlib.sha256(out).hexdigest() == g["sha256"]


def _gloo_stream_rank(rank, world, port, result, nframes):
    import os

    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import jxg
        from jxg.dist import SharedHostBuffer, ShardStream, encode_sharded
        from jxg.synth import synth_rgb8_device

        w, h = 4096, 512
        ts = [synth_rgb8_device(w, h, 0x77 + k) for k in range(nframes)]
        res = {}
        for ans in (False, True):
            flags = jxg.FLAG_ANS if ans else 0
            with jxg.Encoder(flags=flags) as enc:
                bufs = {}  # persistent exchange / payload buffers across frames
                dev = [encode_sharded(enc, t, w, h, rank, world, bufs=bufs) for t in ts]
                host = SharedHostBuffer(rank, world)
                hst = [encode_sharded(enc, t, w, h, rank, world, bufs=bufs, host=host) for t in ts]
                dist.barrier()
                host.close()
                ref = [enc.encode_device(t.data_ptr(), w, h) for t in ts] if rank == 0 else None
            res[ans] = (dev, hst, ref)
        streams = {}
        for name, slots, ahead in (("ShardStream", 6, False), ("ahead", 3, True)):
            # ahead: slots = 3 and frames submitted up to depth + slots - 2
            # before each receive, so submit writes frames out (the write lag
            # and the slot release between ranks on the path)
            with jxg.Encoder(flags=jxg.FLAG_ANS) as enc:
                ss = ShardStream(enc, w, h, rank, world, slots=slots, lanes=2 if ahead else None)
                got = []

                def take():  # a view is valid until the next receive: copy now
                    g = ss.receive()
                    got.append(None if g is None else g.tobytes())

                for t in ts:
                    if ahead:
                        if ss.pending() >= ss.max_ahead:
                            take()
                        ss.submit(t.data_ptr())
                        continue
                    ss.submit(t.data_ptr())
                    while ss.pending() >= ss.max_pending or (ss.pending() and ss.ready()):
                        take()
                if ahead:
                    assert ss.written > ss.received  # submit wrote ahead of receive
                while ss.pending():
                    take()
                ss.close()
            streams[name] = got
        if rank == 0:
            result.put((res, streams))
    finally:
        dist.destroy_process_group()


def test_multiprocess_streamed_frames(jxg_mod, decoder):
    """Two processes (gloo, both ranks on cuda:0) stream 12 frames: the
    one-frame-at-a-time sharded encode with persistent exchange / payload
    buffers, device and host assembly, both coders; and jxg.dist.ShardStream
    (the multi-GPU pipeline: no collective inside a frame, heads swapped in
    /dev/shm).  Prefix codes: every frame == the single-GPU bytes; ANS: the
    streamed bytes == the one-at-a-time sharded bytes, and the image == the
    single-GPU image."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    nframes = 12
    procs = [ctx.Process(target=_gloo_stream_rank, args=(r, 2, port, q, nframes))
             for r in range(2)]
    for p in procs:
        p.start()
    res, streams = q.get(timeout=280)
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    import hashlib

    def digests(xs):  # (a failing comparison of 12 MB byte lists takes pytest minutes to diff)
        return [hashlib.sha256(bytes(x)).hexdigest()[:16] for x in xs]

    dev, hst, ref = res[False]
    assert digests(dev) == digests(ref) and digests(hst) == digests(ref)
    dev, hst, ref = res[True]
    assert digests(dev) == digests(hst)
    assert digests(streams["ShardStream"]) == digests(dev)
    assert digests(streams["ahead"]) == digests(dev)
    got = streams["ShardStream"]
    dr, dg = decoder.decode(ref[3]), decoder.decode(got[3])
    assert dg.npresets == 2
    _same_image(dr, dg)
