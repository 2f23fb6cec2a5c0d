"""GPU group sharding on one device: `world` contexts play the
ranks, the collectives are done with torch ops (sum of the histograms; the
all_to_all of the per-block records by the jxg_shard_exchange splits), and the
assembled codestream must equal the single-context
encode byte for byte (one AC histogram -> one HF preset, so sharding does not
change a bit).  The multi-process RCCL version of the same exchange is
jxg.dist.encode_sharded (bench.py --gpus N)."""
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
    ng = len(dg.group_presets)
    assert list(dg.group_presets) == [min(r for r in range(world) if g < ng * (r + 1) // world)
                                      for g in range(ng)]
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
