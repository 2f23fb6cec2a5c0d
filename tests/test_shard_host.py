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


@pytest.mark.parametrize("w,h,world", [(7680, 4320, 2), (7680, 4320, 8), (16384, 16384, 8),
                                       (3840, 2160, 4), (2100, 600, 8), (4100, 5000, 3)])
def test_record_exchange_plan(jxg_mod, w, h, world):
    """jxg_shard_exchange (C++) against the Python mirror of the LF ownership:
    a rank sends each of its pass groups' records to the owner of the group's
    LF group (if another rank), receives the other ranks' groups inside its
    own LF groups; sends and receives pair up across ranks."""
    rec = 1024 * 2 + 1024 * 4 * 3 + 32  # acs, qf, DC, and the 16 colour tiles ytox / ytob
    owners = jxg_mod.lf_owners(w, h, world)
    gxs, gys = -(-w // 256), -(-h // 256)
    lfxs = -(-w // 2048)
    ng = gxs * gys
    plan = [jxg_mod.shard_exchange(w, h, world, r) for r in range(world)]
    for r in range(world):
        snd, rcv = plan[r]
        for p in range(world):
            want = sum(1 for g in range(ng * r // world, ng * (r + 1) // world)
                       if p != r and owners[(g // gxs) // 8 * lfxs + (g % gxs) // 8] == p)
            assert snd[p] == want * rec
            assert rcv[p] == plan[p][0][r]  # what p sends to r
    # every LF group has an owner that holds part of it; owners spread out
    assert all(0 <= o < world for o in owners)
    _, cap = jxg_mod.shard_sizes(w, h, world)
    assert all(max(sum(s), sum(rv)) <= cap for s, rv in plan)
    if (w, h, world) == (16384, 16384, 8):
        assert all(sum(s) == 0 for s, _ in plan)  # LF groups aligned with the ranks
    if (w, h, world) == (7680, 4320, 8):
        total = sum(sum(s) for s, _ in plan)
        assert total < 7680 * 4320 // 64 * 14  # well under an all-gather's worth
