"""The lane protocol of the rANS chain kernels (csrc/jxg_ac.hip ans_chain /
ans_chain2) restated over 64 model lanes and checked against a sequential
encoder on random record streams: the diagonal hand-over by a whole-wave
rotation, the pre-step state each lane captures, the final state of a stream
(lane 63 / 31 after a full batch, else the state the lane past the last record
captured) and, for two chains per wave, the swap of lanes 31 and 63 at a batch
boundary.  The step itself is a toy rANS (the kernels' arithmetic is checked
on the GPU against the oracle); what this pins is which lane holds which state
when, for every stream length class: empty, shorter than a batch, exactly a
batch, batch + 1, several batches, and an odd number of chains (an empty
partner half)."""
import random

import pytest

INIT = 0x130000


def step(x, rec):
    """toy rANS step: rec = (f, cum); emits the low 16 bits when x >= f << 20"""
    f, cum = rec
    out = None
    if x >= (f << 20):
        out = x & 0xFFFF
        x >>= 16
    return (x // f) * 4096 + cum + x % f, out


DUMMY = (4096, 0)  # the kernels' idle-lane record: never emits (x < 2^32)


def sequential(recs):
    """the chain as the format defines it: records n - 1 .. 0"""
    x, outs = INIT, [None] * len(recs)
    for i in range(len(recs) - 1, -1, -1):
        x, outs[i] = step(x, recs[i])
    return x, outs


def rotate(v):  # wave_ror:1 -- lane L receives lane L - 1 (lane 0 receives lane 63)
    return [v[(l - 1) % 64] for l in range(64)]


def emitted(X, rec):
    f, _ = rec
    return X & 0xFFFF if X >= (f << 20) else None


def single_chain(recs):
    """ans_chain: one stream on the 64-lane diagonal, batches of 64 from the end"""
    n = len(recs)
    x = [INIT] * 64
    outs = [None] * n
    final = INIT
    hi = n
    while hi > 0:
        cnt = min(64, hi)
        rec = [recs[hi - 1 - l] if l < cnt else DUMMY for l in range(64)]
        X = [0] * 64
        for s in range(cnt):  # the tail batch runs cnt steps only
            xin = rotate(x)
            X[s] = xin[s]
            x = [step(xin[l], rec[l])[0] for l in range(64)]
        for l in range(cnt):
            outs[hi - 1 - l] = emitted(X[l], rec[l])
        if hi <= 64:
            final = x[cnt - 1]
        hi -= cnt
    return final, outs


def paired_chain(ra, rb):
    """ans_chain2: stream A on lanes 0-31, stream B (None: no group) on 32-63"""
    streams = [ra, rb if rb is not None else []]
    x = [INIT] * 64
    outs = [[None] * len(s) for s in streams]
    finals = [INIT, INIT]
    hi = [len(streams[0]), len(streams[1])]
    while hi[0] > 0 or hi[1] > 0:
        c = [min(32, max(h, 0)) for h in hi]
        rec = []
        for lane in range(64):
            h, hl = lane >> 5, lane & 31
            rec.append(streams[h][hi[h] - 1 - hl] if hl < c[h] else DUMMY)
        X = [0] * 64
        for s in range(32):  # always 32 steps (both halves)
            xin = rotate(x)
            X[s], X[32 + s] = xin[s], xin[32 + s]
            x = [step(xin[l], rec[l])[0] for l in range(64)]
        for h in range(2):
            for hl in range(c[h]):
                outs[h][hi[h] - 1 - hl] = emitted(X[32 * h + hl], rec[32 * h + hl])
            if 0 < hi[h] <= 32:
                finals[h] = x[32 * h + 31] if c[h] == 32 else X[32 * h + c[h]]
        x[31], x[63] = x[63], x[31]  # the carry swap
        hi = [hi[0] - c[0], hi[1] - c[1]]
    return finals, outs


def rand_stream(rng, n):
    out = []
    for _ in range(n):
        f = rng.choice([1, 2, 7, 64, 300, 1500, 4000, 4096])
        out.append((f, rng.randrange(0, 4097 - f)))
    return out


LENGTHS = [0, 1, 5, 31, 32, 33, 63, 64, 65, 96, 127, 128, 129, 300]


@pytest.mark.parametrize("n", LENGTHS)
def test_single_chain_protocol(n):
    rng = random.Random(n)
    recs = rand_stream(rng, n)
    assert single_chain(recs) == sequential(recs)


def test_paired_chain_protocol():
    rng = random.Random(7)
    for na in LENGTHS:
        for nb in LENGTHS + [None]:
            ra = rand_stream(rng, na)
            rb = None if nb is None else rand_stream(rng, nb)
            (fa, fb), (oa, ob) = paired_chain(ra, rb)
            assert (fa, oa) == sequential(ra), (na, nb)
            if rb is not None:
                assert (fb, ob) == sequential(rb), (na, nb)
