"""The lane protocol of the rANS chain kernel (csrc/jxg_ac.hip ans_chain)
restated over 64 model lanes and checked against a sequential encoder on
random record streams: the diagonal hand-over by a whole-wave rotation, the
pre-step state each lane captures, and the final state of a stream (the lane
of the last record after its batch's last step).  The step itself is a toy
rANS (the kernel's arithmetic is checked on the GPU against the oracle); what
this pins is which lane holds which state when, for every stream length
class: empty, shorter than a batch, exactly a batch, batch + 1, several
batches.  (Round 5 also ran two chains per wave, lanes 0-31 / 32-63 with a
carry swap at the batch boundary: bit-exact on the GPU, but slower alone and
no faster pipelined, DESIGN.md §3.5, so it was removed.)"""
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
