"""GPU parity of the libjxl-shaped masking quant field (JXG_FLAG_AQ_MASKING,
csrc/jxg_aq.hip) with the oracle (oracle/aq.c, JXO_OPT_AQ_MASKING): quant
field, strategies, coefficients, DC and bytes at tile / frame edges, every
distance regime (below / in / past the erosion and dampening ramps), both
coders, hooks P/F, with the restoration filters (the field is computed on the
XYB image before the inverse Gaborish), streamed and sharded."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

AQ_OPT = 4  # oracle filters-mask bit
GAB, EPF = 1, 2

CASES = [
    # (w, h, distance, effort, proposals, oracle filters, ans)
    (64, 64, 1.0, 7, 0, 0, False),
    (1, 1, 1.0, 7, 0, 0, True),
    (9, 7, 0.5, 7, 3, 0, False),
    (200, 136, 1.0, 7, 3, 0, True),
    (517, 389, 2.5, 7, 0, 0, True),
    (300, 200, 14.0, 5, 1, 0, False),
    (777, 333, 1.0, 7, 2, GAB | EPF, True),
    (130, 1100, 3.0, 4, 0, 0, False),
    (1920, 1080, 1.0, 7, 0, 0, True),
]


@pytest.mark.parametrize("w,h,d,e,p,filters,ans", CASES)
def test_masking_aq_matches_oracle(jxg_mod, oracle, w, h, d, e, p, filters, ans):
    from jxg.synth import natural_rgb8, synth_rgb8

    img = (natural_rgb8 if w * h > 100000 else synth_rgb8)(w, h, w * 7 + h)
    flags = (jxg_mod.FLAG_AQ_MASKING | jxg_mod.FLAG_KEEP_MAPS |
             (jxg_mod.FLAG_ANS if ans else 0) |
             (jxg_mod.FLAG_GABORISH if filters & GAB else 0) |
             (jxg_mod.FLAG_EPF if filters & EPF else 0))
    with jxg_mod.Encoder(distance=d, effort=e, proposals=p, flags=flags) as enc:
        got = enc.encode(img)
        st = enc.stats()
    ref = oracle.encode(img, d, e, p, 1 if ans else 0, filters | AQ_OPT)
    assert np.array_equal(st["qf"], ref.qf)
    assert np.array_equal(st["acs"], ref.acs)
    assert np.array_equal(st["dc"], ref.dc)
    assert np.array_equal(st["ac"], ref.ac)
    assert got == ref.bytes


def test_masking_aq_stream_and_shards(jxg_mod, oracle):
    """The field through the streaming pipeline (mixed sizes) and a 2-rank
    shard plan (each rank computes its own tiles' field from the whole
    frame's pixels): the one-at-a-time bytes / the single-GPU image."""
    import torch

    from jxg.synth import natural_rgb8

    frames = [natural_rgb8(1024, 768, 1), natural_rgb8(640, 480, 2), natural_rgb8(1920, 1080, 3)]
    flags = jxg_mod.FLAG_AQ_MASKING | jxg_mod.FLAG_ANS
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=flags) as enc:
        want = [enc.encode(f) for f in frames]
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=flags) as enc:
        for f in frames:
            enc.submit(f)
        got = [enc.receive() for _ in frames]
    assert got == want
    # prefix codes over 3 ranks (the record exchange: 777 x 333 is a kind-2
    # plan), each rank computing its own tiles' field from the whole frame:
    # byte-identical to the single-GPU encode and the oracle
    from test_gpu_shard import sharded_encode

    img = natural_rgb8(777, 333, 5)
    pflags = jxg_mod.FLAG_AQ_MASKING
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=pflags) as enc:
        single = enc.encode(img)
    assert sharded_encode(jxg_mod, img, 3, flags=pflags) == single
    assert oracle.encode(img, 1.0, 7, 0, 0, AQ_OPT).bytes == single
