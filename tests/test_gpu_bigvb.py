"""GPU == oracle for the merge levels 128 / 256 px (effort >= 8: DCT128X128 /
128X64 / 64X128 / 256X256 / 256X128 / 128X256, raw ids 21-26;
csrc/jxg_bigvb.hip, oracle/merge.c jxo_merge_big): codestream bytes, the
AC-strategy map and the coefficients, on smooth frames where the big shapes
are chosen and on frames where they are not, with partial groups, both
coders, the thesis hooks, cjxl's defaults, the batched stream and shards."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BIG = [21, 22, 23, 24, 25, 26]


def gradient_rgb8(w, h, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.stack([128 + 60 * np.sin(x / rng.uniform(150, 400) + y / rng.uniform(150, 400) + c)
                    for c in range(3)], -1)
    return np.clip(img, 0, 255).astype(np.uint8)


CASES = [
    # w, h, distance, proposals, coder (0 prefix, 1 ANS), oracle filters mask
    (512, 512, 1.0, 0, 1, 0),
    (768, 520, 2.0, 0, 0, 0),
    (1024, 1024, 1.0, 3, 1, 0),
    (600, 300, 1.0, 2, 1, 7),
    (520, 776, 3.0, 1, 1, 7),
]


@pytest.mark.parametrize("w,h,d,p,coder,filt", CASES)
def test_effort8_matches_oracle(jxg_mod, oracle, w, h, d, p, coder, filt):
    img = gradient_rgb8(w, h, w * 7 + h)
    flags = jxg_mod.FLAG_KEEP_MAPS | (jxg_mod.FLAG_ANS if coder else 0)
    if filt:
        flags |= jxg_mod.FLAGS_CJXL_DEFAULTS
    ref = oracle.encode(img, d, 8, p, coder, filt)
    with jxg_mod.Encoder(distance=d, effort=8, proposals=p, flags=flags) as enc:
        got = enc.encode(img)
        st = enc.stats()
    assert np.array_equal(st["acs"], ref.acs), "AC strategy map differs"
    assert np.array_equal(st["qf"], ref.qf)
    assert np.array_equal(st["dc"], ref.dc)
    assert np.array_equal(st["ac"], ref.ac)
    assert got == ref.bytes


def test_big_shapes_are_exercised(jxg_mod, oracle):
    """the cases above choose every big shape somewhere (else the parity
    check above would not cover them)"""
    seen = set()
    for w, h, d, p, coder, filt in CASES:
        r = oracle.encode(gradient_rgb8(w, h, w * 7 + h), d, 8, p, coder, filt)
        seen |= set(int(t) for t in np.unique(r.acs[(r.acs & 0x80) == 0]))
    assert set(BIG) <= seen, sorted(seen)


def test_effort8_natural_and_noise(jxg_mod, oracle):
    """content where the big levels mostly keep the 64x64 decisions"""
    from jxg.synth import natural_rgb8, synth_rgb8

    for img in (natural_rgb8(777, 555, 4), synth_rgb8(640, 512, 0x4A584C05)):
        ref = oracle.encode(img, 1.0, 8, 0, 1)
        with jxg_mod.Encoder(distance=1.0, effort=8, flags=jxg_mod.FLAG_ANS) as enc:
            assert enc.encode(img) == ref.bytes


def test_effort8_batch_stream(jxg_mod, oracle):
    """1080p frames at effort 8 through the batched streaming pipeline (four
    frames per launch) == the oracle frame by frame"""
    frames = [gradient_rgb8(1920, 1080, s) for s in (1, 2, 3, 4, 5)]
    with jxg_mod.Encoder(distance=1.0, effort=8, flags=jxg_mod.FLAG_ANS) as enc:
        outs = enc.encode_batch(frames)
    for f, o in zip(frames, outs):
        assert o == oracle.encode(f, 1.0, 8, 0, 1).bytes


def test_effort8_sharded_matches_single(jxg_mod):
    """contexts sharding one frame at effort 8 (prefix codes: the same bytes
    as the one-context encode; the big varblocks stay inside pass groups, so
    inside a rank's shard)"""
    from test_gpu_shard import sharded_encode

    img = gradient_rgb8(1024, 768, 11)
    with jxg_mod.Encoder(distance=1.0, effort=8) as enc:
        single = enc.encode(img)
    for world in (2, 3):
        assert sharded_encode(jxg_mod, img, world, 1.0, 8, 0) == single


def chroma_checker_rgb8(w, h):
    """red / blue one-pixel checkerboard: at d1 e8 a 256x256 group becomes one
    DCT256X256 whose X and B carry little but their last coefficient, so ~129 K
    zero tokens land in one (cluster, token) bin of the group"""
    y, x = np.mgrid[0:h, 0:w]
    m = ((x + y) % 2).astype(bool)[..., None]
    return np.where(m, np.array([255, 0, 0]), np.array([0, 60, 255])).astype(np.uint8)


@pytest.mark.parametrize("coder", [0, 1])
def test_whole_group_histogram_bin_above_u16(jxg_mod, oracle, coder):
    """the whole-group ac_hist_kernel (BR = 32, effort >= 8) counted
    in u16 LDS halves; a bin past 65535 carried into its neighbour.  The oracle
    shows this frame's largest per-group bin above 65535, and the GPU bytes
    (histogram -> codes) equal the oracle's."""
    img = chroma_checker_rgb8(512, 256)
    ref, mx = oracle.max_group_bin(img, 1.0, 8, 0, coder)
    assert mx > 65535, mx
    flags = jxg_mod.FLAG_ANS if coder else 0
    with jxg_mod.Encoder(distance=1.0, effort=8, flags=flags) as enc:
        assert enc.encode(img) == ref.bytes


def test_effort8_sharded_ans_decodes_to_single(jxg_mod, decoder):
    """ANS sharded at effort 8 (one HF preset per rank; the big kinds' quant
    tables of every rank's groups in HfGlobal): decodes to the single-context
    image, with the same explicit tables"""
    from test_gpu_shard import sharded_encode

    img = gradient_rgb8(1024, 768, 11)
    with jxg_mod.Encoder(distance=1.0, effort=8, flags=jxg_mod.FLAG_ANS) as enc:
        single = decoder.decode(enc.encode(img))
    assert single.qm_params
    for world in (2, 3):
        got = decoder.decode(sharded_encode(jxg_mod, img, world, 1.0, 8, 0, jxg_mod.FLAG_ANS))
        assert sorted(got.qm_params) == sorted(single.qm_params)
        assert np.array_equal(got.rgb, single.rgb)
