"""CPU oracle encode -> independent test decoder read-back.

The decoder (oracle/jxl_decode.py) is written from the format's decoding side;
these tests pin that the encoder's bitstream layout (headers, TOC, entropy
codes, modular LF streams, AC token contexts) is self-consistent: every
integer the encoder decided (strategies, quant field, DC, AC, token counts) is
recovered exactly, and the decoded image has sane PSNR (formula of
benchmark-jpegxl/src/image_reader.rs:569-606).
"""
import numpy as np
import pytest

SIZES = [(1, 1), (8, 8), (9, 7), (64, 64), (100, 75), (256, 256), (257, 130), (300, 200)]


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("proposals", [0, 3])
def test_roundtrip_exact(oracle, decoder, w, h, proposals):
    from jxg.synth import synth_rgb8

    img = synth_rgb8(w, h, 1000 + w + h)
    r = oracle.encode(img, 1.0, 7, proposals)
    d = decoder.decode(r.bytes)
    assert (d.xsize, d.ysize) == (w, h)
    assert np.array_equal(d.acs, r.acs)
    assert np.array_equal(d.qf - 1, r.qf)
    assert np.array_equal(d.dc, r.dc)
    assert np.array_equal(d.ac, r.ac)
    assert np.array_equal(d.ac_tokens, r.ac_tokens)
    assert d.rgb.shape == (h, w, 3)


@pytest.mark.parametrize("d_,effort", [(0.5, 7), (1.0, 3), (2.0, 5), (8.0, 7), (25.0, 7)])
def test_distance_sweep(oracle, decoder, d_, effort):
    from jxg.synth import synth_rgb8

    img = synth_rgb8(192, 128, 77)
    r = oracle.encode(img, d_, effort, 0)
    d = decoder.decode(r.bytes)
    assert np.array_equal(d.ac, r.ac)
    if effort < 5:
        assert (r.acs == 0).all()   # DCT8 only below effort 5 (no hooks)


def test_quality_smooth_image(oracle, decoder):
    # a smooth gradient image must come back at high PSNR at d1
    yy, xx = np.mgrid[0:128, 0:192]
    img = np.stack([(xx * 255 // 191), (yy * 255 // 127), ((xx + yy) * 255 // 318)], -1).astype(np.uint8)
    r = oracle.encode(img, 1.0, 7, 0)
    d = decoder.decode(r.bytes)
    mse, psnr = decoder.mse_psnr(img, d.rgb)
    assert psnr > 40.0, psnr


def test_rate_monotone_in_distance(oracle):
    from jxg.synth import synth_rgb8

    img = synth_rgb8(256, 192, 5)
    sizes = [len(oracle.encode(img, d, 7, 0).bytes) for d in (0.5, 1.0, 2.0, 4.0, 8.0)]
    assert sizes == sorted(sizes, reverse=True)


def test_proposals_change_strategies(oracle):
    from jxg.synth import synth_rgb8

    img = synth_rgb8(256, 256, 9)
    base = oracle.encode(img, 1.0, 7, 0)
    p = oracle.encode(img, 1.0, 7, 1)
    # hook P only rewrites blocks the baseline left at DCT8
    changed = base.acs != p.acs
    assert changed.any()
    assert (base.acs[changed] == 0).all()
    assert set(np.unique(p.acs[changed])) <= {3, 12, 13}


def test_invalid_params(oracle):
    img = np.zeros((8, 8, 3), np.uint8)
    with pytest.raises(RuntimeError):
        oracle.encode(img, 0.0, 7, 0)
    with pytest.raises(RuntimeError):
        oracle.encode(img, 30.0, 7, 0)
