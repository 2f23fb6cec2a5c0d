"""Restoration filters (cjxl --gaborish / --epf): the oracle
encoder's inverse Gaborish and EPF signalling against the oracle decoder's
Gaborish and edge-preserving filter (oracle/xyb.c jxo_gab_inverse,
jxo_lf_code; oracle/jxl_decode.py gaborish / epf).  [ext] libjxl's filters are
restated from the format; their parity with libjxl/djxl is unpinned (no codec
here), so these tests pin the encoder/decoder pair's own properties."""
import numpy as np
import pytest

from jxg.synth import natural_rgb8, synth_rgb8

GAB, EPF = 1, 2


def _psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 10 * np.log10(255.0 ** 2 / mse)


@pytest.mark.parametrize("filters", [0, GAB, EPF, GAB | EPF])
@pytest.mark.parametrize("d,iters", [(0.5, 0), (0.7, 1), (1.0, 1), (2.0, 2), (6.0, 3)])
def test_header_round_trip(oracle, decoder, filters, d, iters):
    """EPF iterations by distance (libjxl's 0.7 / 1.5 / 4.0 thresholds as
    recalled): none below d 0.7 -- the sharpness channel is then
    not signalled either."""
    img = synth_rgb8(72, 40, 11)
    r = oracle.encode(img, d, 7, 0, 0, filters)
    dec = decoder.decode(r.bytes)
    assert dec.gab == bool(filters & GAB)
    epf = iters if filters & EPF else 0
    assert dec.epf_iters == epf
    assert np.array_equal(dec.ac, r.ac) and np.array_equal(dec.acs, r.acs)
    # the EPF sharpness channel: a constant 4 through the leaf offset
    assert (dec.sharpness == (4 if epf else 0)).all()


def test_epf_signalling_only_changes_header_and_tree(oracle):
    """EPF is decoder-side: same coefficients, a few bytes of header and tree."""
    img = natural_rgb8(300, 200, 5)
    a = oracle.encode(img, 2.0, 7, 0, 1, 0)
    b = oracle.encode(img, 2.0, 7, 0, 1, EPF)
    assert np.array_equal(a.ac, b.ac) and np.array_equal(a.acs, b.acs)
    assert np.array_equal(a.dc, b.dc) and np.array_equal(a.qf, b.qf)
    assert 0 < len(b.bytes) - len(a.bytes) <= 8


def test_epf_inverse_sigma_known_answer(decoder):
    """sigma = quant_mul * sharp_lut[s] / (G/65536 * qf * kInvSigmaNum)."""
    class D:
        pass
    d = D()
    d.global_scale = 809
    d.qf = np.array([[64, 200]], dtype=np.int32)
    d.sharpness = np.array([[4, 0]], dtype=np.int32)
    inv = decoder.epf_inv_sigma(d)
    sigma = 0.46 * (4 / 7) / (809 / 65536 * 64 * -1.1715728752538099)
    assert inv[0, 0] == pytest.approx(1.0 / sigma, rel=1e-12)
    assert inv[0, 1] == pytest.approx(-1e4)  # sharpness 0: not filtered
    assert inv[0, 1] < decoder.EPF_MIN_SIGMA


def test_epf_keeps_flat_and_unfiltered_blocks(decoder):
    """A flat image is a fixed point of every EPF pass; blocks under the
    sigma threshold keep their input exactly."""
    class D:
        pass
    d = D()
    d.global_scale, d.epf_iters = 809, 3
    d.qf = np.full((3, 4), 40, dtype=np.int32)
    d.sharpness = np.full((3, 4), 7, dtype=np.int32)
    d.sharpness[1, 2] = 0
    flat = [np.full((24, 32), v) for v in (0.01, 0.4, 0.35)]
    out = decoder.epf(*flat, d)
    for o, f in zip(out, flat):
        assert np.allclose(o, f, rtol=0, atol=1e-12)
    rng = np.random.default_rng(3)
    noisy = [f + rng.normal(0, 0.02, f.shape) for f in flat]
    out = decoder.epf(*noisy, d)
    for o, n in zip(out, noisy):
        assert np.array_equal(o[8:16, 16:24], n[8:16, 16:24])  # the sharpness-0 block
        assert not np.array_equal(o[:8, :8], n[:8, :8])


def test_gaborish_pair_is_near_identity(oracle, decoder):
    """Encoder inverse Gaborish + decoder Gaborish ~ identity: at a small
    distance the round trip's PSNR with both filters stays within 1.5 dB of the
    unfiltered one (the 3x3 inverse leaves 5.8 % rms of the spectrum)."""
    img = natural_rgb8(256, 192, 9)
    p0 = _psnr(img, decoder.decode(oracle.encode(img, 0.3, 7, 0, 1, 0).bytes).rgb)
    p1 = _psnr(img, decoder.decode(oracle.encode(img, 0.3, 7, 0, 1, GAB).bytes).rgb)
    assert p1 > p0 - 1.5


def test_gaborish_rd_on_natural_content(oracle, decoder):
    """Natural content: with Gaborish at d1.25 the rate is within 2 % of the
    unfiltered d1.0 rate and the PSNR is not lower."""
    img = natural_rgb8(512, 384, 3)
    a = oracle.encode(img, 1.0, 7, 0, 1, 0)
    b = oracle.encode(img, 1.25, 7, 0, 1, GAB)
    pa = _psnr(img, decoder.decode(a.bytes).rgb)
    pb = _psnr(img, decoder.decode(b.bytes).rgb)
    assert abs(len(b.bytes) / len(a.bytes) - 1) < 0.02
    assert pb >= pa


def test_epf_raises_psnr_at_d2(oracle, decoder):
    img = natural_rgb8(384, 256, 4)
    a = oracle.encode(img, 2.0, 7, 0, 1, 0)
    b = oracle.encode(img, 2.0, 7, 0, 1, EPF)
    pa = _psnr(img, decoder.decode(a.bytes).rgb)
    pb = _psnr(img, decoder.decode(b.bytes).rgb)
    assert pb > pa + 0.1


def test_bad_filters_refused(oracle):
    with pytest.raises(RuntimeError):
        oracle.encode(synth_rgb8(16, 16, 1), 1.0, 7, 0, 0, 8)  # (bit 2 is JXO_OPT_AQ_MASKING)
