"""libjxl-shaped adaptive quantization (SURVEY §8(a) row "adaptive
quantization"): the oracle's masking quant field
(oracle/aq.c, JXO_OPT_AQ_MASKING = filters bit 2) against its own stated
behaviour.  [ext] libjxl's InitialQuantField is restated as recalled; parity
with libjxl is unpinned (no libjxl here), so these tests pin the restatement's
properties: a well-formed field, coarser quantization on masked (textured)
content than on flat content, exact decodability, and the field's known
answers on constant images."""
import numpy as np
import pytest

from jxg.synth import natural_rgb8, synth_rgb8

AQ = 4


def _psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 10 * np.log10(255.0 ** 2 / mse)


@pytest.mark.parametrize("w,h,d", [(1, 1, 1.0), (9, 7, 1.0), (200, 136, 0.5), (300, 200, 3.0),
                                   (517, 389, 8.0)])
def test_masking_field_round_trip(oracle, decoder, w, h, d):
    img = (natural_rgb8 if w * h > 1000 else synth_rgb8)(w, h, 3 * w + h)
    r = oracle.encode(img, d, 7, 0, 1, AQ)
    dec = decoder.decode(r.bytes)
    assert np.array_equal(dec.ac, r.ac) and np.array_equal(dec.acs, r.acs)
    assert np.array_equal(dec.qf, r.qf.astype(np.int32) + 1)  # (the decoder holds raw, the encoder raw - 1)
    assert r.qf.min() >= 0 and r.qf.max() <= 255


def test_flat_image_uniform_field(oracle):
    """A constant image: every block sees the same eroded value (no
    differences), no HF energy and the same gamma ratio, so the field is one
    value everywhere."""
    img = np.full((128, 192, 3), 117, dtype=np.uint8)
    r = oracle.encode(img, 1.0, 7, 0, 1, AQ)
    assert len(np.unique(r.qf)) == 1


def test_texture_is_quantized_coarser(oracle):
    """Masking: a noisy half gets a coarser (smaller) quant field than a flat
    half of the same mean."""
    rng = np.random.default_rng(7)
    img = np.full((256, 256, 3), 128, dtype=np.uint8)
    img[:, 128:] = np.clip(128 + rng.normal(0, 40, (256, 128, 3)), 0, 255).astype(np.uint8)
    r = oracle.encode(img, 1.0, 7, 0, 1, AQ)
    flat, noisy = r.qf[:, :12], r.qf[:, 20:]
    assert flat.mean() > noisy.mean() * 1.3


def test_distance_scales_the_field(oracle):
    """The raw field is qf x 65536 / G with qf ~ 0.79 / d and G ~ 809 / d: at
    d <= 2 (no dampening) it hardly moves with the distance; far above d 2
    the modulation is damped toward 0.48 x qf_base."""
    img = natural_rgb8(256, 192, 4)
    q1 = oracle.encode(img, 1.0, 7, 0, 1, AQ).qf.astype(np.float64)
    q15 = oracle.encode(img, 1.5, 7, 0, 1, AQ).qf.astype(np.float64)
    q14 = oracle.encode(img, 14.0, 7, 0, 1, AQ).qf
    assert abs(q1.mean() - q15.mean()) < 0.15 * q1.mean()
    assert q14.std() < 1.0  # fully damped: a constant field


def test_masking_changes_only_the_field_and_decisions(oracle, decoder):
    """Same pixels, same coder: the option changes the quant field (and with
    it the strategy decisions and coefficients), not the headers' structure;
    both decode."""
    img = natural_rgb8(320, 240, 9)
    a = oracle.encode(img, 1.0, 7, 0, 1, 0)
    b = oracle.encode(img, 1.0, 7, 0, 1, AQ)
    assert not np.array_equal(a.qf, b.qf)
    for r in (a, b):
        dec = decoder.decode(r.bytes)
        assert _psnr(img, dec.rgb) > 30
