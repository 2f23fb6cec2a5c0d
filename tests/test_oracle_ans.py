"""CPU oracle: ANS coding of the AC stream (oracle/ans.c) read back by the
independent test decoder (oracle/jxl_decode.py: histogram parser, alias
table, rANS reader with the 0x130000 final-state check).  [ext] spec
restatement -- parity unpinned against libjxl."""
import numpy as np
import pytest

CASES = [(1, 1, 1.0, 7, 0), (64, 64, 1.0, 7, 0), (300, 200, 1.0, 7, 3), (520, 300, 2.0, 5, 0),
         (1000, 700, 0.5, 7, 2), (640, 480, 25.0, 4, 0), (9, 7, 3.0, 7, 3)]


@pytest.mark.parametrize("w,h,d,e,p", CASES)
def test_ans_roundtrip(oracle, decoder, w, h, d, e, p):
    from jxg.synth import synth_rgb8

    img = synth_rgb8(w, h, w * 5 + h)
    r0 = oracle.encode(img, d, e, p, 0)
    r1 = oracle.encode(img, d, e, p, 1)
    dec = decoder.decode(r1.bytes)
    assert np.array_equal(r1.ac, r0.ac) and np.array_equal(r1.dc, r0.dc)
    assert np.array_equal(dec.ac, r1.ac)
    assert np.array_equal(dec.dc, r1.dc)
    assert np.array_equal(dec.acs, r1.acs)
    assert np.array_equal(dec.ac_tokens, r1.ac_tokens)
    assert np.array_equal(dec.rgb, decoder.decode(r0.bytes).rgb)
    if w * h >= 64 * 64:
        assert len(r1.bytes) <= len(r0.bytes)


def test_ans_tiny_histograms(oracle, decoder):
    """flat images: one- and two-symbol histograms (simple forms)"""
    for v in (0, 128, 255):
        img = np.full((40, 72, 3), v, dtype=np.uint8)
        r = oracle.encode(img, 1.0, 7, 0, 1)
        dec = decoder.decode(r.bytes)
        assert np.array_equal(dec.ac, r.ac)
