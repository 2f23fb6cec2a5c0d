"""Known-answer tests pinning the oracle's thesis selector to the text of
/root/reference/proposals/combined.diff (the patch itself cannot be compiled
here: it needs libjxl's ACSConfig/AcStrategy headers, and stand-ins are not
allowed -- DESIGN.md §2).

Every expected value below is derived by hand from the diff, on images whose
arithmetic is exact in float32 (small integers), so the derivation is in the
comments and the numbers are literals, not a second implementation.

Facts from the diff used throughout:
* Laplacian mask {{0,-1,0},{-1,-4,-1},{0,-1,0}} (:63) has no positive tap, so
  for Y >= 0 every Laplacian value is <= 0 and no zero crossing is counted
  (threshold > 0, :163-168): the crossing term is 0 for real XYB images.
* SML (:83-105) = sum |2p-l-r| + |2p-u-d| over the region.
* Colorfulness (:107-151) is 0 when X = B = 0.
* d1 = H(tl) + H(br)/2 and d2 = H(bl) + H(tr)/2 (operator precedence :200-203).
* Partition (:213-235): r_d > T -> DCT4X4(3); r_h > r_v && r_h > T -> DCT8X4(13);
  r_v > r_h && r_v > T -> DCT4X8(12); else DCT(0); T = 1.5 for d <= 3.
"""
import math

import numpy as np
import pytest

F32 = np.float32


def _frame(Y, X=None, B=None):
    Y = np.asarray(Y, dtype=np.float32)
    X = np.zeros_like(Y) if X is None else np.asarray(X, np.float32)
    B = np.zeros_like(Y) if B is None else np.asarray(B, np.float32)
    return np.stack([X, Y, B])


def _stripes(h, w, amp_rows):
    """vertical stripes: column x even -> amp(row), odd -> 0"""
    Y = np.zeros((h, w), np.float32)
    for y in range(h):
        Y[y, 0::2] = amp_rows(y)
    return Y


def test_zero_image_is_nan_and_dct(oracle):
    r3, t = oracle.homog_map(np.zeros((3, 24, 24), np.float32), 1.0)
    assert np.isnan(r3).all()          # 0/0 (:209-211)
    assert (t == 0).all()              # NaN compares false -> DCT


def test_top_textured_bottom_flat_gives_dct4x4(oracle):
    # 24x24, stripes (amplitude 1) in rows 0..11, zero below; centre block
    # (8..15, 8..15).  Per pixel SML: rows 8-10: 2; row 11: 2 + [col even];
    # row 12: [col even]; rows 13-15: 0.
    # tl = tr = 3*4*2 + (3+2+3+2) = 34, bl = br = 2 -> h1 = 68, h2 = 4,
    # v1 = v2 = 36, d1 = 34 + 2/2 = 35, d2 = 2 + 34/2 = 19.
    Y = _stripes(24, 24, lambda y: 1.0 if y < 12 else 0.0)
    img = _frame(Y)
    H = {(xs, ys, bx, by): oracle.homogeneity(img, 8, 8, xs, ys, bx, by, 1.0)
         for (xs, ys, bx, by) in [(8, 4, 0, 0), (8, 4, 0, 4), (4, 8, 0, 0), (4, 8, 4, 0),
                                  (4, 4, 0, 0), (4, 4, 4, 4), (4, 4, 0, 4), (4, 4, 4, 0)]}
    assert H[(8, 4, 0, 0)] == 68.0 and H[(8, 4, 0, 4)] == 4.0
    assert H[(4, 8, 0, 0)] == 36.0 and H[(4, 8, 4, 0)] == 36.0
    assert H[(4, 4, 0, 0)] == 34.0 and H[(4, 4, 4, 4)] == 2.0
    assert H[(4, 4, 0, 4)] == 2.0 and H[(4, 4, 4, 0)] == 34.0
    r3, t = oracle.homog_map(img, 1.0)
    assert r3[1, 1, 0] == F32(17.0)
    assert r3[1, 1, 1] == F32(1.0)
    assert r3[1, 1, 2] == F32(35.0) / F32(19.0)   # 1.842 > 1.8 at every distance
    for d in (1.0, 5.0, 12.0):
        _, t = oracle.homog_map(img, d)
        assert t[1, 1] == 3                        # DCT4X4 (precedence quirk)


def test_left_textured_right_flat_gives_dct4x8(oracle):
    # transpose of the case above: r_v = 17, r_h = 1, d1 = 34 + 2/2 = 35 =
    # d2 = 34 + 2/2 -> r_d = 1 -> r_v > r_h && r_v > T -> DCT4X8 (12)
    Y = _stripes(24, 24, lambda y: 1.0 if y < 12 else 0.0).T.copy()
    r3, t = oracle.homog_map(_frame(Y), 1.0)
    assert r3[1, 1, 0] == F32(1.0)
    assert r3[1, 1, 1] == F32(17.0)
    assert r3[1, 1, 2] == F32(1.0)
    assert t[1, 1] == 12


def test_graded_top_bottom_gives_dct8x4(oracle):
    # stripes of amplitude 3 in rows 0..11 and 1 below.  Horizontal term
    # 2*amp everywhere; vertical term 2 at rows 11 and 12 in even columns.
    # tl = tr = 16*6 + 2*2 = 100, bl = br = 16*2 + 2*2 = 36
    # r_h = 200/72, r_v = 136/136 = 1, r_d = (100+18)/(36+50) = 118/86 < 1.5
    Y = _stripes(24, 24, lambda y: 3.0 if y < 12 else 1.0)
    r3, t = oracle.homog_map(_frame(Y), 1.0)
    assert r3[1, 1, 0] == F32(200.0) / F32(72.0)
    assert r3[1, 1, 1] == F32(1.0)
    assert r3[1, 1, 2] == F32(118.0) / F32(86.0)
    assert t[1, 1] == 13
    _, t12 = oracle.homog_map(_frame(Y), 12.0)     # T = 1.8 < 2.78: still 8X4
    assert t12[1, 1] == 13


def test_colorfulness_double_sqrt(oracle):
    # Y = 0, X = 0.5, B = 0.25: SML = 0, crossings = 0, var = 0,
    # colorfulness = (float)(sqrt(0) + 0.3 * sqrt((double)(0.25f + 0.0625f)))
    img = _frame(np.zeros((16, 16)), np.full((16, 16), 0.5), np.full((16, 16), 0.25))
    h = oracle.homogeneity(img, 0, 0, 8, 4, 0, 0, 1.0)
    assert h == F32(0.3 * math.sqrt(0.3125))
    r3, t = oracle.homog_map(img, 1.0)
    assert (r3 == 1.0).all() and (t == 0).all()


def test_h1_int_abs_variant(oracle):
    # stripes of amplitude 0.25 on top: every SML term is 0.5 with the float
    # overload and int(0.5) = 0 with int abs(int): the int variant sees a
    # flat block (all H = 0 -> NaN -> DCT), the float variant a top/bottom
    # split (-> DCT4X4)
    Y = _stripes(24, 24, lambda y: 0.25 if y < 12 else 0.0)
    _, t_float = oracle.homog_map(_frame(Y), 1.0, 0)
    r_int, t_int = oracle.homog_map(_frame(Y), 1.0, 1)
    assert t_float[1, 1] == 3
    assert np.isnan(r_int[1, 1]).all() and t_int[1, 1] == 0


def test_bottom_row_sml_skip(oracle):
    # combined.diff:91 skips samples with y+1 >= ysize: on an 8-row frame the
    # last row never contributes.  Stripes everywhere: rows 0..6 give 2 per
    # pixel (vertical terms vanish inside the stripes; row 0 reads row -1 as
    # 0: + [col even]), row 7 gives 0.
    Y = _stripes(8, 16, lambda y: 1.0)
    img = _frame(Y)
    top = oracle.homogeneity(img, 0, 0, 8, 4, 0, 0, 1.0)
    bot = oracle.homogeneity(img, 0, 0, 8, 4, 0, 4, 1.0)
    # top: horizontal 2 per pixel except column 0 (left neighbour is the
    # frame edge, read as 0: |2*1-0-0| = 2 as well) -> 32*2 = 64; row 0
    # vertical term |2p - 0 - p| = p -> 4 even columns -> 68; rows 1-3: 0
    assert top == 68.0
    # bottom: rows 4,5,6 horizontal 2 * 8 each = 48, row 7 skipped
    assert bot == 48.0


@pytest.mark.parametrize("ret,rh,rv,rd", [(10.0, 2.0, 1.0, 3.0), (123.456, 1.07, 2.5, 1.9),
                                          (1e6, 1.0, 1.0, 1.0)])
def test_hook_f(oracle, ret, rh, rv, rd):
    # combined.diff:251-252: avg_r = (r_h + r_v + r_d) / 3 in float,
    # ret = ret * 0.8 * avg_r in double, stored to float
    avg = (F32(rh) + F32(rv) + F32(rd)) / F32(3.0)
    want = F32(float(F32(ret)) * 0.8 * float(avg))
    assert F32(oracle.hook_f(ret, rh, rv, rd)) == want
