"""CPU oracle: merged varblocks (16x8 ... 64x64).

The tables and transforms of oracle/merge.c against independent restatements
(numpy float64 DCT, the test decoder's Python natural order / weights), and
encode -> decode round trips that exercise every merged shape, the thesis hook
F on merge candidates (NaN estimates are accepted, combined.diff:294 context)
and partial tiles.  [ext] libjxl stages: parity unpinned against libjxl.
"""
import math

import numpy as np
import pytest


def smooth_rgb8(w, h, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    fx, fy = rng.uniform(5, 40, 3), rng.uniform(5, 40, 3)
    img = np.stack([128 + 90 * np.sin(x / fx[c] + y / fy[c] + c) for c in range(3)], -1)
    for ty in range(0, h, 64):
        for tx in range(0, w, 64):
            k = rng.integers(0, 6)
            if k == 0:
                img[ty:ty + 64, tx:tx + 64] += rng.normal(0, 25, img[ty:ty + 64, tx:tx + 64].shape)
            elif k == 1:
                img[ty:ty + 64, tx:tx + 64] = rng.uniform(0, 255, 3)
    return np.clip(img, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("n", [1, 2, 4, 8, 16, 32, 64, 128, 256])
def test_lee_dct_matches_float64(oracle, n):
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, n).astype(np.float32)
    k = np.arange(n)[:, None]
    m = np.cos(math.pi * (2 * np.arange(n)[None, :] + 1) * k / (2 * n))
    ref = (m @ x.astype(np.float64)) * np.where(k[:, 0] == 0, 1.0 / n, math.sqrt(2) / n)
    got = oracle.dct(x)
    assert np.allclose(got, ref, atol=2e-6 * max(1, n / 8)), (got, ref)


@pytest.mark.parametrize("kind", range(10))
def test_kind_tables_match_decoder(oracle, decoder, kind):
    w, nat = oracle.kind_tables(kind)
    bands = None
    if kind >= 6:  # written into DequantMatrices: binary16 parameters
        bands = [[64.0 * float(np.float16(r[0] / 64.0))] + [float(np.float16(v)) for v in r[1:]]
                 for r in decoder.KIND_BANDS[kind]]
    iw, order = decoder.kind_tables(kind, bands)
    rows, cols = decoder.KIND_DIM[kind]
    # natural order: a permutation, LLF (rows/8 x cols/8) first in raster order
    assert sorted(nat.tolist()) == list(range(rows * cols))
    inv = np.empty(rows * cols, dtype=np.int64)
    inv[nat] = np.arange(rows * cols)
    assert inv.tolist() == order
    cs, cl = rows // 8, cols // 8
    assert [inv[p] for p in range(cs * cl)] == [y * cols + x for y in range(cs) for x in range(cl)]
    # weights: float32 of the decoder's double computation
    assert np.array_equal(w, (1.0 / iw).astype(np.float32))


CASES = [(256, 256, 1.0, 7, 0), (200, 264, 2.0, 5, 3), (520, 136, 0.5, 6, 2),
         (333, 333, 3.0, 7, 1), (136, 520, 1.0, 7, 3)]


@pytest.mark.parametrize("w,h,d,e,p", CASES)
def test_varblock_roundtrip(oracle, decoder, w, h, d, e, p):
    import jxg

    img = smooth_rgb8(w, h, w * 31 + h)
    r = oracle.encode(img, d, e, p)
    assert (r.acs & 0x80).any()
    dec = decoder.decode(r.bytes)
    assert np.array_equal(dec.acs, r.acs)
    assert np.array_equal(dec.qf - 1, r.qf)
    assert np.array_equal(dec.dc, r.dc)
    assert np.array_equal(dec.ac, r.ac)
    assert np.array_equal(dec.ac_tokens, r.ac_tokens)


@pytest.mark.parametrize("e", [5, 6, 7])
def test_merges_pay_on_smooth_content(oracle, decoder, e):
    """Pure smooth content: the merge stage must shrink the codestream without
    losing PSNR against the 8x8-only search (effort 4)."""
    import jxg

    y, x = np.mgrid[0:256, 0:320].astype(np.float64)
    img = np.stack([128 + 60 * np.sin(x / 19.0 + c) * np.cos(y / 23.0) for c in range(3)],
                   -1).astype(np.uint8)
    r, r4 = oracle.encode(img, 1.0, e, 0), oracle.encode(img, 1.0, 4, 0)
    psnr = jxg.calculate_psnr(jxg.calculate_mse(img, decoder.decode(r.bytes).rgb))
    psnr4 = jxg.calculate_psnr(jxg.calculate_mse(img, decoder.decode(r4.bytes).rgb))
    assert len(r.bytes) < len(r4.bytes)
    assert psnr > psnr4 - 0.25, (psnr, psnr4)


def test_every_shape_is_reachable(oracle):
    seen = set()
    for w, h, d, e, p in CASES:
        r = oracle.encode(smooth_rgb8(w, h, w * 31 + h), d, e, p)
        seen |= set((r.acs[~(r.acs & 0x80).astype(bool)] & 0x7F).tolist())
    # a vertical edge in the middle of every tile over a vertical gradient:
    # two 64x32 (tall) halves per tile
    y, x = np.mgrid[0:128, 0:128].astype(np.float64)
    img = np.stack([100 + 40 * np.sin(y / 37.0 + c) + np.where((x % 64) < 32, 0, 70 + 20 * c)
                    for c in range(3)], -1)
    r = oracle.encode(np.clip(img, 0, 255).astype(np.uint8), 1.0, 7, 0)
    seen |= set((r.acs[~(r.acs & 0x80).astype(bool)] & 0x7F).tolist())
    assert {4, 5, 6, 7, 10, 11, 18, 19, 20} <= seen, sorted(seen)


def test_hook_f_nan_estimates_merge(oracle):
    """An all-black tile has 0/0 similarity ratios (NaN), so with hook F every
    estimate is NaN: the 8x8 search keeps DCT8 (NaN never beats FLT_MAX) but
    the merge comparison `candidate >= current` is false for NaN, so every
    level accepts its last candidate -> two DCT32X64 varblocks at effort 7."""
    img = np.zeros((64, 64, 3), dtype=np.uint8)
    r0 = oracle.encode(img, 1.0, 7, 0)
    rf = oracle.encode(img, 1.0, 7, 2)
    assert (r0.acs == 0).all()
    assert np.isnan(rf.homog).all()
    assert rf.acs[0, 0] == 20 and rf.acs[4, 0] == 20
    assert ((rf.acs & 0x7F) == 20).all()


def _gradient_rgb8(w, h, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.stack([128 + 60 * np.sin(x / rng.uniform(150, 400) + y / rng.uniform(150, 400) + c)
                    for c in range(3)], -1)
    return np.clip(img, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("w,h,d", [(512, 512, 1.0), (768, 520, 2.0)])
def test_big_varblocks_roundtrip(oracle, decoder, w, h, d):
    """Effort 8 adds the 128 / 256 px levels (DCT128X128 / 128X64 / 64X128 /
    256X256 / 256X128 / 128X256, raw ids 21-26; north_star's "2x2...256x256"):
    on smooth content they are chosen, the decoder recovers every integer of
    the codestream, and the RD note of DESIGN.md §3.10 holds (fewer bytes than
    effort 7, PSNR within 0.5 dB)."""
    import jxg

    img = _gradient_rgb8(w, h, w + h)
    r7 = oracle.encode(img, d, 7, 0, 1)
    r8 = oracle.encode(img, d, 8, 0, 1)
    first = r8.acs[(r8.acs & 0x80) == 0]
    assert np.isin(first, [21, 22, 23, 24, 25, 26]).any()
    assert not np.isin(r7.acs & 0x7F, [21, 22, 23, 24, 25, 26]).any()
    dec = decoder.decode(r8.bytes)
    for k in ("acs", "dc", "ac", "ac_tokens"):
        assert np.array_equal(getattr(dec, k), getattr(r8, k)), k
    p7 = jxg.calculate_psnr(jxg.calculate_mse(img, decoder.decode(r7.bytes).rgb))
    p8 = jxg.calculate_psnr(jxg.calculate_mse(img, dec.rgb))
    assert len(r8.bytes) < len(r7.bytes)
    assert p8 > p7 - 0.5


def test_every_big_shape_is_decodable(oracle, decoder):
    """All six 128 / 256 px shapes appear across these frames and decode."""
    seen = set()
    for (w, h, d) in [(512, 512, 1.0), (768, 520, 2.0)]:
        r = oracle.encode(_gradient_rgb8(w, h, w + h), d, 8, 0, 1)
        seen |= set(int(t) for t in np.unique(r.acs[(r.acs & 0x80) == 0]))
        assert np.array_equal(decoder.decode(r.bytes).ac, r.ac)
    assert {21, 22, 23, 24, 25, 26} <= seen


def test_big_quant_tables_travel_in_the_stream(oracle, decoder, monkeypatch):
    """Effort >= 8 streams carry the quant tables of the 128 / 256 px kinds
    (HfGlobal DequantMatrices not all_default: Library for the other 13 tables,
    mode DCT with binary16 band parameters for those of DCT128X128 / 128X64 /
    256X256 / 256X128 the frame uses), so they decode to the same pixels whatever the decoder's built-in
    defaults for those kinds are; effort 7 streams still signal all_default."""
    img = _gradient_rgb8(512, 512, 1024)
    r8 = oracle.encode(img, 1.0, 8, 0, 1)
    assert np.isin(r8.acs[(r8.acs & 0x80) == 0], [21, 22, 23, 24, 25, 26]).any()
    ref = decoder.decode(r8.bytes)
    kind_of = {22: 6, 23: 6, 21: 7, 25: 8, 26: 8, 24: 9}
    used = {kind_of[int(t)] for t in np.unique(r8.acs) if int(t) in kind_of}
    assert sorted(ref.qm_params) == sorted(used) and len(used) >= 2
    # perturb the decoder's built-in tables of every big kind (and its cache)
    bad = [list(b) for b in decoder.KIND_BANDS]
    for k in (6, 7, 8, 9):
        bad[k] = [[r[0] * 0.37] + [v * 1.9 for v in r[1:]] for r in decoder.KIND_BANDS[k]]
    monkeypatch.setattr(decoder, "KIND_BANDS", bad)
    monkeypatch.setattr(decoder, "_KIND_CACHE", {})
    got = decoder.decode(r8.bytes)
    assert np.array_equal(got.rgb, ref.rgb)
    # ... whereas a stream that relies on the defaults would change: e7 keeps
    # all_default, and perturbing a kind it uses (DCT64X64) moves its pixels
    r7 = oracle.encode(img, 1.0, 7, 0, 1)
    assert decoder.decode(r7.bytes).qm_params == {}
    ok7 = decoder.decode(r7.bytes).rgb
    bad[5] = [[r[0] * 0.37] + list(r[1:]) for r in decoder.KIND_BANDS[5]]
    monkeypatch.setattr(decoder, "_KIND_CACHE", {})
    assert np.isin(r7.acs & 0x7F, [18]).any()
    assert not np.array_equal(decoder.decode(r7.bytes).rgb, ok7)


def test_whole_group_bin_can_pass_u16(oracle):
    """the premise of tests/test_gpu_bigvb.py::test_whole_group_histogram_bin_above_u16
    (ADVICE r5): one pass group of this frame puts more than 65535 tokens into
    one (static cluster, token) bin at effort 8"""
    y, x = np.mgrid[0:256, 0:512]
    m = ((x + y) % 2).astype(bool)[..., None]
    img = np.where(m, np.array([255, 0, 0]), np.array([0, 60, 255])).astype(np.uint8)
    r, mx = oracle.max_group_bin(img, 1.0, 8, 0, 0)
    assert mx > 65535 and (r.acs == 24).any()
