"""CPU checks of the decode-side metrics oracle and the harness counterpart.

* oracle/metrics.py: the integer-sum MSE equals the reference's sequential
  f64 accumulation (image_reader.rs:569-600) bit for bit; PSNR follows
  image_reader.rs:602-606; SSIM (metrics.rs:55-84 counterpart, parity with
  ImageMagick unpinned) equals a direct 2-D window evaluation and is exactly
  1.0 on identical images.
* jxg.harness: CSV headers / rows in the csv_writer.rs schema with Rust
  number formatting, and compare_results' diff + summary (benchmark.rs:727-864).
"""
import csv
import math

import numpy as np
import pytest

import metrics


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("h,w,seed", [(1, 1, 0), (7, 5, 1), (16, 24, 2), (33, 17, 3)])
def test_mse_matches_sequential_f64(h, w, seed):
    a, b = _img(h, w, seed), _img(h, w, seed + 100)
    assert metrics.mse(a, b) == metrics.mse_reference(a, b)


def test_mse_extremes_and_psnr():
    a = np.zeros((9, 9, 3), np.uint8)
    b = np.full((9, 9, 3), 255, np.uint8)
    assert metrics.sse(a, b) == 243 * 65025
    assert metrics.mse(a, b) == 65025.0 == metrics.mse_reference(a, b)
    assert metrics.psnr(65025.0) == 0.0
    assert metrics.psnr(0.0) == math.inf
    assert metrics.psnr(1.0) == 10.0 * math.log10(65025.0)


def _ssim_direct(a, b):
    """Textbook 2-D window SSIM (pure Python, different op order)."""
    g1 = metrics.gaussian_window()
    g = np.outer(g1, g1)
    c1, c2 = (0.01 * 255) ** 2, (0.03 * 255) ** 2
    h, w = a.shape
    out = np.zeros((h - 10, w - 10))
    for y in range(h - 10):
        for x in range(w - 10):
            pa = a[y:y + 11, x:x + 11].astype(np.float64)
            pb = b[y:y + 11, x:x + 11].astype(np.float64)
            ma, mb = float(np.sum(g * pa)), float(np.sum(g * pb))
            va = float(np.sum(g * pa * pa)) - ma * ma
            vb = float(np.sum(g * pb * pb)) - mb * mb
            cab = float(np.sum(g * pa * pb)) - ma * mb
            out[y, x] = ((2 * ma * mb + c1) * (2 * cab + c2)) / ((ma * ma + mb * mb + c1) * (va + vb + c2))
    return out


def test_ssim_map_matches_direct_window():
    a = _img(14, 16, 7)
    b = np.clip(a.astype(int) + np.random.default_rng(8).integers(-20, 21, a.shape), 0, 255)
    for ch in range(3):
        np.testing.assert_allclose(metrics.ssim_map(a[:, :, ch], b[:, :, ch]),
                                   _ssim_direct(a[:, :, ch], b[:, :, ch]), rtol=1e-9, atol=1e-12)


def test_ssim_identical_is_one_and_small_is_nan():
    a = _img(20, 23, 9)
    assert metrics.ssim(a, a) == 1.0
    assert math.isnan(metrics.ssim(a[:10], a[:10]))
    assert metrics.ssim(a, 255 - a) < 0.5


def test_gaussian_window_normalized():
    g = metrics.gaussian_window()
    assert g.shape == (11,) and abs(g.sum() - 1.0) < 1e-15
    assert np.allclose(g, g[::-1]) and g[5] == g.max()


def test_rust_number_formatting(jxg_mod):
    f64, f32 = jxg_mod.rust_f64, jxg_mod.rust_f32
    assert [f64(v) for v in (1.0, 0.5, 1e-7, 1e20, -2.5, 0.0)] == [
        "1", "0.5", "0.0000001", "100000000000000000000", "-2.5", "0"]
    assert f64(float("nan")) == "NaN" and f64(float("inf")) == "inf"
    assert f64(0.1 + 0.2) == "0.30000000000000004"
    # f32 distance column: shortest f32 digits (0.1f32 -> "0.1", not 0.10000000149...)
    assert [f32(v) for v in (0.1, 1.0, 1.5, 12.0)] == ["0.1", "1", "1.5", "12"]


def _result(h, name, d, e, fs, psnr, ssim):
    return h.ComparisonResult(name + ".png", "%s-%s-%d.jxl" % (name, d, e), d, e, 1000, fs, 768,
                              768, h.file_size_ratio(1000, fs, "comp"),
                              h.file_size_ratio(768, fs, "comp"), 12.5, psnr, ssim, 0.0, 0.0,
                              0.0, 0.0)


def test_csv_schema_and_compare_results(tmp_path):
    from jxg import harness as h
    r1 = tmp_path / "run1" / "comparisons.csv"
    r2 = tmp_path / "run2" / "comparisons.csv"
    for path, rows in ((r1, [_result(h, "b", 1.0, 7, 200, 40.0, 0.9),
                             _result(h, "a", 0.5, 7, 400, 45.0, 0.95)]),
                       (r2, [_result(h, "a", 0.5, 7, 380, 45.5, 0.96),
                             _result(h, "b", 1.0, 7, 190, 39.0, 0.9)])):
        h.write_csv_header(str(path), h.RESULT_HEADER)
        h.write_csv_header(str(path), h.RESULT_HEADER)  # no second header
        h.write_csv(rows, str(path))
    rows = list(csv.reader(open(r1)))
    assert rows[0] == h.RESULT_HEADER and len(rows[0]) == 17 and len(rows) == 3
    assert rows[1][:4] == ["b.png", "b-1.0-7.jxl", "1", "7"]
    assert rows[1][8] == "5" and rows[1][10] == "12.5" and rows[1][11] == "40"
    back = h.read_csv(str(r1))
    assert back[0] == _result(h, "b", 1.0, 7, 200, 40.0, 0.9)
    diffs, summary = h.compare_results(str(r1), str(r2))
    assert [d.orig_image_name for d in diffs] == ["a.png", "b.png"]
    assert diffs[0].diff_comp_file_size == -20.0 and diffs[1].diff_psnr == -1.0
    assert summary.orig_image_name == "Summary" and summary.effort == 0
    assert summary.diff_psnr == (0.5 + -1.0) / 2
    out = list(csv.reader(open(tmp_path / "run1" / "summary.csv")))
    assert out[0] == h.DIFF_HEADER and out[1][0] == "Summary" and out[1][11] == "-0.25"
    assert len(list(csv.reader(open(tmp_path / "run1" / "comparison_diffs.csv")))) == 3


def test_file_size_ratio():
    from jxg import harness as h
    assert h.file_size_ratio(0, 5, "orig") == 0.0 and h.file_size_ratio(5, 0, "comp") == 0.0
    assert h.file_size_ratio(10, 4, "comp") == 2.5 and h.file_size_ratio(10, 4, "orig") == 0.4
    with pytest.raises(ValueError):
        h.file_size_ratio(1, 1, "x")
