"""CPU oracle of the decode-side quality metrics -- TEST INFRASTRUCTURE ONLY.

Only tests/ (and bench.py's cpu_baseline leg, if ever) may import this; the
product path is csrc/jxg_metrics.hip behind jxg_compare_rgb8.

* ``mse_reference`` restates ImageReader::calculate_mse
  (benchmark-jpegxl/src/image_reader.rs:569-600) literally: one f64
  accumulator, samples in order, ``(o - c).powi(2)``, then ``/= len``.  It is a
  pure-Python loop (small images only).
* ``mse`` is the same number computed as an exact integer sum (every partial
  sum of the reference stays below 2**53, so both agree bit for bit).
* ``psnr`` restates ImageReader::calculate_psnr (image_reader.rs:602-606).
* ``ssim`` restates the harness's SSIM (metrics.rs:55-84 runs ImageMagick
  ``compare -metric SSIM``, which is not in the reference) as the
  Gaussian-window SSIM of Wang et al.: 11x11 window, sigma 1.5, K1 0.01,
  K2 0.03, L 255, every window fully inside the image, mean over windows and
  channels.  Separable sums in f64 with the taps in ascending order, in the
  exact op order of ssim_kernel (so the per-window values match bit for bit;
  only the final mean's summation order differs).  Parity with ImageMagick is
  unpinned.
"""
import math

import numpy as np


def mse_reference(orig, comp) -> float:
    o = np.asarray(orig, dtype=np.uint8).ravel().tolist()
    c = np.asarray(comp, dtype=np.uint8).ravel().tolist()
    if len(o) != len(c):
        raise ValueError("sample count mismatch")
    acc = 0.0
    for a, b in zip(o, c):
        d = float(a) - float(b)
        acc += d * d
    return acc / len(o)


def sse(orig, comp) -> int:
    d = np.asarray(orig, dtype=np.int64) - np.asarray(comp, dtype=np.int64)
    return int(np.sum(d * d))


def mse(orig, comp) -> float:
    n = np.asarray(orig).size
    return float(sse(orig, comp)) / float(n)


def psnr(mse_value: float, max_value: float = 255.0) -> float:
    if mse_value == 0.0:
        return math.inf
    return 10.0 * math.log10((max_value * max_value) / mse_value)


def gaussian_window():
    """== gauss_window() in csrc/jxg_host.cpp (libm exp on both sides)."""
    g = [math.exp(-((k - 5.0) * (k - 5.0)) / (2.0 * 1.5 * 1.5)) for k in range(11)]
    s = 0.0
    for v in g:
        s += v
    return np.array([v / s for v in g], dtype=np.float64)


def ssim_map(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Per-window SSIM of one channel (2-D arrays), valid windows only."""
    g = gaussian_window()
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    h, w = a.shape
    oh, ow = h - 10, w - 10
    if oh <= 0 or ow <= 0:
        return np.zeros((0, 0))
    quant = (a, b, a * a, b * b, a * b)
    hs = []
    for q in quant:
        acc = np.zeros((h, ow))
        for k in range(11):
            acc = acc + g[k] * q[:, k:k + ow]
        hs.append(acc)
    m = []
    for hq in hs:
        acc = np.zeros((oh, ow))
        for k in range(11):
            acc = acc + g[k] * hq[k:k + oh, :]
        m.append(acc)
    c1 = (0.01 * 255.0) * (0.01 * 255.0)
    c2 = (0.03 * 255.0) * (0.03 * 255.0)
    mab = m[0] * m[1]
    maa = m[0] * m[0]
    mbb = m[1] * m[1]
    vaa = m[2] - maa
    vbb = m[3] - mbb
    cab = m[4] - mab
    num = (2.0 * mab + c1) * (2.0 * cab + c2)
    den = (maa + mbb + c1) * (vaa + vbb + c2)
    return num / den


def ssim(orig: np.ndarray, comp: np.ndarray) -> float:
    """Mean over the three channels' valid windows; NaN under 11x11."""
    o = np.asarray(orig)
    c = np.asarray(comp)
    h, w = o.shape[:2]
    if h < 11 or w < 11:
        return math.nan
    tot = 0.0
    for ch in range(3):
        tot += float(np.sum(ssim_map(o[:, :, ch], c[:, :, ch])))
    return tot / (3.0 * (w - 10) * (h - 10))
