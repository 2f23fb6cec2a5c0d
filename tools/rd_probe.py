"""Rate-distortion probe of the CPU oracle (development tool): encodes a few
test images with oracle_ffi, decodes with oracle/jxl_decode.py and prints bpp,
PSNR and per-channel PSNR.  Usage: python tools/rd_probe.py [e4 e7 ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd")]
import jxl_decode  # noqa: E402
import oracle_ffi  # noqa: E402
from jxg.synth import natural_rgb8, synth_rgb8  # noqa: E402


natural_like = natural_rgb8


def images():
    rng = np.random.default_rng(7)
    return {
        "synth768": synth_rgb8(768, 768, 0x4A584C00),
        "natural768": natural_like(768, 768, 3),
        "rgbnoise128": rng.integers(0, 256, (128, 128, 3), dtype=np.uint8),
        "graynoise128": np.repeat(rng.integers(0, 256, (128, 128, 1), dtype=np.uint8), 3, 2),
    }


def psnr(a, b):
    m = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 10 * np.log10(255.0 ** 2 / m) if m > 0 else 99.0


def run(img, d, e, props=0):
    o = oracle_ffi.encode(img, d, e, props)
    dec = jxl_decode.decode(o.bytes).rgb
    h, w, _ = img.shape
    return (len(o.bytes) * 8.0 / (w * h), psnr(img, dec),
            [psnr(img[..., c], dec[..., c]) for c in range(3)])


if __name__ == "__main__":
    efforts = [int(a[1:]) for a in sys.argv[1:] if a.startswith("e")] or [4, 7]
    dists = [float(a[1:]) for a in sys.argv[1:] if a.startswith("d")] or [0.5, 1.0, 2.0]
    for name, img in images().items():
        for d in dists:
            for e in efforts:
                bpp, p, pc = run(img, d, e)
                print("%-13s d%-4g e%d  %6.3f bpp  PSNR %6.2f  (R %5.2f G %5.2f B %5.2f)"
                      % (name, d, e, bpp, p, *pc), flush=True)
