"""RD of the restoration filters (oracle encoder == GPU bytes, oracle decoder;
DESIGN.md §3.8): bpp and PSNR on the bench's 1920x1080 frames."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd")]
import jxl_decode  # noqa: E402
import oracle_ffi  # noqa: E402

import jxg  # noqa: E402
from jxg.synth import config_image, natural_rgb8  # noqa: E402

frames = [("natural_rgb8(1920,1080,3)", natural_rgb8(1920, 1080, 3), (1.0, 2.0, 3.0)),
          ("bench crop 1920x1080", config_image(2)[:1080, :1920], (1.0, 2.0))]
for name, img, dists in frames:
    for d in dists:
        for fl, fname in ((0, "none"), (1, "gab"), (2, "epf"), (3, "gab+epf")):
            t = time.time()
            r = oracle_ffi.encode(img, d, 7, 0, 1, fl)
            dec = jxl_decode.decode(r.bytes)
            mse = jxg.calculate_mse(img, dec.rgb)
            print("%-26s d%.1f %-8s %9d B  %.4f bpp  %.3f dB  (%.0f s)" % (
                name, d, fname, len(r.bytes), len(r.bytes) * 8 / img.shape[0] / img.shape[1],
                jxg.calculate_psnr(mse), time.time() - t), flush=True)
