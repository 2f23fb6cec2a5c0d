"""GPU probe: merge-stage time (ms_front - ms_front_kernel, one-at-a-time
encodes) on the 8K bench frame and on photographic-like content."""
import os
import sys

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import torch  # noqa: F401,E402  (one HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd")]
import numpy as np  # noqa: E402

import jxg  # noqa: E402
from jxg.synth import config_image, natural_rgb8  # noqa: E402

jxg.load()
for name, img in (("bench 8K", config_image(2)), ("natural 3840x2160", natural_rgb8(3840, 2160, 5))):
    with jxg.Encoder(distance=1.0, effort=7, flags=jxg.FLAG_ANS) as enc:
        ms, fk = [], []
        for i in range(6):
            b = enc.encode(img)
            st = enc.stats()
            if i:
                ms.append(st["ms_front"] - st["ms_front_kernel"])
                fk.append(st["ms_front_kernel"])
        print("%-18s merge stage %.4f ms  front %.4f ms  %d bytes" % (
            name, float(np.median(ms)), float(np.median(fk)), len(b)), flush=True)
