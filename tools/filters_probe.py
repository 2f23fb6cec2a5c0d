"""GPU probe: cost of the restoration-filter flags on the 8K bench frame
(one-at-a-time encodes, the front kernel alone)."""
import os
import sys

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import torch  # noqa: F401,E402  (one HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd")]
import numpy as np  # noqa: E402

import jxg  # noqa: E402
from jxg.synth import config_image  # noqa: E402

jxg.load()
img = config_image(2)
for name, fl in (("none", 0), ("gab", jxg.FLAG_GABORISH), ("epf", jxg.FLAG_EPF),
                 ("gab+epf", jxg.FLAG_GABORISH | jxg.FLAG_EPF)):
    with jxg.Encoder(distance=1.0, effort=7, flags=fl | jxg.FLAG_ANS) as enc:
        fk, tot = [], []
        for i in range(6):
            b = enc.encode(img)
            st = enc.stats()
            if i:
                fk.append(st["ms_front_kernel"])
                tot.append(st["ms_total"])
        print("%-8s front_kernel %.4f ms (min %.4f)  total %.3f ms  %d bytes" % (
            name, float(np.median(fk)), min(fk), float(np.median(tot)), len(b)), flush=True)
