"""Debug probe: the GPU's 128 / 256 px candidate estimates (JXG_DEBUG_BIGCOST
dump) beside the oracle's (jxo_set_debug_big_cost), per group and candidate.
The GPU drops candidates whose estimate after Y alone reaches the region's
current sum (hook F off): those read +inf here."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd"),
                os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
os.environ["GPU_MAX_HW_QUEUES"] = "16"
import torch  # noqa: E402,F401  (one HIP runtime, as in tests/conftest.py)
os.environ["JXG_DEBUG_BIGCOST"] = os.path.join(ROOT, "gpurun_out", "bigcost.bin")

import jxg  # noqa: E402

jxg.load()
import oracle_ffi as O  # noqa: E402
from test_gpu_bigvb import gradient_rgb8  # noqa: E402

w, h = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (512, 512)
d = 1.0
img = gradient_rgb8(w, h, w * 7 + h)
_, ref = O.debug_big_costs(img, d, 8, 0, 1)
with jxg.Encoder(distance=d, effort=8, flags=jxg.FLAG_ANS) as enc:
    enc.encode(img)
got = np.fromfile(os.environ["JXG_DEBUG_BIGCOST"], dtype=np.float32)[: ref.size].reshape(ref.shape)
np.set_printoptions(linewidth=200, precision=4, suppress=True)
for g in range(ref.shape[0]):
    print("group", g)
    print(" oracle", ref[g])
    print(" gpu   ", got[g])
    print(" diff  ", got[g] - ref[g])
