"""Experiment: run N 8K encodes through one context (JXG_LIB_PATH selects the
build), so a JXG_MERGE_PROFILE build prints its per-phase cycle sums on destroy."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd"))
import torch  # noqa: F401  (one HIP runtime)
import jxg
from jxg.synth import synth_rgb8
img = synth_rgb8(7680, 4320, 0x4A584C02)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
enc = jxg.Encoder(distance=1.0, effort=7)
for _ in range(n):
    enc.encode(img)
print("ms_front", enc.stats()["ms_front"])
enc.close()
