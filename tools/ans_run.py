"""Experiment: N 8K ANS encodes through one context (JXG_LIB_PATH selects the
build); bytes are checked equal across runs of the same frame."""
import os, sys, hashlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd"))
import torch  # noqa: F401  (one HIP runtime)
import jxg
from jxg.synth import synth_rgb8
img = synth_rgb8(7680, 4320, 0x4A584C02)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
enc = jxg.Encoder(distance=1.0, effort=7, flags=jxg.FLAG_ANS)
h = set()
for _ in range(n):
    h.add(hashlib.sha256(enc.encode(img)).hexdigest()[:16])
print("sha", sorted(h), "ms", enc.stats().get("ms_emit"))
enc.close()
