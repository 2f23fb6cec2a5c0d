"""Regenerate tests/golden/oracle_golden.json (CPU oracle fingerprints).

Usage: python tests/golden/make_golden.py
The fixtures pin the oracle's codestream bytes (sha256), AC-strategy
histogram and per-group AC token totals for fixed synthetic inputs, so any
change to the restated algorithm is deliberate (regenerate + commit).
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd"))

import numpy as np  # noqa: E402

import oracle_ffi  # noqa: E402
from jxg.synth import synth_rgb8  # noqa: E402

CASES = [
    # (w, h, seed, distance, effort, proposals)
    (64, 64, 1, 1.0, 7, 0),
    (256, 256, 2, 1.0, 7, 3),
    (300, 200, 3, 2.0, 5, 1),
    (512, 512, 0x4A584C00, 1.0, 7, 0),
    (777, 333, 4, 0.5, 7, 2),
    (520, 2050, 5, 12.0, 4, 1),
]


def fingerprint(case):
    w, h, seed, d, e, p = case
    img = synth_rgb8(w, h, seed)
    r = oracle_ffi.encode(img, d, e, p)
    return {
        "case": list(case),
        "input_sha256": hashlib.sha256(img.tobytes()).hexdigest(),
        "bytes": len(r.bytes),
        "sha256": hashlib.sha256(r.bytes).hexdigest(),
        "acs_hist": {str(k): int(v) for k, v in zip(*np.unique(r.acs, return_counts=True))},
        "ac_tokens": r.ac_tokens.sum(axis=0).tolist(),
        "global_scale": int(r.global_scale),
        "quant_dc": int(r.quant_dc),
    }


if __name__ == "__main__":
    oracle_ffi.build()
    out = [fingerprint(c) for c in CASES]
    with open(os.path.join(HERE, "oracle_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(out), "fixtures")
