"""Regenerate tests/golden/config_golden.json: CPU-oracle fingerprints of every
BASELINE.json configuration at full size (SURVEY.md §8(d) inputs).

Usage: python tests/golden/make_config_golden.py        (~1 min on 8 cores)

Each entry pins, for the synthetic frame of one config (jxg/synth.py
synth_rgb8, generated here by its C restatement oracle/synth.c), the oracle's
codestream (size + sha256), its per-group AC token counts (sha256 of the
little-endian u32 [groups][X, Y, B] array + total) and the AC-strategy
histogram.  tests/test_gpu_configs.py encodes the same frames on the GPU
(inputs generated on the device by jxg_synth_rgb8_device) and compares.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle_ffi  # noqa: E402

SEED_BASE = 0x4A584C00
# (name, config index, frame, width, height, distance, effort, proposals, coder[,
#  filters]) -- filters: the oracle's mask (oracle/jxo.h), 7 = cjxl's defaults
#  (Gaborish | EPF | masking AQ, = JXG_FLAGS_CJXL_DEFAULTS with coder 1)
CASES = [
    ("cpu512_d1", 0, 0, 512, 512, 1.0, 7, 0, 0),
    ("4k_d1", 1, 0, 3840, 2160, 1.0, 7, 0, 0),
    ("8k_d1_prefix", 2, 0, 7680, 4320, 1.0, 7, 0, 0),
    ("8k_d1_ans", 2, 0, 7680, 4320, 1.0, 7, 0, 1),
    ("8k_d1_pf", 2, 0, 7680, 4320, 1.0, 7, 3, 0),
    ("1080p_f0_d0.5", 3, 0, 1920, 1080, 0.5, 7, 0, 0),
    ("1080p_f0_d1", 3, 0, 1920, 1080, 1.0, 7, 0, 0),
    ("1080p_f0_d2", 3, 0, 1920, 1080, 2.0, 7, 0, 0),
    ("1080p_f1_d0.5", 3, 1, 1920, 1080, 0.5, 7, 0, 0),
    ("1080p_f1_d1", 3, 1, 1920, 1080, 1.0, 7, 0, 0),
    ("1080p_f1_d2", 3, 1, 1920, 1080, 2.0, 7, 0, 0),
    ("16k_d1_pf", 4, 0, 16384, 16384, 1.0, 7, 3, 0),
    # round 5: the encode the harness's argv gets (bench.py's headline preset)
    ("cpu512_d1_cjxl", 0, 0, 512, 512, 1.0, 7, 0, 1, 7),
    ("4k_d1_cjxl", 1, 0, 3840, 2160, 1.0, 7, 0, 1, 7),
    ("8k_d1_cjxl", 2, 0, 7680, 4320, 1.0, 7, 0, 1, 7),
    ("8k_d1_cjxl_pf", 2, 0, 7680, 4320, 1.0, 7, 3, 1, 7),
    ("8k_d1_cjxl_f100", 2, 100, 7680, 4320, 1.0, 7, 0, 1, 7),
    # round 6: configs 3 and 4 at the headline preset too
    ("1080p_f0_d0.5_cjxl", 3, 0, 1920, 1080, 0.5, 7, 0, 1, 7),
    ("1080p_f0_d1_cjxl", 3, 0, 1920, 1080, 1.0, 7, 0, 1, 7),
    ("1080p_f0_d2_cjxl", 3, 0, 1920, 1080, 2.0, 7, 0, 1, 7),
    ("1080p_f1_d0.5_cjxl", 3, 1, 1920, 1080, 0.5, 7, 0, 1, 7),
    ("1080p_f1_d1_cjxl", 3, 1, 1920, 1080, 1.0, 7, 0, 1, 7),
    ("1080p_f1_d2_cjxl", 3, 1, 1920, 1080, 2.0, 7, 0, 1, 7),
    ("16k_d1_cjxl_pf", 4, 0, 16384, 16384, 1.0, 7, 3, 1, 7),
]


def seed_of(case):
    return SEED_BASE + case[1] + case[2]


def filters_of(case):
    return case[9] if len(case) > 9 else 0


def fingerprint_of(case, img, r):
    name, cfg, fr, w, h, d, e, p, coder = case[:9]
    tok = np.ascontiguousarray(r.ac_tokens.astype("<u4"))
    out = {
        "name": name, "config": cfg, "frame": fr, "width": w, "height": h, "distance": d,
        "effort": e, "proposals": p, "coder": coder, "seed": seed_of(case),
        "input_sha256": hashlib.sha256(img.tobytes()).hexdigest(),
        "bytes": len(r.bytes),
        "sha256": hashlib.sha256(r.bytes).hexdigest(),
        "ac_tokens_sha256": hashlib.sha256(tok.tobytes()).hexdigest(),
        "ac_tokens_total": [int(x) for x in tok.sum(axis=0)],
        "acs_hist": {str(k): int(v) for k, v in zip(*np.unique(r.acs, return_counts=True))},
    }
    if filters_of(case):
        out["filters"] = filters_of(case)
    return out


if __name__ == "__main__":
    oracle_ffi.build()
    oracle_ffi.set_threads(os.cpu_count() or 1)
    out, imgs = [], {}
    for case in CASES:
        key = (case[3], case[4], seed_of(case))
        if key not in imgs:
            imgs.clear()
            imgs[key] = oracle_ffi.synth_rgb8(case[3], case[4], seed_of(case))
        img = imgs[key]
        r = oracle_ffi.encode(img, case[5], case[6], case[7], case[8], filters_of(case))
        out.append(fingerprint_of(case, img, r))
        print(case[0], out[-1]["bytes"], flush=True)
    with open(os.path.join(HERE, "config_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(out), "fixtures")
