"""The synthetic input generator: the C restatement used for
the full-size fixtures (oracle/synth.c) equals jxg/synth.py byte for byte, and
the committed full-size fixtures hash the frames the GPU tests regenerate."""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("w,h,seed", [(777, 333, 4), (200, 136, 0x4A584C00), (65, 1, 7),
                                      (1, 70, 9), (1920, 1080, 0x4A584C03)])
def test_c_synth_equals_numpy(oracle, w, h, seed):
    from jxg.synth import synth_rgb8

    assert np.array_equal(oracle.synth_rgb8(w, h, seed), synth_rgb8(w, h, seed))


def test_config_fixture_inputs(oracle):
    gold = json.load(open(os.path.join(HERE, "golden", "config_golden.json")))
    for g in gold:
        if g["width"] * g["height"] > 3840 * 2160:
            continue  # the full 8K / 16K frames are hashed by the GPU tests
        img = oracle.synth_rgb8(g["width"], g["height"], g["seed"])
        assert hashlib.sha256(img.tobytes()).hexdigest() == g["input_sha256"], g["name"]


def test_config_fixture_small_encodes(oracle):
    """the 512x512 and 1080p fixtures re-encode to the same fingerprint"""
    import sys

    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_config_golden as mk

    for case in mk.CASES:
        if case[3] * case[4] > 1920 * 1080:
            continue
        img = oracle.synth_rgb8(case[3], case[4], mk.seed_of(case))
        r = oracle.encode(img, case[5], case[6], case[7], case[8], mk.filters_of(case))
        want = [g for g in json.load(open(os.path.join(HERE, "golden", "config_golden.json")))
                if g["name"] == case[0]][0]
        assert mk.fingerprint_of(case, img, r) == want, case[0]
