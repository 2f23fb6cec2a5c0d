"""Every BASELINE.json configuration at full size on the GPU against the CPU
oracle's committed fingerprints (tests/golden/config_golden.json, made by
tests/golden/make_config_golden.py): codestream bytes (sha256), per-group AC
token counts (sha256) and, where the maps are kept, the AC-strategy histogram.
The *_cjxl cases encode with JXG_FLAGS_CJXL_DEFAULTS (bench.py's headline).
Inputs are generated on the device (jxg_synth_rgb8_device) and their bytes are
checked against the fixture's input hash first.  The 1080p frames go through
the batch entry point (jxg_encode_batch_rgb8) at d0.5 / d1 / d2."""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "config_golden.json")))
BY_NAME = {g["name"]: g for g in GOLD}

pytestmark = pytest.mark.gpu


def _tok_sha(ac_tokens):
    return hashlib.sha256(np.ascontiguousarray(ac_tokens.astype("<u4")).tobytes()).hexdigest()


def _device_frame(jxg_mod, g):
    import torch

    from jxg.synth import synth_rgb8_device

    t = synth_rgb8_device(g["width"], g["height"], g["seed"])
    torch.cuda.synchronize()
    host = t.cpu().numpy()
    assert hashlib.sha256(host.tobytes()).hexdigest() == g["input_sha256"], "device synth drifted"
    return t


@pytest.mark.parametrize("name", [g["name"] for g in GOLD if g["config"] != 3])
def test_config_matches_oracle(jxg_mod, name):
    g = BY_NAME[name]
    t = _device_frame(jxg_mod, g)
    flags = (jxg_mod.FLAG_ANS if g["coder"] else 0) | (
        jxg_mod.FLAG_KEEP_MAPS if g["width"] * g["height"] <= 8294400 else 0)
    if g.get("filters"):  # cjxl's defaults (the bench headline's preset)
        assert g["filters"] == jxg_mod.ORACLE_FILTERS_CJXL_DEFAULTS and g["coder"] == 1
        flags |= jxg_mod.FLAGS_CJXL_DEFAULTS
    with jxg_mod.Encoder(distance=g["distance"], effort=g["effort"], proposals=g["proposals"],
                         flags=flags) as enc:
        data = enc.encode_device(t.data_ptr(), g["width"], g["height"])
        st = enc.stats()
    del t
    assert _tok_sha(st["ac_tokens"]) == g["ac_tokens_sha256"], "AC token counts differ"
    if "acs" in st:
        hist = {str(k): int(v) for k, v in zip(*np.unique(st["acs"], return_counts=True))}
        assert hist == g["acs_hist"], "AC strategy map differs"
    assert len(data) == g["bytes"]
    assert hashlib.sha256(data).hexdigest() == g["sha256"], "codestream differs from the oracle"


@pytest.mark.parametrize("preset", ["plain", "cjxl"])
@pytest.mark.parametrize("distance", [0.5, 1.0, 2.0])
def test_batch_1080p_matches_oracle(jxg_mod, distance, preset):
    """config 3 (1080p frames through jxg_encode_batch_rgb8) with no flags and
    at cjxl's defaults (the preset bench.py's config-3 line times)"""
    from jxg.synth import synth_rgb8_device

    cjxl = preset == "cjxl"
    gs = [g for g in GOLD if g["config"] == 3 and g["distance"] == distance
          and bool(g.get("filters")) == cjxl]
    assert len(gs) == 2
    frames = [synth_rgb8_device(g["width"], g["height"], g["seed"]).cpu().numpy() for g in gs]
    for f, g in zip(frames, gs):
        assert hashlib.sha256(f.tobytes()).hexdigest() == g["input_sha256"]
    flags = jxg_mod.FLAGS_CJXL_DEFAULTS if cjxl else 0
    with jxg_mod.Encoder(distance=distance, effort=7, flags=flags) as enc:
        outs = enc.encode_batch(frames)
    for data, g in zip(outs, gs):
        assert len(data) == g["bytes"] and hashlib.sha256(data).hexdigest() == g["sha256"], g["name"]


@pytest.mark.parametrize("coder", ["prefix", "ans"])
def test_one_stream_fallback_same_bytes(jxg_mod, coder):
    """The split assembly's fallback (one-stream stage_concat, taken when the
    prefix bound is exceeded; forced here by JXG_FLAG_FORCE_ONE_STREAM) gives
    the split path's bytes, and both equal the oracle's fingerprint."""
    name = "8k_d1_ans" if coder == "ans" else "4k_d1"
    g = BY_NAME[name]
    t = _device_frame(jxg_mod, g)
    base = jxg_mod.FLAG_ANS if coder == "ans" else 0
    outs = []
    for extra in (0, jxg_mod.FLAG_FORCE_ONE_STREAM):
        with jxg_mod.Encoder(distance=g["distance"], effort=g["effort"], proposals=g["proposals"],
                             flags=base | extra) as enc:
            outs.append(enc.encode_device(t.data_ptr(), g["width"], g["height"]))
    del t
    assert outs[0] == outs[1]
    assert hashlib.sha256(outs[1]).hexdigest() == g["sha256"]
