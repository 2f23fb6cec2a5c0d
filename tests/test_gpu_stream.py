"""Streaming encode (jxg_submit_rgb8[_device] / jxg_receive): the library's
one-thread software pipeline (4-12 lanes) returns, in submission order,
exactly the codestreams of one-at-a-time jxg_encode_rgb8 calls -- for frames of
mixed sizes and content, both AC coders, receives interleaved with submits, and
a full-size 8K ANS sequence against the oracle's committed fingerprint; the
batch entry point (jxg_encode_batch_rgb8, built on the same pipeline) too."""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = {g["name"]: g for g in json.load(open(os.path.join(HERE, "golden", "config_golden.json")))}

pytestmark = pytest.mark.gpu


def _frames():
    from jxg.synth import natural_rgb8, synth_rgb8

    sizes = [(640, 480), (333, 250), (640, 480), (1024, 520), (64, 64), (777, 301), (640, 480),
             (9, 7), (1280, 720)]
    out = []
    for i, (w, h) in enumerate(sizes):
        out.append(natural_rgb8(w, h, 50 + i) if i % 2 and min(w, h) >= 200 else
                   synth_rgb8(w, h, 90 + i))
    return out


@pytest.mark.parametrize("flags_name", ["prefix", "ans"])
def test_stream_equals_single(jxg_mod, flags_name):
    flags = jxg_mod.FLAG_ANS if flags_name == "ans" else 0
    frames = _frames()
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=flags) as enc:
        want = [enc.encode(f) for f in frames]
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=flags) as enc:
        got = []
        for i, f in enumerate(frames):
            enc.submit(f)
            if i == 2:  # a receive in the middle of the stream
                got.append(enc.receive())
        assert enc.pending() == len(frames) - 1
        while enc.pending():
            got.append(enc.receive())
        with pytest.raises(jxg_mod.JxgError):
            enc.receive()
        # the context still encodes one-at-a-time afterwards
        assert enc.encode(frames[0]) == want[0]
    assert [len(g) for g in got] == [len(w) for w in want]
    assert got == want


def test_stream_device_8k_ans_matches_oracle(jxg_mod):
    import torch

    from jxg.synth import synth_rgb8_device

    g = GOLD["8k_d1_ans"]
    t = synth_rgb8_device(g["width"], g["height"], g["seed"])
    torch.cuda.synchronize()
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS) as enc:
        for _ in range(6):
            enc.submit_device(t.data_ptr(), g["width"], g["height"])
        outs = [enc.receive() for _ in range(6)]
        st = enc.stats()
    del t
    for data in outs:
        assert hashlib.sha256(data).hexdigest() == g["sha256"]
    assert st["bytes"] == g["bytes"]


def test_stream_many_small_frames_ans(jxg_mod):
    """Small frames run the deepest pipeline (12 lanes, codes joined three
    submits later, three helpers at once): 30 frames, receives only once more
    than 14 are pending, so lanes are recycled by submit itself."""
    from jxg.synth import natural_rgb8, synth_rgb8

    frames = [(natural_rgb8 if i % 3 == 0 else synth_rgb8)(320 + 16 * (i % 5), 240 + 8 * (i % 4), 300 + i)
              for i in range(30)]
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS) as enc:
        want = [enc.encode(f) for f in frames]
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS) as enc:
        got = []
        for f in frames:
            enc.submit(f)
            while enc.pending() > 14:
                got.append(enc.receive())
        while enc.pending():
            got.append(enc.receive())
    assert got == want


def test_batch_ans_equals_single_and_refuses_pending(jxg_mod):
    """jxg_encode_batch_rgb8 runs through the streaming pipeline: its outputs
    equal one-at-a-time encodes (ANS, 20 frames, so completions interleave
    with submits), and it refuses while streamed frames are pending."""
    from jxg.synth import natural_rgb8, synth_rgb8

    frames = [(natural_rgb8 if i % 2 else synth_rgb8)(480, 272, 700 + i) for i in range(20)]
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS) as enc:
        want = [enc.encode(f) for f in frames]
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS) as enc:
        assert enc.encode_batch(frames) == want
        enc.submit(frames[0])
        with pytest.raises(jxg_mod.JxgError):
            enc.encode_batch(frames[:2])
        assert enc.receive() == want[0]
        assert enc.encode_batch(frames[:3]) == want[:3]
        assert enc.pending() == 0


def test_mixed_stream_equals_single(jxg_mod):
    """Small ANS frames of mixed sizes through the pipeline: 41 frames (not a
    multiple of the depth), host and device inputs, a 4K frame (135 groups)
    in the middle, receives interleaved -- every codestream equals the
    one-at-a-time encode's."""
    import torch

    from jxg.synth import natural_rgb8, synth_rgb8

    sizes = [(640, 480), (1920, 1080), (333, 250), (800, 600)]
    frames = [(natural_rgb8 if i % 3 else synth_rgb8)(*sizes[i % 4], 900 + i) for i in range(41)]
    frames[17] = synth_rgb8(3840, 2160, 77)
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS) as enc:
        want = [enc.encode(f) for f in frames]
    dev = [torch.from_numpy(f).cuda() if i % 2 else None for i, f in enumerate(frames)]
    torch.cuda.synchronize()
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_ANS) as enc:
        got = []
        for i, f in enumerate(frames):
            if dev[i] is None:
                enc.submit(f)
            else:
                h, w, _ = f.shape
                enc.submit_device(dev[i].data_ptr(), w, h)
            while enc.pending() > 30:
                got.append(enc.receive())
            if i == 5:
                got.append(enc.receive())
        while enc.pending():
            got.append(enc.receive())
        # one-at-a-time on the same context afterwards
        assert enc.encode(frames[1]) == want[1]
    assert [len(g) for g in got] == [len(w) for w in want]
    assert got == want
