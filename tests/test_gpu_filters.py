"""GPU parity of the restoration-filter path (JXG_FLAG_GABORISH / JXG_FLAG_EPF,
cjxl --gaborish / --epf): the front kernel's in-place inverse
Gaborish of the LDS tile (csrc/jxg_front.hip gab_ring / gab_sweep) and the
frame header / EPF tree the host writes must equal the oracle
(oracle/xyb.c jxo_gab_inverse, oracle/encode.c) byte for byte, through every
entry point that writes headers: one-at-a-time, streamed, sharded (the payload
heads carry the loop-filter code) and the CLI."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GAB, EPF = 1, 2


def _flags(jxg_mod, filters, ans=False):
    return ((jxg_mod.FLAG_GABORISH if filters & GAB else 0) |
            (jxg_mod.FLAG_EPF if filters & EPF else 0) | (jxg_mod.FLAG_ANS if ans else 0))


# (width, height, distance, effort, proposals, filters, ans): tile and frame
# edges (1x1, 9x7, widths/heights that are not multiples of 8 or 64), every
# EPF iteration count, hooks P/F on the filtered tile
CASES = [
    (64, 64, 1.0, 7, 0, GAB, False),
    (1, 1, 1.0, 7, 3, GAB | EPF, False),
    (9, 7, 3.0, 7, 3, GAB, True),
    (200, 136, 1.0, 7, 3, GAB | EPF, True),
    (517, 389, 2.0, 7, 0, GAB | EPF, False),
    (300, 200, 6.0, 5, 1, EPF, False),
    (777, 333, 0.5, 7, 2, GAB, True),
    (130, 1100, 1.0, 4, 0, GAB, False),
    (1920, 1080, 1.0, 7, 0, GAB | EPF, True),
]


@pytest.mark.parametrize("w,h,d,e,p,filters,ans", CASES)
def test_filtered_encode_matches_oracle(jxg_mod, oracle, decoder, w, h, d, e, p, filters, ans):
    from jxg.synth import natural_rgb8, synth_rgb8

    img = (natural_rgb8 if w * h > 100000 else synth_rgb8)(w, h, w * 5 + h)
    flags = _flags(jxg_mod, filters, ans) | jxg_mod.FLAG_KEEP_MAPS
    with jxg_mod.Encoder(distance=d, effort=e, proposals=p, flags=flags) as enc:
        got = enc.encode(img)
        st = enc.stats()
    ref = oracle.encode(img, d, e, p, 1 if ans else 0, filters)
    assert np.array_equal(st["acs"], ref.acs)
    assert np.array_equal(st["qf"], ref.qf)
    assert np.array_equal(st["dc"], ref.dc)
    assert np.array_equal(st["ac"], ref.ac)
    if p:
        assert np.array_equal(st["homog"].view(np.uint32), ref.homog.view(np.uint32))
    assert got == ref.bytes
    if w * h <= 300 * 200:
        dec = decoder.decode(got)
        assert dec.gab == bool(filters & GAB)
        assert (dec.epf_iters > 0) == bool(filters & EPF)


def test_gaborish_changes_the_encode(jxg_mod):
    """The filter is live: the inverse Gaborish changes the coefficients."""
    from jxg.synth import natural_rgb8

    img = natural_rgb8(640, 480, 2)
    with jxg_mod.Encoder(distance=1.0, effort=7) as enc:
        a = enc.encode(img)
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAG_GABORISH) as enc:
        b = enc.encode(img)
    assert a != b and len(b) > len(a)


def test_filtered_stream_equals_one_at_a_time(jxg_mod):
    from jxg.synth import natural_rgb8, synth_rgb8

    frames = [natural_rgb8(1024, 768, 1), synth_rgb8(700, 500, 2), natural_rgb8(1920, 1080, 3),
              synth_rgb8(64, 64, 4)] * 2
    flags = _flags(jxg_mod, GAB | EPF, True)
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=flags) as enc:
        ref = [enc.encode(f) for f in frames]
        got = []
        for f in frames:
            enc.submit(f)
        while enc.pending():
            got.append(enc.receive())
    assert got == ref


@pytest.mark.parametrize("world", [2, 3])
def test_filtered_sharded_equals_single(jxg_mod, world):
    """Prefix-coded shards assemble to the single-GPU bytes: the loop-filter
    code travels in the payload heads (word 2, high half)."""
    from test_gpu_shard import sharded_encode

    from jxg.synth import natural_rgb8

    img = natural_rgb8(1500, 900, 7)
    flags = _flags(jxg_mod, GAB | EPF)
    with jxg_mod.Encoder(distance=2.0, effort=7, flags=flags) as enc:
        ref = enc.encode(img)
    assert sharded_encode(jxg_mod, img, world, 2.0, 7, 0, flags=flags) == ref


def test_cli_filter_flags(jxg_mod, oracle, tmp_path):
    from jxg.synth import natural_rgb8

    img = natural_rgb8(333, 222, 8)
    src = tmp_path / "in.ppm"
    src.write_bytes(b"P6 333 222 255\n" + img.tobytes())
    exe = os.path.join(os.path.dirname(jxg_mod.__file__), "jxg_cjxl")
    out = tmp_path / "out.jxl"
    r = subprocess.run([exe, str(src), str(out), "--distance=2.0", "--effort=7",
                        "--gaborish=1", "--epf=-1"], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr
    # (the CLI's defaults: ANS and the masking quant field besides the filters)
    assert out.read_bytes() == oracle.encode(img, 2.0, 7, 0, 1, GAB | EPF | 4).bytes
    r = subprocess.run([exe, str(src), str(out), "--epf=2"], capture_output=True, timeout=120)
    assert r.returncode == 1


def test_filtered_ans_shards_decode_to_single_image(jxg_mod, decoder):
    """ANS shards (one HF preset per rank, version-2 payload heads) with both
    filters: the assembled frame header carries the loop filters, and the
    codestream decodes (Gaborish + EPF applied) to exactly the single-GPU image."""
    from test_gpu_shard import _same_image, sharded_encode

    from jxg.synth import natural_rgb8

    img = natural_rgb8(1200, 700, 19)
    flags = _flags(jxg_mod, GAB | EPF, True)
    with jxg_mod.Encoder(distance=2.0, effort=7, flags=flags) as enc:
        ref = enc.encode(img)
    got = sharded_encode(jxg_mod, img, 3, 2.0, 7, 0, flags=flags)
    dr, dg = decoder.decode(ref), decoder.decode(got)
    assert dg.npresets == 3 and dr.npresets == 1
    assert dg.gab and dr.gab and dg.epf_iters == dr.epf_iters == 2
    _same_image(dr, dg)
