"""Edge cases of the drop-in encode on the GPU (through the C ABI): frames the
library must refuse (empty, past the 2^18 side limit, a row stride shorter
than the row) leave the context usable, and the next frames still equal the
oracle's bytes -- 1-pixel-wide and 1-pixel-high strips, a frame that is a
single partial 8x8 block, and sides one past a group / tile boundary at the
headline preset (cjxl's defaults)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# the oracle's options for cjxl's defaults: ANS (coder 1), Gaborish | EPF |
# masking AQ (tests/test_gpu_filters.py, oracle/oracle_ffi.py)
CJXL = 1 | 2 | 4


def _refused(jxg_mod, enc, w, h, stride):
    lib = jxg_mod.load()
    buf = jxg_mod._Buffer()
    img = np.zeros(max(1, stride * max(h, 1)), np.uint8)
    st = lib.jxg_encode_rgb8(enc._ctx, img.ctypes.data_as(ctypes.c_void_p), w, h, stride,
                             ctypes.byref(buf))
    return st == -1


@pytest.mark.parametrize("flags_name", ["plain", "cjxl"])
def test_refused_frames_leave_the_context_usable(jxg_mod, oracle, flags_name):
    from jxg.synth import synth_rgb8

    flags = jxg_mod.FLAGS_CJXL_DEFAULTS if flags_name == "cjxl" else 0
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=flags) as enc:
        assert _refused(jxg_mod, enc, 0, 8, 24)
        assert _refused(jxg_mod, enc, 8, 0, 24)
        assert _refused(jxg_mod, enc, (1 << 18) + 1, 1, 3 * ((1 << 18) + 1))
        assert _refused(jxg_mod, enc, 16, 16, 47)  # stride < 3 * width
        img = synth_rgb8(67, 41, 0x4A584C77)
        got = enc.encode(img)
    ref = oracle.encode(img, 1.0, 7, 0, *((1, CJXL) if flags_name == "cjxl" else (0, 0)))
    assert got == ref.bytes


# strips and boundary sizes at cjxl's defaults (Gaborish + EPF + masking AQ,
# ANS): the AQ halo and the inverse Gaborish clamp at every edge
SIZES = [(1, 300), (300, 1), (5, 3), (257, 65), (65, 257), (2049, 9)]


@pytest.mark.parametrize("w,h", SIZES)
def test_edge_sizes_at_cjxl_defaults(jxg_mod, oracle, decoder, w, h):
    from jxg.synth import synth_rgb8

    img = synth_rgb8(w, h, 0x4A584C10 + 3 * w + h)
    with jxg_mod.Encoder(distance=1.0, effort=7, flags=jxg_mod.FLAGS_CJXL_DEFAULTS) as enc:
        got = enc.encode(img)
    ref = oracle.encode(img, 1.0, 7, 0, 1, CJXL)
    assert got == ref.bytes
    dec = decoder.decode(got)
    assert dec.rgb.shape[:2] == (h, w)
