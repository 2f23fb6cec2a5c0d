"""GPU vs oracle codestreams, section by section (TOC of each): which section
differs first and at which byte, plus per-group AC token counts.  For
debugging a parity failure in one GPU call.
  python tools/diag_sections.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd")]
import torch  # noqa: F401,E402  (one HIP runtime)
import numpy as np  # noqa: E402

import jxl_decode  # noqa: E402
import oracle_ffi  # noqa: E402
import jxg  # noqa: E402
from jxg.synth import synth_rgb8  # noqa: E402


def toc(data):
    try:
        jxl_decode.decode(data, want_pixels=False)
        err = None
    except Exception as e:  # noqa: BLE001
        err = repr(e)[:200]
    return jxl_decode.LAST_TOC, err


for (w, h, ans) in ((64, 64, False), (64, 64, True), (600, 400, False), (600, 400, True),
                    (2100, 300, True)):
    img = synth_rgb8(w, h, w * 7 + h)
    flags = jxg.FLAG_KEEP_MAPS | (jxg.FLAG_ANS if ans else 0)
    with jxg.Encoder(distance=1.0, effort=7, flags=flags) as enc:
        got = enc.encode(img)
        st = enc.stats()
    ref = oracle_ffi.encode(img, 1.0, 7, 0, 1 if ans else 0, 0)
    same_maps = all(np.array_equal(st[k], getattr(ref, k)) for k in ("qf", "acs", "dc", "ac"))
    print("%dx%d %s: bytes %s (gpu %d, oracle %d), maps %s" % (
        w, h, "ans" if ans else "prefix", "EQUAL" if got == ref.bytes else "DIFFER",
        len(got), len(ref.bytes), "equal" if same_maps else "DIFFER"), flush=True)
    if got == ref.bytes:
        continue
    tg, eg = toc(got)
    tr, er = toc(ref.bytes)
    print("  decode gpu: %s | oracle: %s" % (eg or "ok", er or "ok"))
    if tg and tr:
        print("  sizes gpu    %s" % tg[1][:16])
        print("  sizes oracle %s" % tr[1][:16])
        for i, (og, sg, orr, sr) in enumerate(zip(tg[0], tg[1], tr[0], tr[1])):
            a, b = got[og:og + sg], ref.bytes[orr:orr + sr]
            if a != b:
                k = next((j for j in range(min(len(a), len(b))) if a[j] != b[j]), min(len(a), len(b)))
                print("  first differing section %d (of %d): sizes %d vs %d, first diff byte %d: gpu %s oracle %s"
                      % (i, len(tg[1]), sg, sr, k, a[k:k + 8].hex(), b[k:k + 8].hex()))
                break
