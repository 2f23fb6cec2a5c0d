"""The cjxl-argv CLI (jxg_cjxl) on its success path, as the harness calls it:
`cjxl IN OUT --distance=D --effort=E` (benchmark-jpegxl/src/docker_manager.rs:
126-136, output named {stem}-{distance}-{effort}.jxl by benchmark.rs:644-650)
on a PNG written here (zlib; rows cycle through the five PNG filter types so
the reader's unfiltering is exercised), bytes checked against the oracle."""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# oracle filters mask of cjxl's defaults: Gaborish 1 | EPF 2 | masking AQ 4
CJXL_DEFAULTS = 7


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def write_png(path, img):
    h, w, _ = img.shape
    x = img.astype(np.int32)
    raw = bytearray()
    for y in range(h):
        ft = y % 5
        cur = x[y].reshape(-1)
        prev = x[y - 1].reshape(-1) if y else np.zeros_like(cur)
        left = np.concatenate([np.zeros(3, np.int32), cur[:-3]])
        ul = np.concatenate([np.zeros(3, np.int32), prev[:-3]])
        pred = [np.zeros_like(cur), left, prev, (left + prev) // 2, _paeth(left, prev, ul)][ft]
        raw.append(ft)
        raw += ((cur - pred) & 0xFF).astype(np.uint8).tobytes()

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
                + chunk(b"IDAT", zlib.compress(bytes(raw), 6)) + chunk(b"IEND", b""))


@pytest.mark.parametrize("distance,effort", [(1.0, 7), (0.5, 5), (2.0, 4)])
def test_cjxl_png_success(jxg_mod, oracle, tmp_path, distance, effort):
    from jxg.synth import synth_rgb8

    img = synth_rgb8(333, 200, 0x4A584C07)
    src = tmp_path / "photo-a.png"
    write_png(str(src), img)
    out = tmp_path / "out" / jxg_mod.comp_image_name("photo-a", distance, effort)
    ok, msg = jxg_mod.execute_cjxl(str(src), str(out), distance, effort)
    assert ok, msg
    assert out.name == "photo-a-%s-%d.jxl" % (jxg_mod.rust_f64(distance), effort)
    # cjxl's VarDCT defaults: ANS, Gaborish, EPF by distance, masking AQ
    assert out.read_bytes() == oracle.encode(img, distance, effort, 0, 1, CJXL_DEFAULTS).bytes


def test_cjxl_plain_argv(jxg_mod, oracle, tmp_path):
    """exactly the argv of docker_manager.rs:126-136 (no extra flags)"""
    from jxg.synth import synth_rgb8

    img = synth_rgb8(64, 48, 0x4A584C08)
    src = tmp_path / "in.png"
    write_png(str(src), img)
    out = tmp_path / "in-1-7.jxl"
    p = subprocess.run([jxg_mod.CLI_PATH, str(src), str(out), "--distance=1", "--effort=7"],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    assert out.read_bytes() == oracle.encode(img, 1.0, 7, 0, 1, CJXL_DEFAULTS).bytes


def test_cjxl_flags_override_defaults(jxg_mod, oracle, tmp_path):
    """--coder=prefix --gaborish=0 --epf=0 --aq=activity: the library's
    default (unfiltered, activity AQ, prefix codes) encode; each flag alone."""
    from jxg.synth import natural_rgb8

    img = natural_rgb8(200, 136, 0x4A584C09)
    src = tmp_path / "in.png"
    write_png(str(src), img)
    out = tmp_path / "o.jxl"
    cases = [(["--coder=prefix", "--gaborish=0", "--epf=0", "--aq=activity"], 0, 0),
             (["--gaborish=0"], 1, CJXL_DEFAULTS & ~1), (["--epf=0"], 1, CJXL_DEFAULTS & ~2),
             (["--aq=activity"], 1, CJXL_DEFAULTS & ~4)]
    for extra, coder, filters in cases:
        p = subprocess.run([jxg_mod.CLI_PATH, str(src), str(out), "--distance=1.5", "--effort=7"]
                           + extra, capture_output=True, text=True)
        assert p.returncode == 0, p.stderr
        assert out.read_bytes() == oracle.encode(img, 1.5, 7, 0, coder, filters).bytes, extra
    p = subprocess.run([jxg_mod.CLI_PATH, str(src), str(out), "--aq=butteraugli"],
                       capture_output=True, text=True)
    assert p.returncode == 1


@pytest.mark.parametrize("distance,effort,proposals", [(1.0, 7, "none"), (2.0, 5, "PF"),
                                                       (0.5, 7, "F")])
def test_cli_and_c_abi_give_the_same_bytes(jxg_mod, oracle, tmp_path, distance, effort, proposals):
    """The two drop-in routes agree: the same PNG through
    `jxg_cjxl IN OUT --distance=D --effort=E [--proposals=..]` and through the
    C ABI (jxg_create with JXG_FLAGS_CJXL_DEFAULTS, jxg_encode_rgb8 -- what
    INTEGRATION.md's Rust execute_cjxl does) give identical bytes, equal to the
    oracle's encode of cjxl's defaults."""
    from jxg.synth import natural_rgb8

    img = natural_rgb8(419, 263, 11)
    src = tmp_path / "in.png"
    write_png(str(src), img)
    out = tmp_path / "cli.jxl"
    ok, msg = jxg_mod.execute_cjxl(str(src), str(out), distance, effort, proposals=proposals)
    assert ok, msg
    props = {"none": 0, "P": 1, "F": 2, "PF": 3}[proposals]
    with jxg_mod.Encoder(distance=distance, effort=effort, proposals=props,
                         flags=jxg_mod.FLAGS_CJXL_DEFAULTS) as enc:
        lib_bytes = enc.encode(img)
    assert out.read_bytes() == lib_bytes
    assert lib_bytes == oracle.encode(img, distance, effort, props, 1,
                                      jxg_mod.ORACLE_FILTERS_CJXL_DEFAULTS).bytes
