"""jxg_cjxl's PNG reader on the CPU (JXG_CJXL_DECODE_ONLY=1: the decoded
image is written as a PPM, no GPU is touched): every PNG filter type, gray /
gray+alpha / RGB / RGBA, the IDAT stream split over many chunks (and a
frame larger than the reader's 1 MB inflate window), against the image the
PNG was made from.  The harness's input format (image_reader.rs:332 reads
PNGs with image::open; execute_cjxl hands cjxl the PNG path,
docker_manager.rs:126-136)."""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd", "jxg", "jxg_cjxl")


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def png_bytes(img, ctype, pieces=1, filt=None):
    """img (H, W, ch) uint8; rows cycle through the five filters (or `filt`)"""
    h, w, ch = img.shape
    x = img.astype(np.int32).reshape(h, w * ch)
    raw = bytearray()
    for y in range(h):
        ft = y % 5 if filt is None else filt
        cur = x[y]
        prev = x[y - 1] if y else np.zeros_like(cur)
        left = np.concatenate([np.zeros(ch, np.int32), cur[:-ch]])
        ul = np.concatenate([np.zeros(ch, np.int32), prev[:-ch]])
        pred = [np.zeros_like(cur), left, prev, (left + prev) // 2, _paeth(left, prev, ul)][ft]
        raw.append(ft)
        raw += ((cur - pred) & 0xFF).astype(np.uint8).tobytes()

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    z = zlib.compress(bytes(raw), 6)
    cut = [len(z) * i // pieces for i in range(pieces + 1)]
    out = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0))
    for i in range(pieces):
        out += chunk(b"IDAT", z[cut[i]:cut[i + 1]])
    return out + chunk(b"IEND", b"")


def decode(tmp_path, data):
    src, dst = tmp_path / "in.png", tmp_path / "out.ppm"
    src.write_bytes(data)
    p = subprocess.run([CLI, str(src), str(dst)], capture_output=True, text=True,
                       env=dict(os.environ, JXG_CJXL_DECODE_ONLY="1"))
    return p, (dst.read_bytes() if p.returncode == 0 else None)


def ppm_image(d):
    parts = d.split(b"\n", 3)
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], np.uint8).reshape(h, w, 3)


@pytest.fixture(scope="module", autouse=True)
def _built():
    if not os.path.exists(CLI):
        pytest.skip("jxg_cjxl not built")


@pytest.mark.parametrize("ctype,ch", [(2, 3), (6, 4), (0, 1), (4, 2)])
@pytest.mark.parametrize("pieces", [1, 7])
def test_png_layouts_and_filters(tmp_path, ctype, ch, pieces):
    rng = np.random.default_rng(ctype * 10 + pieces)
    img = rng.integers(0, 256, (37, 53, ch), dtype=np.uint8)
    img[:, :20] = img[:, :1]  # runs, so the filters differ from plain bytes
    p, d = decode(tmp_path, png_bytes(img, ctype, pieces))
    assert p.returncode == 0, p.stderr
    rgb = img[..., :3] if ch >= 3 else np.repeat(img[..., :1], 3, axis=2)
    assert np.array_equal(ppm_image(d), rgb)


@pytest.mark.parametrize("filt", [0, 1, 2, 3, 4])
def test_png_larger_than_the_inflate_window(tmp_path, filt):
    """rows straddle the reader's 1 MB inflate pieces (a 1500 x 400 RGB frame
    is 1.8 MB of filtered rows)"""
    rng = np.random.default_rng(filt)
    img = rng.integers(0, 256, (400, 1500, 3), dtype=np.uint8)
    p, d = decode(tmp_path, png_bytes(img, 2, 3, filt))
    assert p.returncode == 0, p.stderr
    assert np.array_equal(ppm_image(d), img)


def test_png_errors(tmp_path):
    img = np.zeros((8, 8, 3), np.uint8)
    good = png_bytes(img, 2)
    p, _ = decode(tmp_path, good[:60])  # IDAT cut short
    assert p.returncode == 1 and p.stderr
    p, _ = decode(tmp_path, b"not a png at all")
    assert p.returncode == 1 and "not a PNG" in p.stderr
    bad = bytearray(png_bytes(img, 2))
    p, _ = decode(tmp_path, bytes(bad[:-12]))  # no IEND: still decodes
    assert p.returncode == 0
