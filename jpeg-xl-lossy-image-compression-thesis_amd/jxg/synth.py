"""Deterministic, integer-only synthetic RGB8 generator.

``synth_rgb8(w, h, seed)`` splits the frame into 64x64 tiles; splitmix64 of
(seed ^ tile index) picks one of {flat, horizontal gradient, vertical
gradient, horizontal stripes, vertical stripes, diagonal checker, quadrant
edge, uniform noise, smooth-plus-noise} and its two colours; per-pixel noise is
one splitmix64(seed, x, y) whose low three bytes feed R, G, B.  One flat tile in
five is all-black, which drives the thesis selector's 0/0 -> NaN -> DCT path
(proposals/combined.diff:209-211).  Seeds: 0x4A584C00 + config index.
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0x4A584C00


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    z = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth_rgb8(w: int, h: int, seed: int) -> np.ndarray:
    """Returns an (h, w, 3) uint8 array."""
    with np.errstate(over="ignore"):
        return _synth(w, h, seed)


def _synth(w: int, h: int, seed: int) -> np.ndarray:
    s = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
    ntx, nty = (w + 63) // 64, (h + 63) // 64
    th = _splitmix64(s ^ np.arange(ntx * nty, dtype=np.uint64)).reshape(nty, ntx)
    kind_t = (th % np.uint64(9)).astype(np.int8)
    period_t = (2 + (th >> np.uint64(56)) % np.uint64(14)).astype(np.int32)
    black_t = ((th >> np.uint64(40)) % np.uint64(5)) == 0
    ty = np.arange(h) // 64
    tx = np.arange(w) // 64
    kind = kind_t[ty][:, tx]
    period = period_t[ty][:, tx]
    ly = (np.arange(h, dtype=np.int32) % 64)[:, None]
    lx = (np.arange(w, dtype=np.int32) % 64)[None, :]
    key = (np.arange(h, dtype=np.uint64)[:, None] << np.uint64(32)) | np.arange(w, dtype=np.uint64)[None, :]
    noise64 = _splitmix64((s * np.uint64(0x100000001B3)) ^ key)
    out = np.empty((h, w, 3), dtype=np.uint8)
    cond = [kind == k for k in range(9)]
    for c in range(3):
        c0 = ((th >> np.uint64(8 + 8 * c)) & np.uint64(0xFF)).astype(np.int32)[ty][:, tx]
        c1 = ((th >> np.uint64(32 + 8 * c)) & np.uint64(0xFF)).astype(np.int32)[ty][:, tx]
        noise = ((noise64 >> np.uint64(8 * c)) & np.uint64(0xFF)).astype(np.int32)
        flat = np.where(black_t[ty][:, tx], 0, c0)
        hgrad = c0 + (c1 - c0) * lx // 63
        vgrad = c0 + (c1 - c0) * ly // 63
        hstripe = np.where((ly // period) % 2 == 0, c0, c1)
        vstripe = np.where((lx // period) % 2 == 0, c0, c1)
        checker = np.where(((lx // period + ly // period) % 2) == 0, c0, c1)
        quad = np.where((lx < 32) ^ (ly < 32), c0, c1)
        smooth = (hgrad + vgrad) // 2 + (noise % 17) - 8
        v = np.select(cond, [flat, hgrad, vgrad, hstripe, vstripe, checker, quad, noise, smooth])
        out[..., c] = np.clip(v, 0, 255)
    return out


def synth_rgb8_device(w: int, h: int, seed: int, device=0, enc=None):
    """The same frame as :func:`synth_rgb8`, generated on the GPU
    (jxg_synth_rgb8_device) into a new uint8 CUDA tensor (h, w, 3)."""
    import torch

    from . import Encoder

    t = torch.empty((h, w, 3), dtype=torch.uint8, device=torch.device("cuda", device))
    own = enc is None
    e = Encoder(device=device) if own else enc
    try:
        torch.cuda.synchronize(t.device)
        e.synth_device(t.data_ptr(), w, h, seed)
    finally:
        if own:
            e.close()
    return t


def natural_rgb8(w: int, h: int, seed: int) -> np.ndarray:
    """A photographic stand-in for rate-distortion checks: smooth colour
    fields, a dozen soft-blended discs (edges) and band-limited texture (a
    Gaussian low-pass of white noise, not aligned to any block grid).
    Deterministic for a given numpy (PCG64 + FFT).  Returns (h, w, 3) uint8."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.zeros((h, w, 3))
    for c in range(3):
        img[..., c] = 128 + 60 * np.sin(x / (17 + 7 * c)) * np.cos(y / (23 + 5 * c))
    for _ in range(12):
        cx, cy, r = rng.uniform(0, w), rng.uniform(0, h), rng.uniform(8, w / 4)
        col = rng.uniform(0, 255, 3)
        m = (x - cx) ** 2 + (y - cy) ** 2 < r * r
        img[m] = 0.6 * img[m] + 0.4 * col
    wn = rng.normal(0, 1, (h, w, 3))
    fy = np.fft.fftfreq(h)[:, None]
    fx = np.fft.fftfreq(w)[None, :]
    lp = np.exp(-(fx ** 2 + fy ** 2) / (2 * 0.06 ** 2))[..., None]
    tex = np.real(np.fft.ifft2(np.fft.fft2(wn, axes=(0, 1)) * lp, axes=(0, 1)))
    tex *= 8.0 / tex.std()
    return np.clip(img + tex, 0, 255).astype(np.uint8)


# SURVEY.md §8(d) workload shapes: (name, width, height, frames)
CONFIGS = {
    0: ("cpu512", 512, 512, 1),
    1: ("4k", 3840, 2160, 1),
    2: ("8k", 7680, 4320, 1),
    3: ("1080p_x64", 1920, 1080, 64),
    4: ("16k", 16384, 16384, 1),
}


def config_image(idx: int, frame: int = 0) -> np.ndarray:
    _, w, h, _ = CONFIGS[idx]
    return synth_rgb8(w, h, SEED_BASE + idx + frame)
