"""CPU restatement of jxg_bigvb.hip's breadth-first Lee DCT (lee_batch: every
split stage over the whole vector, then every recombination stage) against
the oracle's recursive one: the same float32 ops in another order, so the
results must be bit-identical for the 64 / 128 / 256-point transforms of the
128 / 256 px merge levels (the kernel's index math, checked without a GPU)."""
import math

import numpy as np
import pytest


def lee_c(N):
    l = int(math.log2(N))
    return [np.float32(1.0 / (2.0 * math.cos(math.pi * (2 * i + 1) / (2.0 * N)))) for i in range(N // 2)]


def lee_breadth_first(x):
    """the kernel's lee_batch for one vector (float32 numpy scalars)"""
    N = len(x)
    L = int(math.log2(N))
    src = [np.float32(v) for v in x]
    for d in range(L):
        n = N >> d
        h = n >> 1
        c = lee_c(n)
        dst = [None] * N
        for i in range(N // 2):
            seg, j = divmod(i, h)
            s0 = seg * n
            a, b = src[s0 + j], src[s0 + n - 1 - j]
            dst[s0 + j] = np.float32(a + b)
            dst[s0 + h + j] = np.float32(np.float32(a - b) * c[j])
        src = dst
    for d in range(L - 2, -1, -1):
        n = N >> d
        h = n >> 1
        dst = [None] * N
        for o in range(N):
            seg, k = divmod(o, n)
            s0 = seg * n
            if k % 2 == 0:
                dst[o] = src[s0 + k // 2]
            elif k < n - 1:
                dst[o] = np.float32(src[s0 + h + k // 2] + src[s0 + h + k // 2 + 1])
            else:
                dst[o] = src[s0 + n - 1]
        src = dst
    s = [np.float32(1.0 / N)] + [np.float32(math.sqrt(2.0) / N)] * (N - 1)
    return np.array([np.float32(v * sc) for v, sc in zip(src, s)], dtype=np.float32)


@pytest.mark.parametrize("N", [2, 8, 64, 128, 256])
def test_breadth_first_lee_is_bit_identical(oracle, N):
    rng = np.random.default_rng(N)
    for _ in range(3):
        x = rng.uniform(-200, 200, N).astype(np.float32)
        assert np.array_equal(lee_breadth_first(x), oracle.dct(x))
