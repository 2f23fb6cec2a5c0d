"""The XCD-aware tile order of front_kernel / aq_kernel (csrc/jxg_front.hip,
csrc/jxg_aq.hip), restated: a 1-D grid of 8 x chunk workgroups, workgroup w
runs on XCD w % 8 and takes tile (w % 8) chunk + w / 8 of the raster order.
Every tile is encoded exactly once, the idle workgroups are only the tail of
the last XCDs' chunks, and every XCD holds at most chunk = ceil(N / 8) tiles --
the column-strip split it replaced gave a 1080p frame's 510 tiles 68 to each of
seven XCDs (64 workgroup slots each: two rounds)."""
import pytest


def order(tiles_x, tiles_y):
    n = tiles_x * tiles_y
    chunk = (n + 7) >> 3
    out, per_xcd = [], [0] * 8
    for w in range(8 * chunk):
        j, x = w >> 3, w & 7
        tile = x * chunk + j
        if j >= chunk or tile >= n:
            continue
        out.append((tile % tiles_x, tile // tiles_x))
        per_xcd[x] += 1
    return n, chunk, out, per_xcd


@pytest.mark.parametrize("w,h", [(1, 1), (9, 7), (512, 512), (1920, 1080), (3840, 2160),
                                 (7680, 4320), (16384, 16384), (600, 300), (1100, 700)])
def test_every_tile_once_and_balanced(w, h):
    tiles_x, tiles_y = -(-w // 64), -(-h // 64)
    n, chunk, out, per_xcd = order(tiles_x, tiles_y)
    assert sorted(out) == sorted((x, y) for y in range(tiles_y) for x in range(tiles_x))
    assert max(per_xcd) <= chunk and sum(per_xcd) == n
    # only the last XCDs run short
    assert all(per_xcd[i] == chunk for i in range(n // chunk))


def test_1080p_fits_one_round():
    n, chunk, _, per_xcd = order(30, 17)
    assert n == 510 and max(per_xcd) == 64  # 64 workgroup slots per XCD (2 per CU)
