"""The streaming pipeline's shape (csrc/jxg_host.cpp pipe_shape), restated:
lanes x frames per lane from the pass groups and 64x64 tiles of a frame or
shard, and jxg_pipeline_depth = (lanes - 1) x batch + 1.  DESIGN.md §3.7's
table (8K 7 x 1, 4K 12 x 1, 1080p 12 x 4, a rank's eighth of 8K 10 x 4) and
the lane cap of jxg_set_pipeline_lanes.  (The GPU tests check the library's
own jxg_pipeline_depth against the refusal it enforces.)"""
import pytest

MAX_LANES, MIN_LANES, CHAIN_GROUPS, MAX_BATCH, BATCH_TILES = 12, 4, 3570, 4, 1280


def pipe_shape(ngroups, ntiles, cap=0, queues=16):
    want = (CHAIN_GROUPS + ngroups - 1) // max(1, ngroups)
    lmax = max(2, min(MAX_LANES, queues - 1))
    if cap:
        lmax = min(lmax, cap)
    kt = MAX_BATCH if ntiles <= BATCH_TILES else 1
    k = min(kt, max(1, (want + lmax - 1) // lmax))
    lanes = min(lmax, max(min(MIN_LANES, lmax), (want + k - 1) // k))
    return lanes, k


def frame(w, h):
    groups = ((w + 255) // 256) * ((h + 255) // 256)
    tiles = ((w + 63) // 64) * ((h + 63) // 64)
    return groups, tiles


@pytest.mark.parametrize("w,h,shape", [(7680, 4320, (7, 1)), (3840, 2160, (12, 1)),
                                       (1920, 1080, (12, 4)), (7680, 544, (10, 4)),
                                       (7680, 1088, (12, 1)), (16384, 16384, (4, 1))])
def test_documented_shapes(w, h, shape):
    assert pipe_shape(*frame(w, h)) == shape


def test_depth_and_caps():
    lanes, k = pipe_shape(*frame(7680, 544))
    assert (lanes - 1) * k + 1 == 37  # the 1/8-slice probe's depth (profiles/r04l)
    assert pipe_shape(*frame(7680, 544), cap=2) == (2, 4)
    assert pipe_shape(*frame(7680, 544), cap=1) == (1, 4)
    assert pipe_shape(*frame(1920, 1080), queues=4) == (3, 4)  # HIP's default 4 queues
