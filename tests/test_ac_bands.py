"""ac_hist's band record layout (csrc/jxg_ac.hip rec_index, CPU restatement):
a pass group's token stream is its four bands' streams in order, band j's
records at [j * kBandTokStride, ...); the coders map stream position k to its
record slot.  Every band-count pattern, empty bands included (partial groups:
a 64-px-tall frame has one non-empty band), must give the concatenation."""
import itertools

import pytest

K_BAND_TOK_STRIDE = 256 * 3 * 64  # jxg_kernels.h kBandTokStride


def rec_index(bt, k):
    j = lo = cum = 0
    for i in range(3):
        cum += bt[i]
        past = k >= cum
        lo = cum if past else lo
        j += 1 if past else 0
    return j * K_BAND_TOK_STRIDE + (k - lo)


@pytest.mark.parametrize("bt", list(itertools.product((0, 1, 7, 64), repeat=4)))
def test_rec_index_concatenates_bands(bt):
    want = [j * K_BAND_TOK_STRIDE + i for j in range(4) for i in range(bt[j])]
    assert [rec_index(bt, k) for k in range(sum(bt))] == want
