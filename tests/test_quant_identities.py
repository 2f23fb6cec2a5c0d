"""The float identities the round-5 quantization code relies on
(csrc/jxg_front.hip quant_lane / quant_xb, csrc/jxg_merge.hip quant_pass),
checked in IEEE single precision on the CPU (numpy float32 arithmetic rounds
to nearest like the GPU's VALU; no contraction is involved):

* non-zero counts from exponent sums: a quantized magnitude qf is an
  integer-valued float in [0, 32767]; a zero has biased exponent E = 0, a
  non-zero E = 127 + floor(log2 qf) in [127, 141], so for <= 8 values
  sum(E) / 127 (integer division) is their non-zero count and
  2 sum(E) - 250 nz is the rate sum over non-zeros of 2 + 2 bitlen(qf)
  (oracle/front.c jxo_quantize_block).  Sixteen values can break the division
  -- the merge stage splits a 16-row item into two sums of eight;
* the signed error: with sq = copysign(qf, vq), (vq - sq) * sd is +-((|vq| -
  qf) * sd) exactly, so its square -- the only use -- is the oracle's;
* the tabulated AdjustQuantBias: adj(q) for q < 256 is the same float
  expression the kernels evaluated per coefficient before;
* the signed value: (int)copysign(qf, vq) == (vq < 0 ? -(int)qf : (int)qf),
  and v_cvt_pk_i16_i32's pair packing equals the mask / shift form at
  |q| <= 32767.
"""
import numpy as np
import pytest

f32 = np.float32


def quantize(vq):
    """qf of the kernels: |vq| < 0.58 -> 0 else floor(min(|vq|, 32767) + 0.5), in f32"""
    a = np.abs(vq).astype(f32)
    q = np.floor(np.minimum(a, f32(32767.0)) + f32(0.5)).astype(f32)
    return np.where(a < f32(0.58), f32(0.0), q).astype(f32)


def biased_exp(qf):
    return (qf.astype(f32).view(np.uint32) >> 23).astype(np.int64)


def bitlen(v):
    v = np.asarray(v, dtype=np.int64)
    out = np.zeros_like(v)
    for b in range(16):
        out = np.where(v >> b != 0, b + 1, out)
    return out


@pytest.mark.parametrize("n", [1, 2, 7, 8])
def test_nonzero_count_from_exponent_sum(n):
    rng = np.random.default_rng(100 + n)
    # magnitudes across the whole range, many zeros, the extremes included
    vals = rng.integers(0, 32768, size=(20000, n))
    vals[rng.random(vals.shape) < 0.4] = 0
    vals[0, :] = 32767
    vals[1, :] = 1
    qf = vals.astype(f32)
    E = biased_exp(qf)
    nz = (vals != 0).sum(axis=1)
    assert np.array_equal(E.sum(axis=1) // 127, nz)
    rate = np.where(vals != 0, 2 + 2 * bitlen(vals), 0).sum(axis=1)
    assert np.array_equal(2 * E.sum(axis=1) - 250 * nz, rate)


def test_sixteen_values_need_two_sums():
    vals = np.array([32767] * 10 + [0] * 6)
    E = biased_exp(vals.astype(f32))
    assert E.sum() // 127 != 10  # one sum over 16 miscounts
    assert E[:8].sum() // 127 + E[8:].sum() // 127 == 10  # the merge stage's split


def test_signed_error_is_plus_minus_the_oracle_error():
    rng = np.random.default_rng(7)
    vq = (rng.standard_normal(200000) * rng.choice([0.3, 3.0, 300.0, 3e4], 200000)).astype(f32)
    vq[:4] = [f32(0.0), f32(-0.0), f32(0.58), f32(-0.57999)]
    sd = rng.uniform(0.01, 4.0, vq.size).astype(f32)
    qf = quantize(vq)
    sq = np.copysign(qf, vq).astype(f32)
    e_oracle = ((np.abs(vq) - qf).astype(f32) * sd).astype(f32)
    e_signed = ((vq - sq).astype(f32) * sd).astype(f32)
    assert np.array_equal(np.abs(e_signed), np.abs(e_oracle))
    assert np.array_equal((e_signed * e_signed).astype(f32), (e_oracle * e_oracle).astype(f32))
    # the signed quantized value and its int16 pair packing
    q_old = np.where(vq < 0, -qf.astype(np.int64), qf.astype(np.int64))
    q_new = sq.astype(np.int64)  # C's (int) truncation; sq is integer-valued
    assert np.array_equal(q_old, q_new)
    lo, hi = q_new[0::2], q_new[1::2]
    mask_form = (lo & 0xFFFF) | ((hi & 0xFFFF) << 16)
    sat = lambda v: np.clip(v, -32768, 32767) & 0xFFFF  # v_cvt_pk_i16_i32
    assert np.array_equal(mask_form, sat(lo) | (sat(hi) << 16))


def test_bias_table_is_the_per_coefficient_expression():
    kbias1 = f32(1.0) - f32(0.07005449891748593)
    for q in range(256):
        qf = f32(q)
        per_coef = f32(0.0) if q == 0 else (kbias1 if q == 1 else f32(qf - f32(0.145) / qf))
        table = f32(0.0) if q == 0 else (kbias1 if q == 1 else f32(f32(q) - f32(0.145) / f32(q)))
        assert per_coef.view(np.uint32) == table.view(np.uint32)
