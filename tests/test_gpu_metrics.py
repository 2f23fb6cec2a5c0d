"""GPU parity of the decode-side quality kernels (jxg_metrics.hip through the
C ABI jxg_compare_rgb8 / _device) against oracle/metrics.py: SSE, MSE and
PSNR bit-exact (the reference's f64 sum is exact, image_reader.rs:569-606);
SSIM within a relative 1e-12 (per-window values use the oracle's op order,
only the final mean's summation order differs)."""
import math

import numpy as np
import pytest

import metrics

pytestmark = pytest.mark.gpu


def _pair(h, w, seed, noise=12):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    b = np.clip(a.astype(np.int32) + rng.integers(-noise, noise + 1, a.shape), 0, 255)
    return a, b.astype(np.uint8)


@pytest.fixture(scope="module")
def enc(jxg_mod):
    with jxg_mod.Encoder(distance=1.0, effort=7) as e:
        yield e


@pytest.mark.parametrize("h,w", [(1, 1), (10, 10), (11, 11), (13, 37), (64, 64), (100, 257),
                                 (270, 481)])
def test_metrics_match_oracle(enc, h, w):
    a, b = _pair(h, w, h * 1000 + w)
    q = enc.compare(a, b)
    assert q["sse"] == metrics.sse(a, b)
    assert q["samples"] == a.size
    assert q["mse"] == metrics.mse(a, b)
    assert q["psnr"] == metrics.psnr(metrics.mse(a, b))
    ref = metrics.ssim(a, b)
    if math.isnan(ref):
        assert math.isnan(q["ssim"])
    else:
        assert q["ssim"] == pytest.approx(ref, rel=1e-12, abs=1e-15)


def test_identical_images(enc):
    a, _ = _pair(40, 50, 5)
    q = enc.compare(a, a)
    assert q["sse"] == 0 and q["mse"] == 0.0 and q["psnr"] == math.inf and q["ssim"] == 1.0


def test_extreme_difference(enc):
    a = np.zeros((33, 35, 3), np.uint8)
    q = enc.compare(a, a + 255)
    assert q["mse"] == 65025.0 and q["psnr"] == 0.0
    assert q["ssim"] == pytest.approx(metrics.ssim(a, a + 255), rel=1e-12)


def test_device_pointers_and_strides(enc):
    torch = pytest.importorskip("torch")
    a, b = _pair(123, 77, 11)
    pad = np.zeros((123, 77 * 3 + 5), np.uint8)
    pa, pb = pad.copy(), pad.copy()
    pa[:, :231] = a.reshape(123, -1)
    pb[:, :231] = b.reshape(123, -1)
    da = torch.from_numpy(pa).cuda()
    db = torch.from_numpy(pb).cuda()
    torch.cuda.synchronize()
    q = enc.compare_device(da.data_ptr(), db.data_ptr(), 77, 123, 236, 236)
    assert q["sse"] == metrics.sse(a, b) and q["mse"] == metrics.mse(a, b)
    assert q["ssim"] == pytest.approx(metrics.ssim(a, b), rel=1e-12)


def test_full_8k_frame_sse(enc, jxg_mod):
    from jxg.synth import synth_rgb8
    a = synth_rgb8(7680, 4320, 0x4A584C02)
    b = a.copy()
    b[::7, ::3, 1] ^= 0x5A
    q = enc.compare(a, b, ssim=False)
    assert q["sse"] == metrics.sse(a, b) and q["mse"] == metrics.mse(a, b)
    assert math.isnan(q["ssim"])


def test_encode_decode_psnr(enc, jxg_mod, decoder):
    """End to end: GPU encode -> oracle decoder -> GPU PSNR == host PSNR, with
    quality floors at d1 e7 (tests/test_oracle_rd.py has the RD checks)."""
    from jxg.synth import natural_rgb8, synth_rgb8
    img = synth_rgb8(200, 136, 0x4A584C00)
    dec = decoder.decode(enc.encode(img)).rgb
    q = enc.compare(img, dec)
    assert q["mse"] == jxg_mod.calculate_mse(img, dec) or q["mse"] == metrics.mse(img, dec)
    assert q["psnr"] == metrics.psnr(metrics.mse(img, dec))
    # the synthetic mix holds full-range RGB noise tiles (their chroma is
    # quantized coarsely at d1), so the floor is modest
    assert q["psnr"] >= 24.0, q["psnr"]
    nat = natural_rgb8(256, 256, 3)
    qn = enc.compare(nat, decoder.decode(enc.encode(nat)).rgb)
    assert qn["psnr"] >= 38.0, qn["psnr"]


def test_harness_compare_to_orig(enc, decoder, tmp_path):
    from jxg import harness
    from jxg.synth import synth_rgb8
    img = synth_rgb8(128, 96, 0x4A584C05)
    data = enc.encode(img)
    dec = decoder.decode(data).rgb
    res = harness.compare_to_orig(enc, "s.png", img, 40000, "s-1-7.jxl", dec, len(data), 1.0, 7,
                                  result_file=str(tmp_path / "comparisons.csv"))
    assert res.mse == metrics.mse(img, dec) and res.comp_raw_size == 128 * 96 * 3
    assert res.raw_file_size_ratio == 128 * 96 * 3 / len(data)
    assert harness.read_csv(str(tmp_path / "comparisons.csv"))[0].psnr == res.psnr
