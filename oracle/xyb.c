/*
 * xyb.c -- ORACLE (test infrastructure).  sRGB8 -> linear -> XYB ("opsin")
 * restatement.  [ext] libjxl ToXYB (lib/jxl/enc_xyb.cc, not in
 * /root/reference): opsin absorbance matrix + bias, cube root, minus
 * cbrt(bias), X=(L-M)/2, Y=(L+M)/2, B=S.  Parity vs libjxl unpinned; the GPU
 * kernel must match this bit-for-bit (fixed op order, -ffp-contract=off,
 * deterministic in-house cube root).
 */
#include <math.h>
#include <string.h>

#include "jxo_internal.h"

/* deterministic cube root, multiply/fma only (no division): bit-hack seed of
 * x^(-1/3), three Newton steps r <- r + (r*(1 - x*r^3))/3 written with
 * explicit fmaf, then cbrt = x*r*r.  Every op is a correctly rounded IEEE
 * mul/fma, so the GPU (jxg_device.h cbrt_det) reproduces it bit for bit.
 * Max relative error vs cbrt() ~1e-7 over the opsin range [bias, 1.1]. */
float jxo_cbrtf(float x) {
  if (!(x > 0.0f)) return 0.0f;
  uint32_t i;
  memcpy(&i, &x, 4);
  i = 0x54a2fa8cu - i / 3u;
  float r;
  memcpy(&r, &i, 4);
  for (int it = 0; it < 3; it++) {
    const float r3 = (r * r) * r;
    const float e = fmaf(-x, r3, 1.0f);
    r = fmaf(r * e, 0x1.555556p-2f, r);
  }
  return (x * r) * r;
}

void jxo_srgb_lut(float lut[256]) {
  for (int u = 0; u < 256; u++) {
    double v = u / 255.0;
    double l = v <= 0.04045 ? v / 12.92 : pow((v + 0.055) / 1.055, 2.4);
    lut[u] = (float)l;
  }
}

void jxo_pixel_xyb(const float lut[256], const float cb, uint8_t r8, uint8_t g8,
                   uint8_t b8, float* X, float* Y, float* B) {
  const float r = lut[r8], g = lut[g8], b = lut[b8];
  float m0 = ((JXO_M00 * r + JXO_M01 * g) + JXO_M02 * b) + JXO_BIAS;
  float m1 = ((JXO_M10 * r + JXO_M11 * g) + JXO_M12 * b) + JXO_BIAS;
  float m2 = ((JXO_M20 * r + JXO_M21 * g) + JXO_M22 * b) + JXO_BIAS;
  m0 = jxo_cbrtf(m0) - cb;
  m1 = jxo_cbrtf(m1) - cb;
  m2 = jxo_cbrtf(m2) - cb;
  *X = 0.5f * (m0 - m1);
  *Y = 0.5f * (m0 + m1);
  *B = m2;
}

/* padded frame: pixels beyond the image replicate the last column/row
 * (libjxl pads the opsin image to a block multiple by edge replication) */
void jxo_srgb8_to_xyb(const uint8_t* rgb, uint32_t w, uint32_t h,
                      size_t row_stride, uint32_t xp, uint32_t yp, float* xyb) {
  float lut[256];
  jxo_srgb_lut(lut);
  const float cb = jxo_cbrtf(JXO_BIAS);
  const size_t plane = (size_t)xp * yp;
#pragma omp parallel for schedule(static)
  for (uint32_t y = 0; y < yp; y++) {
    const uint8_t* row = rgb + (size_t)(y < h ? y : h - 1) * row_stride;
    for (uint32_t x = 0; x < xp; x++) {
      const uint8_t* p = row + 3 * (size_t)(x < w ? x : w - 1);
      size_t o = (size_t)y * xp + x;
      jxo_pixel_xyb(lut, cb, p[0], p[1], p[2], &xyb[o], &xyb[plane + o],
                    &xyb[2 * plane + o]);
    }
  }
}
