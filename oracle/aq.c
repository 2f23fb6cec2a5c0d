/* aq.c -- ORACLE (test infrastructure): libjxl-shaped adaptive quantization,
 * the masking-based initial quant field (JXO_OPT_AQ_MASKING; the GPU's
 * jxg_aq.hip must match it bit for bit).
 *
 * [ext] libjxl enc_adaptive_quantization.cc InitialQuantField ->
 * AdaptiveQuantizationMap: the field ACSConfig carries into the AC-strategy
 * search (proposals/combined.diff:412-418 context: masking_field_row,
 * masking1x1_field_stride) and Quantizer::SetQuantField uses.  libjxl is not
 * in /root/reference or this image: the structure and constants below are
 * restated as recalled, PARITY UNPINNED against libjxl.  Stages, on the
 * block-padded XYB frame (neighbours clamped to it, i.e. edge replication):
 *   1. per pixel of Y: diff = gammac * (Y - mean of the 4 neighbours), squared,
 *      limited to 0.2, MaskingSqrt; gammac = the ratio of derivatives of the
 *      cube root and butteraugli's simple gamma at Y + 0.019;
 *   2. pre_erosion: per 4x4 cell, 0.25 x (sum over the 4 columns of the
 *      4-row sums);
 *   3. FuzzyErosion: per cell the 4 smallest of its clamped 3x3 neighbourhood,
 *      weighted (distance-dependent weights, normalised to 0.2996), summed
 *      over the block's 2x2 cells;
 *   4. PerBlockModulations: ComputeMask (a rational function of the eroded
 *      value), HfModulation (sum of min(0.0206, |neighbour differences|) of Y
 *      inside the block), GammaModulation (log2 of the mean inverse gamma
 *      ratio of Y +- X + 0.16); quant field = FastPow2f(val / ln 2) x mul +
 *      add, mul / add damping the modulation above d 2.
 * The raw quant field is round(qf x 65536 / G) in [1, 256] (G: the
 * distance-only global scale of jxo_frame_init; libjxl derives its global
 * scale from the field's median -- not restated, so that sharded ranks need no
 * collective).  Every float op in a fixed order with explicit fmaf (libjxl's
 * MulAdd), IEEE division and sqrtf. */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "jxo_internal.h"

/* libjxl FastLog2f / FastPow2f [ext base/fast_math-inl.h, as recalled] */
static float jxo_fast_log2f(float x) {
  static const float p[3] = {-1.8503833400518310E-06f, 1.4287160470083755E+00f,
                             7.4245873327820566E-01f};
  static const float q[3] = {9.9032814277590719E-01f, 1.0096718572241148E+00f,
                             1.7409343003366853E-01f};
  int32_t xb;
  memcpy(&xb, &x, 4);
  const int32_t eb = xb - 0x3f2aaaab;
  const int32_t es = eb >> 23; /* arithmetic shift */
  const int32_t mb = xb - (int32_t)((uint32_t)es << 23);
  float m;
  memcpy(&m, &mb, 4);
  const float t = m - 1.0f;
  float yp = p[2], yq = q[2];
  yp = fmaf(yp, t, p[1]);
  yq = fmaf(yq, t, q[1]);
  yp = fmaf(yp, t, p[0]);
  yq = fmaf(yq, t, q[0]);
  return yp / yq + (float)es;
}
static float jxo_fast_pow2f(float x) {
  const float fl = floorf(x);
  const int32_t eb = ((int32_t)fl + 127) << 23;
  float e;
  memcpy(&e, &eb, 4);
  const float fr = x - fl;
  float num = fr + 1.01749063e+01f;
  num = fmaf(num, fr, 4.88687798e+01f);
  num = fmaf(num, fr, 9.85506591e+01f);
  num = num * e;
  float den = fmaf(fr, 2.10242958e-01f, -2.22328856e-02f);
  den = fmaf(den, fr, -1.94414990e+01f);
  den = fmaf(den, fr, 9.85506633e+01f);
  return num / den;
}

/* RatioOfDerivativesOfCubicRootToSimpleGamma [ext, as recalled]: den / num
 * (invert: num / den) */
#define AQ_SG_MUL 226.77216153508914f
#define AQ_SG_MUL2 (1.0f / 73.377132366608819f)
#define AQ_LOG2 0.693147181f
#define AQ_SG_RET_MUL (AQ_SG_MUL2 * 18.6580932135f * AQ_LOG2)
#define AQ_SG_VOFFSET 7.7825991679894591f
#define AQ_EPS 1e-2f
static float jxo_aq_ratio(float v, int invert) {
  const float num_mul = AQ_SG_RET_MUL * 3.0f * AQ_SG_MUL;
  const float num_off = AQ_EPS;
  const float den_off = AQ_SG_VOFFSET * AQ_LOG2 + AQ_EPS;
  const float den_mul = AQ_LOG2 * AQ_SG_MUL;
  if (!(v > 0.0f)) v = 0.0f;
  const float v2 = v * v;
  const float num = fmaf(num_mul, v2, num_off);
  const float den = fmaf(den_mul * v, v2, den_off);
  return invert ? num / den : den / num;
}

/* MaskingSqrt: 0.25 sqrt(v sqrt(kMul 1e8) + 28) */
static float jxo_masking_sqrt(float v) {
  const float mul = (float)((double)211.50759899638012f * 1e8);
  return 0.25f * sqrtf(fmaf(v, sqrtf(mul), 28.0f));
}

float jxo_aq_diff(const float* Y, uint32_t xp, uint32_t yp, int x, int y) {
  const int xm = x > 0 ? x - 1 : x, xq = x + 1 < (int)xp ? x + 1 : x;
  const int ym = y > 0 ? y - 1 : y, yq = y + 1 < (int)yp ? y + 1 : y;
  const float* r = Y + (size_t)y * xp;
  const float base = 0.25f * (((Y[(size_t)yq * xp + x] + Y[(size_t)ym * xp + x]) + r[xm]) + r[xq]);
  const float gammac = jxo_aq_ratio(r[x] + 0.019f, 0);
  float diff = gammac * (r[x] - base);
  diff = diff * diff;
  if (diff >= 0.2f) diff = 0.2f;
  return jxo_masking_sqrt(diff);
}

/* pre_erosion cell (cx, cy): rows accumulated in order, columns summed in
 * order, x 0.25 */
float jxo_aq_cell(const float* Y, uint32_t xp, uint32_t yp, int cx, int cy) {
  float col[4];
  for (int j = 0; j < 4; j++) {
    float s = jxo_aq_diff(Y, xp, yp, 4 * cx + j, 4 * cy);
    for (int i = 1; i < 4; i++) s += jxo_aq_diff(Y, xp, yp, 4 * cx + j, 4 * cy + i);
    col[j] = s;
  }
  return (((col[0] + col[1]) + col[2]) + col[3]) * 0.25f;
}

void jxo_aq_erosion_weights(float distance, float w[4]) {
  float mul = 0.0f;
  if (distance < 2.0f) mul = (2.0f - distance) * (1.0f / 2.0f);
  w[0] = 0.125f + mul * 0.0f;
  w[1] = 0.10f + mul * -0.10f;
  w[2] = 0.09f + mul * -0.09f;
  w[3] = 0.06f + mul * -0.06f;
  const float norm = 0.29959705784054957f / (((w[0] + w[1]) + w[2]) + w[3]);
  for (int i = 0; i < 4; i++) w[i] *= norm;
}

static void store_min4(float v, float* m0, float* m1, float* m2, float* m3) {
  if (v < *m3) {
    if (v < *m0) {
      *m3 = *m2;
      *m2 = *m1;
      *m1 = *m0;
      *m0 = v;
    } else if (v < *m1) {
      *m3 = *m2;
      *m2 = *m1;
      *m1 = v;
    } else if (v < *m2) {
      *m3 = *m2;
      *m2 = v;
    } else {
      *m3 = v;
    }
  }
}
#define SWAP_GT(a, b)  \
  if ((a) > (b)) {     \
    const float t_ = a; \
    a = b;             \
    b = t_;            \
  }
/* FuzzyErosion value of cell (cx, cy) of the ncx x ncy cell grid */
float jxo_aq_erode(const float* cells, int ncx, int ncy, int cx, int cy, const float w[4]) {
  const int xm = cx > 0 ? cx - 1 : cx, xq = cx + 1 < ncx ? cx + 1 : cx;
  const int ym = cy > 0 ? cy - 1 : cy, yq = cy + 1 < ncy ? cy + 1 : cy;
  const float* rt = cells + (size_t)ym * ncx;
  const float* rw = cells + (size_t)cy * ncx;
  const float* rb = cells + (size_t)yq * ncx;
  float m0 = rw[cx], m1 = rw[xm], m2 = rw[xq], m3 = rt[xm];
  SWAP_GT(m0, m1);
  SWAP_GT(m0, m2);
  SWAP_GT(m0, m3);
  SWAP_GT(m1, m2);
  SWAP_GT(m1, m3);
  SWAP_GT(m2, m3);
  store_min4(rt[cx], &m0, &m1, &m2, &m3);
  store_min4(rt[xq], &m0, &m1, &m2, &m3);
  store_min4(rb[xm], &m0, &m1, &m2, &m3);
  store_min4(rb[cx], &m0, &m1, &m2, &m3);
  store_min4(rb[xq], &m0, &m1, &m2, &m3);
  return ((w[0] * m0 + w[1] * m1) + w[2] * m2) + w[3] * m3;
}

/* ComputeMask [ext, as recalled] */
float jxo_aq_mask(float v) {
  const float v1 = fmaxf(v * 0.74760422233706747f, 1e-3f);
  const float v2 = 1.0f / (v1 + 305.04035728311436f);
  const float v3 = 1.0f / fmaf(v1, v1, 2.1925739705298404f);
  const float v4 = 1.0f / fmaf(v1, v1, 0.25f * 2.1925739705298404f);
  return -0.74174993f +
         fmaf(3.2353257320940401f, v4, fmaf(12.906028311180409f, v2, 5.0220313103171232f * v3));
}

/* the 8-lane tree sum of the GPU (lane = block column) */
static float tree8f(const float* v) {
  return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
}

/* HfModulation + GammaModulation of block (bx, by), added to v */
float jxo_aq_modulate(const float* X, const float* Y, uint32_t xp, int bx, int by, float v) {
  const float valmin = 0.020602694503245016f;
  float hs[8], gs[8];
  for (int j = 0; j < 8; j++) {
    float s = 0.0f, g = 0.0f;
    for (int dy = 0; dy < 8; dy++) {
      const size_t o = (size_t)(by * 8 + dy) * xp + bx * 8 + j;
      const size_t on = dy < 7 ? o + xp : o;
      const float p = Y[o];
      s += j < 7 ? fminf(valmin, fabsf(p - Y[o + 1])) : 0.0f;
      s += fminf(valmin, fabsf(p - Y[on]));
      const float iny = p + 0.16f, inx = X[o];
      const float rr = jxo_aq_ratio(iny - inx, 1), rg = jxo_aq_ratio(iny + inx, 1);
      g += 0.5f * (rr + rg);
    }
    hs[j] = s;
    gs[j] = g;
  }
  const float hf = (tree8f(hs) + -1.110929106987477f) * -0.38078920620238305f;
  v = hf + v;
  const float ratio = tree8f(gs) * (1.0f / 64.0f);
  return fmaf(-0.15526878023684174f * 0.693147180559945f, jxo_fast_log2f(ratio), v);
}

/* quant field raw (1..256) of every block: [bys][bxs] */
void jxo_aq_masking(const jxo_frame* f, const float* xyb, uint8_t* raw) {
  const size_t plane = (size_t)f->xp * f->yp;
  const float* X = xyb;
  const float* Y = xyb + plane;
  const int ncx = (int)f->xp / 4, ncy = (int)f->yp / 4;
  float* cells = (float*)malloc(sizeof(float) * (size_t)ncx * ncy);
#pragma omp parallel for schedule(static)
  for (int cy = 0; cy < ncy; cy++)
    for (int cx = 0; cx < ncx; cx++) cells[(size_t)cy * ncx + cx] = jxo_aq_cell(Y, f->xp, f->yp, cx, cy);
  float w[4];
  jxo_aq_erosion_weights(f->distance, w);
  float dampen = 1.0f;
  if (f->distance >= 2.0f) {
    dampen = 1.0f - ((f->distance - 2.0f) / (14.0f - 2.0f));
    if (dampen < 0.0f) dampen = 0.0f;
  }
  const float scale = f->qf_base;
  const float mul = scale * dampen, add = (1.0f - dampen) * (0.48f * scale);
#pragma omp parallel for schedule(static)
  for (int by = 0; by < (int)f->bys; by++)
    for (int bx = 0; bx < (int)f->bxs; bx++) {
      const float e00 = jxo_aq_erode(cells, ncx, ncy, 2 * bx, 2 * by, w);
      const float e10 = jxo_aq_erode(cells, ncx, ncy, 2 * bx + 1, 2 * by, w);
      const float e01 = jxo_aq_erode(cells, ncx, ncy, 2 * bx, 2 * by + 1, w);
      const float e11 = jxo_aq_erode(cells, ncx, ncy, 2 * bx + 1, 2 * by + 1, w);
      float v = ((e00 + e10) + e01) + e11;
      v = jxo_aq_mask(v);
      v = jxo_aq_modulate(X, Y, f->xp, bx, by, v);
      const float qf = jxo_fast_pow2f(v * 1.442695041f) * mul + add;
      int r = (int)(qf * f->inv_g + 0.5f);
      if (r < 1) r = 1;
      if (r > 256) r = 256;
      raw[(size_t)by * f->bxs + bx] = (uint8_t)(r - 1);
    }
  free(cells);
}
