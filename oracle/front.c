/*
 * front.c -- ORACLE (test infrastructure).  Per-8x8-block front end of the
 * VarDCT encode: block DC, adaptive quantization, AC-strategy choice among the
 * 8x8-class transforms (with the thesis hooks P and F), forward transforms,
 * chroma-from-luma residual and quantization.
 *
 * [ext] libjxl stages restated (enc_ac_strategy.cc, enc_adaptive_quantization.cc,
 * enc_transforms-inl.h, quant_weights.cc); not in /root/reference -> parity
 * unpinned against libjxl.  The thesis hooks follow
 * /root/reference/proposals/combined.diff:247-253 (F) and :270-274 (P).
 * Every float operation order here is the contract the HIP kernel mirrors.
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "jxo_internal.h"

/* ---------- default dequantization weights [ext quant_weights.cc] ---------- */
static double mult_band(double v) { return v > 0 ? 1.0 + v : 1.0 / (1.0 - v); }

static void get_quant_weights(int rows, int cols, const double bands_in[3][6],
                              int nb, double out[3][64]) {
  for (int c = 0; c < 3; c++) {
    double bands[6];
    bands[0] = bands_in[c][0];
    for (int i = 1; i < nb; i++) bands[i] = bands[i - 1] * mult_band(bands_in[c][i]);
    double scale = (nb - 1) / (1.4142135623730951 + 1e-6);
    double rcpcol = scale / (cols - 1), rcprow = scale / (rows - 1);
    for (int y = 0; y < rows; y++) {
      double dy = y * rcprow;
      for (int x = 0; x < cols; x++) {
        double dx = x * rcpcol;
        double pos = sqrt(dx * dx + dy * dy);
        int idx = (int)pos;
        if (idx > nb - 2) idx = nb - 2;
        double frac = pos - idx;
        double a = bands[idx], b = bands[idx + 1];
        out[c][y * cols + x] = a * pow(b / a, frac);
      }
    }
  }
}

void jxo_quant_weights(int kind, float out[3][64]) {
  static const double dct8[3][6] = {{3150.0, 0.0, -0.4, -0.4, -0.4, -2.0},
                                    {560.0, 0.0, -0.3, -0.3, -0.3, -0.3},
                                    {512.0, -2.0, -1.0, 0.0, -1.0, -2.0}};
  static const double dct4[3][6] = {{2200.0, 0.0, 0.0, 0.0},
                                    {392.0, 0.0, 0.0, 0.0},
                                    {112.0, -0.25, -0.25, -0.5}};
  static const double dct4x8[3][6] = {
      {2198.050556016380522, -0.96269623020744692, -0.76194253026666783, -0.6551140670773547},
      {764.3655248643528689, -0.92630200888366945, -0.9675229603596517, -0.27845290869168118},
      {527.107573587542228, -1.4594385811273854, -1.450082094097871593, -1.5843722511996204}};
  /* IDENTITY: every slot weight [0], the DC-combination slots 1 / 8 weight
   * [1], slot 9 weight [2]; DCT2X2: slots 1 / 8 [0], 9 [1], the level-2
   * quadrants [2] (off-diagonal) / [3] (diagonal), the level-1 quadrants [4] /
   * [5] [ext quant_weights.cc kQuantModeID / kQuantModeDCT2 defaults] */
  static const float id_w[3][3] = {{280.0f, 3160.0f, 3160.0f},
                                    {60.0f, 864.0f, 864.0f},
                                    {18.0f, 200.0f, 200.0f}};
  static const float dct2_w[3][6] = {{3840.0f, 2560.0f, 1280.0f, 640.0f, 480.0f, 300.0f},
                                     {960.0f, 640.0f, 320.0f, 180.0f, 140.0f, 120.0f},
                                     {640.0f, 320.0f, 128.0f, 64.0f, 32.0f, 16.0f}};
  if (kind == JXO_QK_ID) {
    for (int c = 0; c < 3; c++) {
      for (int i = 0; i < 64; i++) out[c][i] = id_w[c][0];
      out[c][1] = out[c][8] = id_w[c][1];
      out[c][9] = id_w[c][2];
    }
    return;
  }
  if (kind == JXO_QK_DCT2) {
    for (int c = 0; c < 3; c++)
      for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
          int k;
          if (y < 2 && x < 2) k = (y && x) ? 1 : 0;
          else if (y < 4 && x < 4) k = (y >= 2 && x >= 2) ? 3 : 2;
          else k = (y >= 4 && x >= 4) ? 5 : 4;
          out[c][y * 8 + x] = dct2_w[c][k];
        }
    return;
  }
  double w[3][64];
  if (kind == JXO_QK_DCT8) {
    get_quant_weights(8, 8, dct8, 6, w);
    for (int c = 0; c < 3; c++)
      for (int i = 0; i < 64; i++) out[c][i] = (float)w[c][i];
  } else if (kind == JXO_QK_DCT4) {
    get_quant_weights(4, 4, dct4, 4, w);
    for (int c = 0; c < 3; c++)
      for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) out[c][y * 8 + x] = (float)w[c][(y / 2) * 4 + x / 2];
  } else {
    get_quant_weights(4, 8, dct4x8, 4, w);
    for (int c = 0; c < 3; c++)
      for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) out[c][y * 8 + x] = (float)w[c][(y / 2) * 8 + x];
  }
}

/* Distortion weight of one quantized coefficient in the rate-distortion
 * estimates of the strategy search (8x8 class here, merged varblocks in
 * merge.c).  e = |v| - |q| is the quantization error in quantizer steps;
 * the step of a coefficient with weight w is 1/(w scale) in coefficient
 * units, and with this DCT normalization (out[0] = mean) a coefficient error
 * spreads sqrt(area) times its size over the `area` pixels its basis covers
 * (Parseval).  e * jxo_dist_weight(c, area, w) / scale is therefore the
 * pixel-domain (XYB) error of channel c, normalized by the channel's DCT8
 * band-0 weight jxo_w0[c] so that the three channels stay comparable
 * (the per-channel multiplier of libjxl's EstimateEntropy loss [ext]) and so
 * that a DCT8 band-0 coefficient keeps weight 1.  Without it the estimate
 * measured error in step units, which stay below 0.58 however coarse the
 * step, so coarse (large) transforms looked cheap.  Computed in double,
 * rounded once. */
const float jxo_w0[3] = {3150.0f, 560.0f, 512.0f};
float jxo_dist_weight(int c, int area, float w) {
  return (float)(sqrt((double)area / 64.0) * ((double)jxo_w0[c] / (double)w));
}

/* [ext] natural coefficient order of an 8x8 varblock (zigzag) */
void jxo_natural_order8(uint8_t order[64]) {
  int cur = 1;
  order[0] = 0;
  for (int i = 0; i < 8; i++)
    for (int j = 0; j <= i; j++) {
      int x = j, y = i - j;
      if (i & 1) {
        int t = x;
        x = y;
        y = t;
      }
      if (x == 0 && y == 0) continue;
      order[cur++] = (uint8_t)(y * 8 + x);
    }
  for (int ip = 7; ip > 0; ip--) {
    int i = ip - 1;
    for (int j = 0; j <= i; j++) {
      int x = 7 - (i - j), y = 7 - j;
      if (i & 1) {
        int t = x;
        x = y;
        y = t;
      }
      order[cur++] = (uint8_t)(y * 8 + x);
    }
  }
}

/* ---------- frame scalars (host-side, double precision) ---------- */
void jxo_frame_init(jxo_frame* f, uint32_t w, uint32_t h, const jxo_params* p) {
  memset(f, 0, sizeof(*f));
  f->w = w;
  f->h = h;
  f->bxs = (w + 7) / 8;
  f->bys = (h + 7) / 8;
  f->xp = f->bxs * 8;
  f->yp = f->bys * 8;
  f->gxs = (w + 255) / 256;
  f->gys = (h + 255) / 256;
  f->ngroups = f->gxs * f->gys;
  f->lfxs = (w + 2047) / 2048;
  f->lfys = (h + 2047) / 2048;
  f->nlf = f->lfxs * f->lfys;
  f->distance = p->distance;
  f->effort = p->effort;
  f->proposals = p->proposals;
  double d = p->distance;
  double qfb = 0.79 / d;
  f->qf_base = (float)qfb;
  long G = (long)floor(qfb * 1024.0 + 0.5);
  if (G < 1) G = 1;
  if (G > 73727) G = 73727;
  f->G = (uint32_t)G;
  f->inv_g = (float)(65536.0 / (double)G);
  double t = 0.3 * pow(d / 0.3, 0.66);
  if (t > d) t = d;
  if (t < 0.5 * d) t = 0.5 * d;
  double qdc_f = 1.12 / t;
  if (qdc_f > 50.0) qdc_f = 50.0;
  long qdc = (long)floor(qdc_f * 65536.0 / (double)G + 0.5);
  if (qdc < 1) qdc = 1;
  if (qdc > 65536) qdc = 65536;
  f->qdc = (uint32_t)qdc;
  static const double m_lf[3] = {1.0 / 4096.0, 1.0 / 512.0, 1.0 / 256.0};
  for (int c = 0; c < 3; c++) {
    f->dc_mul[c] = (float)((double)G * (double)qdc / 65536.0 / m_lf[c]);
    f->dc_step[c] = (float)(65536.0 / (double)G / (double)qdc * m_lf[c]);
  }
  for (int k = 0; k < 5; k++) jxo_quant_weights(k, f->wts[k]);
  /* distortion weights per 8x8-class strategy (table index DCT8, DCT4X4,
   * DCT4X8, DCT8X4, DCT2X2, IDENTITY -- jxo_tindex) and coefficient-layout
   * position: the lowest-frequency combine slots span the whole block (area
   * 64); other DCT4X4 coefficients span a 4x4 sub-block (16), DCT4X8 / DCT8X4
   * ones a 4x8 half (32); DCT2X2 level-2 coefficients a 4x4 quarter (16),
   * level-1 ones a 2x2 cell (4); IDENTITY residuals one pixel (1) */
  for (int ti = 0; ti < 6; ti++) {
    static const int qks[6] = {JXO_QK_DCT8, JXO_QK_DCT4, JXO_QK_DCT4X8, JXO_QK_DCT4X8,
                               JXO_QK_DCT2, JXO_QK_ID};
    const int qk = qks[ti];
    for (int c = 0; c < 3; c++)
      for (int co = 0; co < 64; co++) {
        const int row = co >> 3, col = co & 7;
        int area = 64;
        if (ti == 1 && !(row < 2 && col < 2)) area = 16;
        if ((ti == 2 || ti == 3) && !(row < 2 && col == 0)) area = 32;
        if (ti == 4 && !(row < 2 && col < 2)) area = row < 4 && col < 4 ? 16 : 4;
        if (ti == 5 && !(row < 2 && col < 2)) area = 1;
        f->sdw[ti][c][co] = jxo_dist_weight(c, area, f->wts[qk][c][co]);
      }
  }
}

/* ---------- transforms ----------
 * DCT-II scaled so that out[0] is the mean (out[k] = a_k/N sum x_n
 * cos(pi(2n+1)k/2N), a_0 = 1, a_k = sqrt 2), computed by a fixed even/odd
 * butterfly with explicit fmaf chains.  The constants are float(sqrt2/N *
 * cos(...)) written as hex literals; the HIP kernel uses the same sequence. */
#define K_A 0x1.63150cp-3f  /* sqrt2/8 cos(pi/16)  */
#define K_B 0x1.2d062ep-3f  /* sqrt2/8 cos(3pi/16) */
#define K_C 0x1.92469cp-4f  /* sqrt2/8 cos(5pi/16) */
#define K_D 0x1.1a855ep-5f  /* sqrt2/8 cos(7pi/16) */
#define K_E1 0x1.4e7aeap-3f /* sqrt2/8 cos(pi/8)   */
#define K_E3 0x1.1517a8p-4f /* sqrt2/8 cos(3pi/8)  */
#define K_F1 0x1.4e7aeap-2f /* sqrt2/4 cos(pi/8)   */
#define K_F3 0x1.1517a8p-3f /* sqrt2/4 cos(3pi/8)  */

static void dct8_1d(float* v, int st) {
  const float x0 = v[0], x1 = v[st], x2 = v[2 * st], x3 = v[3 * st], x4 = v[4 * st],
              x5 = v[5 * st], x6 = v[6 * st], x7 = v[7 * st];
  const float s0 = x0 + x7, s1 = x1 + x6, s2 = x2 + x5, s3 = x3 + x4;
  const float d0 = x0 - x7, d1 = x1 - x6, d2 = x2 - x5, d3 = x3 - x4;
  const float a0 = s0 + s3, a1 = s1 + s2, b0 = s0 - s3, b1 = s1 - s2;
  v[0] = (a0 + a1) * 0.125f;
  v[4 * st] = (a0 - a1) * 0.125f;
  v[2 * st] = fmaf(b1, K_E3, b0 * K_E1);
  v[6 * st] = fmaf(b1, -K_E1, b0 * K_E3);
  v[1 * st] = fmaf(d3, K_D, fmaf(d2, K_C, fmaf(d1, K_B, d0 * K_A)));
  v[3 * st] = fmaf(d3, -K_C, fmaf(d2, -K_A, fmaf(d1, -K_D, d0 * K_B)));
  v[5 * st] = fmaf(d3, K_B, fmaf(d2, K_D, fmaf(d1, -K_A, d0 * K_C)));
  v[7 * st] = fmaf(d3, -K_A, fmaf(d2, K_B, fmaf(d1, -K_C, d0 * K_D)));
}
static void dct4_1d(float* v, int st) {
  const float x0 = v[0], x1 = v[st], x2 = v[2 * st], x3 = v[3 * st];
  const float s0 = x0 + x3, s1 = x1 + x2, d0 = x0 - x3, d1 = x1 - x2;
  v[0] = (s0 + s1) * 0.25f;
  v[2 * st] = (s0 - s1) * 0.25f;
  v[st] = fmaf(d1, K_F3, d0 * K_F1);
  v[3 * st] = fmaf(d1, -K_F1, d0 * K_F3);
}

/* 2D DCT of an R x C region (row stride 8) -> out[R][C]; rows first */
static void dct2d(const float* in, int R, int C, float* out) {
  float t[64];
  for (int r = 0; r < R; r++)
    for (int c = 0; c < C; c++) t[r * 8 + c] = in[r * 8 + c];
  for (int r = 0; r < R; r++) {
    if (C == 8) dct8_1d(t + r * 8, 1);
    else dct4_1d(t + r * 8, 1);
  }
  for (int c = 0; c < C; c++) {
    if (R == 8) dct8_1d(t + c, 8);
    else dct4_1d(t + c, 8);
  }
  for (int r = 0; r < R; r++)
    for (int c = 0; c < C; c++) out[r * C + c] = t[r * 8 + c];
}

/* forward transform of one channel of an 8x8 block into the coefficient
 * layout of raw strategy t [ext enc_transforms-inl.h].  Slot 0 is unused by
 * the AC coder (DC travels in the LF image). */
void jxo_transform(int t, const float* px /* 8x8, stride 8 */, float* co) {
  float o[64];
  if (t == JXO_DCT8) {
    dct2d(px, 8, 8, co);
  } else if (t == JXO_DCT4X4) {
    for (int sy = 0; sy < 2; sy++)
      for (int sx = 0; sx < 2; sx++) {
        dct2d(px + sy * 32 + sx * 4, 4, 4, o);
        for (int iy = 0; iy < 4; iy++)
          for (int ix = 0; ix < 4; ix++) co[(sy + 2 * iy) * 8 + sx + 2 * ix] = o[iy * 4 + ix];
      }
    float A = co[0], B = co[1], C = co[8], D = co[9];
    co[0] = (((A + B) + C) + D) * 0.25f;
    co[1] = (((A + B) - C) - D) * 0.25f;
    co[8] = (((A - B) + C) - D) * 0.25f;
    co[9] = (((A - B) - C) + D) * 0.25f;
  } else if (t == JXO_DCT8X4) { /* two 4-row x 8-col halves stacked */
    for (int sy = 0; sy < 2; sy++) {
      dct2d(px + sy * 32, 4, 8, o);
      for (int iy = 0; iy < 4; iy++)
        for (int ix = 0; ix < 8; ix++) co[(sy + 2 * iy) * 8 + ix] = o[iy * 8 + ix];
    }
    float A = co[0], B = co[8];
    co[0] = (A + B) * 0.5f;
    co[8] = (A - B) * 0.5f;
  } else if (t == JXO_DCT2X2) {
    /* three levels of 2x2 Haar steps, 0.25 per level [ext enc_transforms-inl.h
     * DCT2TopBlock<8, 4, 2>]: per 2x2 cell the row sums / differences
     * a = c00 + c01, b = c00 - c01, then r00 = (a_top + a_bottom) / 4 ->
     * (y, x), r01 = (a_top - a_bottom) / 4 -> (y, n + x), r10 = (b_top +
     * b_bottom) / 4 -> (n + y, x), r11 = (b_top - b_bottom) / 4 -> (n + y,
     * n + x), n = S / 2 */
    for (int i = 0; i < 64; i++) co[i] = px[i];
    for (int S = 8; S >= 2; S >>= 1) {
      const int n = S / 2;
      for (int i = 0; i < 64; i++) o[i] = co[i];
      for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) {
          const float c00 = o[(2 * y) * 8 + 2 * x], c01 = o[(2 * y) * 8 + 2 * x + 1];
          const float c10 = o[(2 * y + 1) * 8 + 2 * x], c11 = o[(2 * y + 1) * 8 + 2 * x + 1];
          const float at = c00 + c01, bt = c00 - c01, ab = c10 + c11, bb = c10 - c11;
          co[y * 8 + x] = (at + ab) * 0.25f;
          co[y * 8 + n + x] = (at - ab) * 0.25f;
          co[(n + y) * 8 + x] = (bt + bb) * 0.25f;
          co[(n + y) * 8 + n + x] = (bt - bb) * 0.25f;
        }
    }
  } else if (t == JXO_IDENTITY) {
    /* per 4x4 sub-block (y, x): residuals against its pixel (1, 1) in the
     * interleaved slots (y + 2 iy, x + 2 ix); the (0, 0) residual moves to
     * the slot of (1, 1); slot (y, x) holds the sub-block mean (row sums left
     * to right, rows ((0 + 1) + (2 + 3)), / 16); the four means are then
     * combined like DCT4X4's [ext enc_transforms-inl.h IDENTITY] */
    for (int y = 0; y < 2; y++)
      for (int x = 0; x < 2; x++) {
        const float* sb = px + (4 * y) * 8 + 4 * x;
        float rs[4];
        for (int iy = 0; iy < 4; iy++)
          rs[iy] = ((sb[iy * 8] + sb[iy * 8 + 1]) + sb[iy * 8 + 2]) + sb[iy * 8 + 3];
        const float dc = ((rs[0] + rs[1]) + (rs[2] + rs[3])) * (1.0f / 16.0f);
        const float p11 = sb[8 + 1];
        for (int iy = 0; iy < 4; iy++)
          for (int ix = 0; ix < 4; ix++) co[(y + 2 * iy) * 8 + x + 2 * ix] = sb[iy * 8 + ix] - p11;
        co[(y + 2) * 8 + x + 2] = sb[0] - p11;
        co[y * 8 + x] = dc;
      }
    float A = co[0], B = co[1], C = co[8], D = co[9];
    co[0] = (((A + B) + C) + D) * 0.25f;
    co[1] = (((A + B) - C) - D) * 0.25f;
    co[8] = (((A - B) + C) - D) * 0.25f;
    co[9] = (((A - B) - C) + D) * 0.25f;
  } else { /* JXO_DCT4X8: two 8-row x 4-col halves side by side, stored transposed */
    for (int sx = 0; sx < 2; sx++) {
      dct2d(px + sx * 4, 8, 4, o);
      for (int ry = 0; ry < 8; ry++)
        for (int cx = 0; cx < 4; cx++) co[(sx + 2 * cx) * 8 + ry] = o[ry * 4 + cx];
    }
    float A = co[0], B = co[8];
    co[0] = (A + B) * 0.5f;
    co[8] = (A - B) * 0.5f;
  }
}

/* [ext] default quant biases (decoder side, OpsinInverseMatrix defaults) */
static const float kBias[4] = {1.0f - 0.05465007330715401f, 1.0f - 0.07005449891748593f,
                               1.0f - 0.049935103337343655f, 0.145f};
static inline float adjust_bias(int c, int q) {
  if (q == 0) return 0.0f;
  if (q == 1) return kBias[c];
  if (q == -1) return -kBias[c];
  return (float)q - kBias[3] / (float)q;
}
/* pairwise (tree) sum of 8 lane partials: ((0+1)+(2+3))+((4+5)+(6+7)) -- the
 * order an XOR-butterfly reduction over the 8 lanes of a GPU group yields */
static inline float tree8(const float* v) {
  return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
}
/* dead zone 0.58, round half up, clamp to int16 (the coefficient storage
 * type of the GPU path; |q| <= 32767 holds for distance >= ~0.05) */
static inline int quant1(float v) {
  float a = fabsf(v);
  if (a < 0.58f) return 0;
  int q = a < 32767.0f ? (int)(a + 0.5f) : 32767;
  if (q > 32767) q = 32767;
  return v < 0.0f ? -q : q;
}
static inline int bitlen(uint32_t v) {
  int n = 0;
  while (v) {
    n++;
    v >>= 1;
  }
  return n;
}

static int qkind(int t) {
  if (t == JXO_IDENTITY) return JXO_QK_ID;
  if (t == JXO_DCT2X2) return JXO_QK_DCT2;
  return t == JXO_DCT8 ? JXO_QK_DCT8 : (t == JXO_DCT4X4 ? JXO_QK_DCT4 : JXO_QK_DCT4X8);
}
/* table index of an 8x8-class strategy (distortion weights; GPU tables) */
static int jxo_tindex(int t) {
  switch (t) {
    case JXO_DCT8: return 0;
    case JXO_DCT4X4: return 1;
    case JXO_DCT4X8: return 2;
    case JXO_DCT8X4: return 3;
    case JXO_DCT2X2: return 4;
    default: return 5; /* JXO_IDENTITY */
  }
}

/* Quantize one block under strategy t.  Channel order Y, X, B (Y first: X/B
 * subtract the dequantized Y -- CfL with ytox=0, ytob base 1.0).  Returns the
 * rate/distortion cost; writes q[3][64] (X,Y,B order) if q != NULL. */
/* raster position (in the coefficient layout of t) of the transform's
 * working-array element p = prow*8 + pcol (inverse of the layout permutation
 * applied in jxo_transform). */
static int co_index(int t, int p) {
  const int prow = p >> 3, pcol = p & 7;
  if (t == JXO_DCT8) return p;
  /* IDENTITY / DCT2X2: GPU lane pcol holds one layout row (IDENTITY: pixel row
   * pcol's residuals, pixel column prow -> slot column (prow >> 2) + 2 (prow &
   * 3)); DCT2X2: lane pcol's k-th value after the three Haar levels (odd
   * lanes: level-1 bottom rows; even lanes: level-1 top row (k >= 4) and the
   * level-2 / level-3 outputs (k < 4)) */
  if (t == JXO_IDENTITY) return ((pcol >> 2) + 2 * (pcol & 3)) * 8 + (prow >> 2) + 2 * (prow & 3);
  if (t == JXO_DCT2X2) {
    const int q = pcol >> 1;
    const int row = (pcol & 1) ? 4 + q : (prow >= 4 ? q : ((q & 1) ? 2 + (q >> 1) : (q >> 1)));
    return row * 8 + prow;
  }
  if (t == JXO_DCT4X4)
    return ((prow >> 2) + 2 * (prow & 3)) * 8 + (pcol >> 2) + 2 * (pcol & 3);
  if (t == JXO_DCT8X4) return ((prow >> 2) + 2 * (prow & 3)) * 8 + pcol;
  return ((pcol >> 2) + 2 * (pcol & 3)) * 8 + prow; /* JXO_DCT4X8 */
}

/* The distortion sum follows the GPU decomposition (8 lanes per block, lane r
 * owns working-array column r after the column pass): lane r accumulates
 * e*e with fmaf over channels Y, X, B and rows k = 0..7 (skipping the DC
 * slot); the 8 lane partials are then tree-summed (tree8).  The Y dequant
 * used for the B residual multiplies by the inverse weight (1/w) and the
 * inverse scale (1/scale), like libjxl's dequantization [ext]. */
float jxo_quantize_block(const jxo_frame* f, int t, const float px[3][64],
                         float scale, int32_t q[3][64], const float cfl[2]) {
  float co[3][64];
  for (int c = 0; c < 3; c++) jxo_transform(t, px[c], co[c]);
  const int qk = qkind(t);
  const float inv_scale = 1.0f / scale;
  const float(*sd)[64] = f->sdw[jxo_tindex(t)];
  float yd[64];
  float part[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int bits = 0;
  static const int corder[3] = {1, 0, 2};
  for (int ci = 0; ci < 3; ci++) {
    const int c = corder[ci];
    int nz = 0;
    for (int r = 0; r < 8; r++) {
      for (int k = 0; k < 8; k++) {
        const int ci_ = co_index(t, k * 8 + r);
        if (ci_ == 0) continue;
        const float ws = f->wts[qk][c][ci_] * scale;
        float rv = co[c][ci_];
        /* chroma from luma: X - kx Yd, B - kb Yd (the tile's factors) */
        if (c == 0) rv = rv - cfl[0] * yd[ci_];
        if (c == 2) rv = rv - cfl[1] * yd[ci_];
        const float v = rv * ws;
        const int qq = quant1(v);
        if (c == 1) yd[ci_] = adjust_bias(1, qq) * ((1.0f / f->wts[qk][c][ci_]) * inv_scale);
        const uint32_t aq = (uint32_t)(qq < 0 ? -qq : qq);
        const float e = (fabsf(v) - (float)aq) * sd[c][ci_];
        part[r] = fmaf(e, e, part[r]);
        if (aq) {
          bits += 2 + 2 * bitlen(aq);
          nz++;
        }
        if (q) q[c][ci_] = qq;
      }
    }
    bits += bitlen((uint32_t)nz);
    if (q) q[c][0] = 0;
  }
  const float dist = tree8(part);
  static const float tmul[14] = {1.0f, JXO_TMUL_ID, JXO_TMUL_DCT2, 1.05f, 0, 0, 0, 0, 0, 0, 0, 0,
                                 1.02f, 1.02f};
  return ((float)bits + 8.0f * dist) * tmul[t];
}

/* DC quantization: Y first, B residual against dequantized Y (base
 * correlation b = 1.0, x = 0.0) [ext] */
void jxo_quant_dc(const jxo_frame* f, const float dc[3], int32_t dcq[3]) {
  int qy = dc[1] * f->dc_mul[1] >= 0.0f ? (int)(dc[1] * f->dc_mul[1] + 0.5f)
                                        : -(int)(-(dc[1] * f->dc_mul[1]) + 0.5f);
  float ydq = (float)qy * f->dc_step[1];
  float xv = dc[0] * f->dc_mul[0];
  float bv = (dc[2] - ydq) * f->dc_mul[2];
  dcq[1] = qy;
  dcq[0] = xv >= 0.0f ? (int)(xv + 0.5f) : -(int)(-xv + 0.5f);
  dcq[2] = bv >= 0.0f ? (int)(bv + 0.5f) : -(int)(-bv + 0.5f);
}

/* block-level front end: pixels px[c][64] (X,Y,B), returns chosen strategy,
 * writes qf raw (1..256), quantized AC and DC. */
int jxo_front_block(const jxo_frame* f, const float px[3][64], const float* homog,
                    int32_t q[3][64], int32_t dcq[3], int* qf_raw, float* ent_out,
                    const float cfl[2], int aq_raw) {
  /* block DC = mean: row partial sums (left to right), then the 8 row sums
   * tree-summed -- the 8-lane order of the GPU path (lane = row) */
  float dc[3];
  for (int c = 0; c < 3; c++) {
    float rs[8];
    for (int y = 0; y < 8; y++) {
      rs[y] = 0.0f;
      for (int x = 0; x < 8; x++) rs[y] += px[c][y * 8 + x];
    }
    dc[c] = tree8(rs) * (1.0f / 64.0f);
  }
  /* DC quantization: Y first, B residual against dequantized Y (base
   * correlation b = 1.0, x = 0.0) */
  jxo_quant_dc(f, dc, dcq);

  /* adaptive quantization: mean absolute gradient of Y inside the block;
   * per row y: horizontal diffs of row y plus vertical diffs to row y+1,
   * the 8 row partials tree-summed (lane order of the GPU path) */
  const float* Y = px[1];
  float ra[8];
  for (int y = 0; y < 8; y++) {
    float hr = 0.0f, vr = 0.0f;
    for (int x = 0; x < 7; x++) hr += fabsf(Y[y * 8 + x + 1] - Y[y * 8 + x]);
    if (y < 7)
      for (int x = 0; x < 8; x++) vr += fabsf(Y[(y + 1) * 8 + x] - Y[y * 8 + x]);
    ra[y] = hr + vr;
  }
  const float act = tree8(ra);
  float am = act * (1.0f / 112.0f);
  float mult = 1.5f / sqrtf(1.0f + am * 40.0f);
  if (mult < 0.45f) mult = 0.45f;
  if (mult > 1.5f) mult = 1.5f;
  float qff = f->qf_base * mult;
  int raw = (int)(qff * f->inv_g + 0.5f);
  if (raw < 1) raw = 1;
  if (raw > 256) raw = 256;
  if (aq_raw > 0) raw = aq_raw; /* the masking field (aq.c, JXO_OPT_AQ_MASKING) */
  *qf_raw = raw;
  const float scale = (float)f->G * (float)raw / 65536.0f;

  /* AC strategy search over the 8x8-class candidates [ext
   * FindBest8x8Transform], hook F on every estimate, hook P on a DCT8 win */
  /* scan order of libjxl's kTransforms8x8 (DCT, DCT4X4, DCT2X2, DCT4X8,
   * DCT8X4, IDENTITY; AFV0-3 not searched) */
  static const int cand[6] = {JXO_DCT8, JXO_DCT4X4, JXO_DCT2X2, JXO_DCT4X8, JXO_DCT8X4,
                              JXO_IDENTITY};
  const int ncand = f->effort >= 5 ? 6 : 1;
  int best_t = JXO_DCT8;
  float best = FLT_MAX;
  if (ncand > 1) {
    for (int i = 0; i < ncand; i++) {
      float e = jxo_quantize_block(f, cand[i], px, scale, NULL, cfl);
      if (f->proposals & 2) e = jxo_hook_f(e, homog[0], homog[1], homog[2]);
      if (e < best) {
        best = e;
        best_t = cand[i];
      }
    }
  }
  /* the estimate the merge stage sums is stored before the P override
   * (homogeneity-partitioning.diff:271 context) */
  if (ent_out) *ent_out = best;
  /* hook P sits inside FindBest8x8Transform (combined.diff:266-276), which
   * libjxl's AC-strategy heuristics do not run at the all-DCT8 speed tiers
   * (effort < 5 here, the same condition as the candidate search above) [ext]:
   * no override there */
  if ((f->proposals & 1) && ncand > 1 && best_t == JXO_DCT8) {
    /* HomogeneityPartition thresholds, combined.diff:219-234 */
    float T = 1.60f;
    if ((double)f->distance > 10.0)
      T = 1.80f;
    else if ((double)f->distance <= 3.0)
      T = 1.50f;
    const float rh = homog[0], rv = homog[1], rd = homog[2];
    if (rd > T)
      best_t = JXO_DCT4X4;
    else if (rh > rv && rh > T)
      best_t = JXO_DCT8X4;
    else if (rv > rh && rv > T)
      best_t = JXO_DCT4X8;
  }
  jxo_quantize_block(f, best_t, px, scale, q, cfl);
  return best_t;
}

/* ---------- chroma from luma: per-64x64-tile factors ----------
 * [ext] libjxl enc_chroma_from_luma (per colour tile, before the AC-strategy
 * search; EstimateEntropy then scores every candidate on the CfL residual --
 * the cmap_factors argument of combined.diff:240), restated as a weighted
 * least-squares fit in quantization steps over the DCT8 AC coefficients of
 * the tile's blocks:
 *   X ~ kx Y : kx = sum(wx^2 x y) / sum(wx^2 y^2)
 *   B ~ (1 + kb) Y : kb = sum(wb^2 (b - y) y) / sum(wb^2 y^2)
 * (w = the DCT8 quant weight of the coefficient), stored as int8 multiples of
 * 1/84 (the default colour_factor): ytox = clamp(round(84 kx)).  The decoder
 * (and the quantizer) use kx = ytox / 84, kb = 1 + ytob / 84.
 * Summation order = the GPU's: per block, lane r (= coefficient column r)
 * accumulates rows k = 0..7 with fmaf, the 8 lane partials are tree-summed
 * (tree8), and the tile sums the blocks inside the frame in raster order.
 * Effort < 5 (no AC-strategy search either): no fit, factors 0. */
static int8_t cfl_quant(float k) {
  float v = k * 84.0f;
  v = fminf(fmaxf(v, -128.0f), 127.0f);
  const int q = v >= 0.0f ? (int)(v + 0.5f) : -(int)(-v + 0.5f);
  return (int8_t)(q > 127 ? 127 : (q < -128 ? -128 : q));
}
void jxo_cfl_tile(const jxo_frame* f, const float* xyb, int tx, int ty, int8_t* ytox,
                  int8_t* ytob) {
  *ytox = 0;
  *ytob = 0;
  if (f->effort < 5) return;
  const size_t plane = (size_t)f->xp * f->yp;
  float T[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int lby = 0; lby < 8; lby++)
    for (int lbx = 0; lbx < 8; lbx++) {
      const int bx = tx * 8 + lbx, by = ty * 8 + lby;
      if (bx >= (int)f->bxs || by >= (int)f->bys) continue;
      float px[64], co[3][64];
      for (int c = 0; c < 3; c++) {
        for (int y = 0; y < 8; y++)
          for (int x = 0; x < 8; x++)
            px[y * 8 + x] = xyb[c * plane + (size_t)(by * 8 + y) * f->xp + bx * 8 + x];
        jxo_transform(JXO_DCT8, px, co[c]);
      }
      float acc[4][8];
      for (int r = 0; r < 8; r++) {
        float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
        for (int k = 0; k < 8; k++) {
          const int p = k * 8 + r;
          if (p == 0) continue;
          const float wx = f->wts[JXO_QK_DCT8][0][p], wb = f->wts[JXO_QK_DCT8][2][p];
          const float w2x = wx * wx, w2b = wb * wb;
          const float y = co[1][p], x = co[0][p], b = co[2][p];
          a0 = fmaf(w2x * x, y, a0);
          a1 = fmaf(w2x * y, y, a1);
          a2 = fmaf(w2b * (b - y), y, a2);
          a3 = fmaf(w2b * y, y, a3);
        }
        acc[0][r] = a0;
        acc[1][r] = a1;
        acc[2][r] = a2;
        acc[3][r] = a3;
      }
      for (int i = 0; i < 4; i++) T[i] = T[i] + tree8(acc[i]);
    }
  *ytox = cfl_quant(T[1] > 0.0f ? T[0] / T[1] : 0.0f);
  *ytob = cfl_quant(T[3] > 0.0f ? T[2] / T[3] : 0.0f);
}
void jxo_cfl_factors(int8_t ytox, int8_t ytob, float cfl[2]) {
  cfl[0] = (float)ytox * (1.0f / 84.0f);
  cfl[1] = 1.0f + (float)ytob * (1.0f / 84.0f);
}
