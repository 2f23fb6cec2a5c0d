/*
 * homog.c -- ORACLE (test infrastructure).  Plain-C restatement of the
 * thesis homogeneity-based AC-strategy selector.
 *
 * Reference: /root/reference/proposals/combined.diff
 *   CalculateNumZeroCrossings             :17-55
 *   CalculateLaplacianFilter              :57-81
 *   CalculateSumModifiedLaplacian         :83-105
 *   CalculateColorfulness                 :107-151
 *   CalculateHomogeneity                  :153-181
 *   CalculateHomogeneitySimilarityIndices :183-211
 *   HomogeneityPartition                  :213-235
 *   hook F (EstimateEntropy)              :247-253
 *
 * Floating-point conventions are fixed here and mirrored bit-for-bit by the
 * HIP kernel:
 *   H1  canonical abs = fabsf (JXO_H1_INT_ABS selects int abs(int)).
 *   H2  samples outside the padded frame read as 0.0f; SML skips a sample
 *       when y+1 >= ysize (combined.diff:91), never on x (stride > xsize).
 *   H3  colorfulness: double sqrt of the float argument, double sum, one
 *       rounding to float (combined.diff:148-150).
 *   H4  IEEE 0/0 -> NaN -> DCT, x/0 -> inf.
 *   H5  compiled with -ffp-contract=off.
 */
#include <math.h>
#include <stdlib.h>

#include "jxo.h"

static inline float pix(const jxo_xyb* img, int c, long x, long y) {
  if (x < 0 || y < 0 || (size_t)x >= img->xsize || (size_t)y >= img->ysize)
    return 0.0f;
  return img->plane[c][(size_t)y * img->stride + (size_t)x];
}

/* combined.diff:57-81.  3x3 mask {{0,-1,0},{-1,-4,-1},{0,-1,0}} on Y only,
 * k-outer/l-inner; the zero taps add +-0 and never change the sum. */
static void laplacian(const jxo_xyb* img, size_t x, size_t y, size_t xs,
                      size_t ys, size_t bx, size_t by, float* out) {
  for (size_t i = by; i < ys + by; i++) {
    for (size_t j = bx; j < xs + bx; j++) {
      long px = (long)(x + j), py = (long)(y + i);
      float sum = 0.0f;
      sum += pix(img, 1, px, py - 1) * -1.0f;
      sum += pix(img, 1, px - 1, py) * -1.0f;
      sum += pix(img, 1, px, py) * -4.0f;
      sum += pix(img, 1, px + 1, py) * -1.0f;
      sum += pix(img, 1, px, py + 1) * -1.0f;
      out[(i - by) * xs + (j - bx)] = sum;
    }
  }
}

/* combined.diff:17-55 */
static size_t zero_crossings(size_t xs, size_t ys, float t, const float* L) {
  size_t nh = 0;
  for (size_t i = 0; i < ys; i++) {
    int in_edge = 0;
    for (size_t j = 0; j < xs; j++) {
      float v = L[i * xs + j];
      if (!in_edge && v > t) {
        nh++;
        in_edge = 1;
      } else if (in_edge && v <= t) {
        in_edge = 0;
      }
    }
  }
  float avg_h = (float)nh / (float)ys;
  size_t nv = 0;
  for (size_t i = 0; i < xs; i++) {
    int in_edge = 0;
    for (size_t j = 0; j < ys; j++) {
      float v = L[j * xs + i];
      if (!in_edge && v > t) {
        nv++;
        in_edge = 1;
      } else if (in_edge && v <= t) {
        in_edge = 0;
      }
    }
  }
  float avg_v = (float)nv / (float)xs;
  return (size_t)(avg_h + avg_v); /* returns size_t: truncation (:17, :54) */
}

/* combined.diff:83-105 */
static float sum_modified_laplacian(const jxo_xyb* img, size_t x, size_t y,
                                    size_t xs, size_t ys, size_t bx, size_t by,
                                    int h1_mode) {
  float sum = 0.0f;
  for (size_t i = by; i < ys + by; i++) {
    for (size_t j = bx; j < xs + bx; j++) {
      /* the '< 0' tests are dead on size_t; x+j+1 >= stride never holds
       * because stride > xsize (H2) */
      if (y + i + 1 >= img->ysize) continue;
      long px = (long)(x + j), py = (long)(y + i);
      float p = pix(img, 1, px, py);
      float l = pix(img, 1, px - 1, py);
      float r = pix(img, 1, px + 1, py);
      float u = pix(img, 1, px, py - 1);
      float d = pix(img, 1, px, py + 1);
      float a = 2.0f * p - l - r;
      float b = 2.0f * p - u - d;
      if (h1_mode == JXO_H1_INT_ABS) {
        int ia = abs((int)a), ib = abs((int)b);
        sum += (float)(ia + ib);
      } else {
        sum += fabsf(a) + fabsf(b);
      }
    }
  }
  return sum;
}

/* combined.diff:107-151 */
static float colorfulness(const jxo_xyb* img, size_t x, size_t y, size_t xs,
                          size_t ys, size_t bx, size_t by) {
  const float n = (float)(xs * ys);
  float mean_x = 0.0f;
  for (size_t i = by; i < ys + by; i++)
    for (size_t j = bx; j < xs + bx; j++)
      mean_x += pix(img, 0, (long)(x + j), (long)(y + i));
  mean_x /= n;
  float mean_b = 0.0f;
  for (size_t i = by; i < ys + by; i++)
    for (size_t j = bx; j < xs + bx; j++)
      mean_b += pix(img, 2, (long)(x + j), (long)(y + i));
  mean_b /= n;
  float var_x = 0.0f;
  for (size_t i = by; i < ys + by; i++)
    for (size_t j = bx; j < xs + bx; j++) {
      float diff = pix(img, 0, (long)(x + j), (long)(y + i)) - mean_x;
      var_x += diff * diff;
    }
  var_x /= n;
  float var_b = 0.0f;
  for (size_t i = by; i < ys + by; i++)
    for (size_t j = bx; j < xs + bx; j++) {
      float diff = pix(img, 2, (long)(x + j), (long)(y + i)) - mean_b;
      var_b += diff * diff;
    }
  var_b /= n;
  float vsum = var_x + var_b;
  float msum = mean_x * mean_x + mean_b * mean_b;
  double c = sqrt((double)vsum) + 0.3 * sqrt((double)msum);
  return (float)c;
}

/* combined.diff:153-181 */
float jxo_homogeneity(const jxo_xyb* img, size_t x, size_t y, size_t xs,
                      size_t ys, size_t bx, size_t by, float distance,
                      int h1_mode) {
  float L[64];
  laplacian(img, x, y, xs, ys, bx, by, L);
  float t = 0.25f;
  if ((double)distance > 10.0) {
    t = 0.40f;
  } else if ((double)distance <= 2.0) {
    t = 0.15f;
  }
  size_t nc = zero_crossings(xs, ys, t, L);
  float sml = sum_modified_laplacian(img, x, y, xs, ys, bx, by, h1_mode);
  float col = colorfulness(img, x, y, xs, ys, bx, by);
  return ((float)nc + sml) + col;
}

static inline float fmax_std(float a, float b) { return (a < b) ? b : a; }
static inline float fmin_std(float a, float b) { return (b < a) ? b : a; }

/* combined.diff:183-211 (operator precedence of :200-203 kept as written) */
void jxo_homog_indices(const jxo_xyb* img, size_t x, size_t y, float distance,
                       int h1_mode, float* r_h, float* r_v, float* r_d) {
  float h1 = jxo_homogeneity(img, x, y, 8, 4, 0, 0, distance, h1_mode);
  float h2 = jxo_homogeneity(img, x, y, 8, 4, 0, 4, distance, h1_mode);
  float v1 = jxo_homogeneity(img, x, y, 4, 8, 0, 0, distance, h1_mode);
  float v2 = jxo_homogeneity(img, x, y, 4, 8, 4, 0, distance, h1_mode);
  float d1 = jxo_homogeneity(img, x, y, 4, 4, 0, 0, distance, h1_mode) +
             jxo_homogeneity(img, x, y, 4, 4, 4, 4, distance, h1_mode) / 2.0f;
  float d2 = jxo_homogeneity(img, x, y, 4, 4, 0, 4, distance, h1_mode) +
             jxo_homogeneity(img, x, y, 4, 4, 4, 0, distance, h1_mode) / 2.0f;
  *r_h = fmax_std(h1, h2) / fmin_std(h1, h2);
  *r_v = fmax_std(v1, v2) / fmin_std(v1, v2);
  *r_d = fmax_std(d1, d2) / fmin_std(d1, d2);
}

/* combined.diff:213-235 */
static uint8_t partition_from_r(float r_h, float r_v, float r_d,
                                float distance) {
  float T = 1.60f;
  if ((double)distance > 10.0) {
    T = 1.80f;
  } else if ((double)distance <= 3.0) {
    T = 1.50f;
  }
  if (r_d > T) return JXO_DCT4X4;
  if (r_h > r_v && r_h > T) return JXO_DCT8X4;
  if (r_v > r_h && r_v > T) return JXO_DCT4X8;
  return JXO_DCT8;
}

uint8_t jxo_homog_partition(const jxo_xyb* img, size_t x, size_t y,
                            float distance, int h1_mode) {
  float r_h, r_v, r_d;
  jxo_homog_indices(img, x, y, distance, h1_mode, &r_h, &r_v, &r_d);
  return partition_from_r(r_h, r_v, r_d, distance);
}

/* combined.diff:247-253: avg_r in float, ret*0.8*avg_r in double */
float jxo_hook_f(float ret, float r_h, float r_v, float r_d) {
  float avg_r = (r_h + r_v + r_d) / 3.0f;
  return (float)((double)ret * 0.8 * (double)avg_r);
}

void jxo_homog_map(const jxo_xyb* img, float distance, int h1_mode, float* r3,
                   uint8_t* type) {
  size_t bxs = img->xsize / 8, bys = img->ysize / 8;
#pragma omp parallel for schedule(dynamic)
  for (size_t by = 0; by < bys; by++) {
    for (size_t bx = 0; bx < bxs; bx++) {
      size_t b = by * bxs + bx;
      float rh, rv, rd;
      jxo_homog_indices(img, bx * 8, by * 8, distance, h1_mode, &rh, &rv, &rd);
      if (r3) {
        r3[3 * b + 0] = rh;
        r3[3 * b + 1] = rv;
        r3[3 * b + 2] = rd;
      }
      if (type) type[b] = partition_from_r(rh, rv, rd, distance);
    }
  }
}
