// jxg_front.hip -- fused front end of the VarDCT encode on gfx950:
//   RGB8 -> linear -> XYB (LDS tile + 1 px halo, never written to HBM)
//   -> thesis homogeneity indices per 8x8 block (proposals/combined.diff:17-211)
//   -> block DC + adaptive quantization
//   -> AC-strategy search over the 8x8-class transforms with hooks F
//      (combined.diff:247-253) and P (:270-274)
//   -> forward transform, CfL residual, quantization -> int32 coefficients
//      ([block][X,Y,B][64 zigzag]), quantized DC, strategy, quant field.
//
// One 256-thread workgroup per 64x64 pixel tile (8x8 blocks).
// Transform/quantization work is done by 8-lane groups: lane r of a group owns
// pixel row r for the row pass and working-array column r for the column pass
// (transpose through a per-group LDS scratch), so each lane carries 8 values
// per channel instead of a whole block.  A wave runs 8 blocks of one block
// row with one (wave-uniform) candidate strategy at a time.
// Float op order == oracle/front.c (see jxo_quantize_block's sum order).
#include <float.h>

#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

__constant__ float c_lut[256];
__constant__ float c_wts[3][3][64];  // [quant kind][channel X,Y,B][raster k]

constexpr int kTile = 64;
constexpr int kRows = 66;  // 64 + halo above/below
constexpr int kW = 72;     // LDS row stride; pixel column gx maps to gx - (tile_x0 - kOff)
constexpr int kOff = 4;    // interior column 0 at LDS column 4 (16-B aligned)
constexpr int kXbuf = 8 * 9;  // per-group transpose scratch (8 x 9 floats)

// ---------------------------------------------------------------------------
// thesis homogeneity (combined.diff:17-181) on the LDS tile
// ---------------------------------------------------------------------------
struct Tile {
  const float* X;
  const float* Y;
  const float* B;
  int ox, oy;  // padded-frame coordinate of LDS (0,0)
  __device__ __forceinline__ float at(const float* p, int gx, int gy) const {
    return p[(gy - oy) * kW + (gx - ox)];
  }
};

// Laplacian sample (combined.diff:57-81): 3x3 mask on Y, k-outer/l-inner order
// with the zero taps dropped (they add +-0 and never change the sum)
__device__ __forceinline__ float lap(const Tile& t, int px, int py) {
  float sum = 0.0f;
  sum += t.at(t.Y, px, py - 1) * -1.0f;
  sum += t.at(t.Y, px - 1, py) * -1.0f;
  sum += t.at(t.Y, px, py) * -4.0f;
  sum += t.at(t.Y, px + 1, py) * -1.0f;
  sum += t.at(t.Y, px, py + 1) * -1.0f;
  return sum;
}

// The Laplacian is recomputed for the column walk instead of being kept in a
// per-lane array (identical values; keeps the function register-light).
template <int XS, int YS>
__device__ float homogeneity(const Tile& t, int x, int y, int bx, int by, float dist,
                             int ysize, int h1_int) {
  float thr = 0.25f;
  if ((double)dist > 10.0)
    thr = 0.40f;
  else if ((double)dist <= 2.0)
    thr = 0.15f;
  const int x0 = x + bx, y0 = y + by;
  uint32_t nh = 0;
#pragma unroll 1
  for (int i = 0; i < YS; i++) {
    bool in_edge = false;
#pragma unroll
    for (int j = 0; j < XS; j++) {
      const float v = lap(t, x0 + j, y0 + i);
      if (!in_edge && v > thr) {
        nh++;
        in_edge = true;
      } else if (in_edge && v <= thr) {
        in_edge = false;
      }
    }
  }
  const float avg_h = (float)nh / (float)YS;
  uint32_t nv = 0;
#pragma unroll 1
  for (int i = 0; i < XS; i++) {
    bool in_edge = false;
#pragma unroll
    for (int j = 0; j < YS; j++) {
      const float v = lap(t, x0 + i, y0 + j);
      if (!in_edge && v > thr) {
        nv++;
        in_edge = true;
      } else if (in_edge && v <= thr) {
        in_edge = false;
      }
    }
  }
  const float avg_v = (float)nv / (float)XS;
  const uint32_t nc = (uint32_t)(avg_h + avg_v);
  float sml = 0.0f;
#pragma unroll 1
  for (int i = 0; i < YS; i++)
#pragma unroll
    for (int j = 0; j < XS; j++) {
      const int px = x + bx + j, py = y + by + i;
      if (py + 1 >= ysize) continue;
      const float p = t.at(t.Y, px, py);
      const float l = t.at(t.Y, px - 1, py);
      const float r = t.at(t.Y, px + 1, py);
      const float u = t.at(t.Y, px, py - 1);
      const float d = t.at(t.Y, px, py + 1);
      const float a = 2.0f * p - l - r;
      const float b = 2.0f * p - u - d;
      if (h1_int) {
        int ia = abs((int)a), ib = abs((int)b);
        sml += (float)(ia + ib);
      } else {
        sml += fabsf(a) + fabsf(b);
      }
    }
  const float n = (float)(XS * YS);
  float mx = 0.0f, mb = 0.0f;
#pragma unroll 1
  for (int i = 0; i < YS; i++)
#pragma unroll
    for (int j = 0; j < XS; j++) mx += t.at(t.X, x + bx + j, y + by + i);
  mx /= n;
#pragma unroll 1
  for (int i = 0; i < YS; i++)
#pragma unroll
    for (int j = 0; j < XS; j++) mb += t.at(t.B, x + bx + j, y + by + i);
  mb /= n;
  float vx = 0.0f, vb = 0.0f;
#pragma unroll 1
  for (int i = 0; i < YS; i++)
#pragma unroll
    for (int j = 0; j < XS; j++) {
      const float diff = t.at(t.X, x + bx + j, y + by + i) - mx;
      vx += diff * diff;
    }
  vx /= n;
#pragma unroll 1
  for (int i = 0; i < YS; i++)
#pragma unroll
    for (int j = 0; j < XS; j++) {
      const float diff = t.at(t.B, x + bx + j, y + by + i) - mb;
      vb += diff * diff;
    }
  vb /= n;
  const float vsum = vx + vb;
  const float msum = mx * mx + mb * mb;
  const double col = sqrt((double)vsum) + 0.3 * sqrt((double)msum);
  return ((float)nc + sml) + (float)col;
}

// region r of CalculateHomogeneitySimilarityIndices (combined.diff:189-204):
// 0 h1(8,4,0,0) 1 h2(8,4,0,4) 2 v1(4,8,0,0) 3 v2(4,8,4,0)
// 4 (4,4,0,0) 5 (4,4,4,4) 6 (4,4,0,4) 7 (4,4,4,0)
__device__ float homog_region(const Tile& t, int r, int x, int y, float dist, int ysize,
                              int h1) {
  switch (r) {
    case 0: return homogeneity<8, 4>(t, x, y, 0, 0, dist, ysize, h1);
    case 1: return homogeneity<8, 4>(t, x, y, 0, 4, dist, ysize, h1);
    case 2: return homogeneity<4, 8>(t, x, y, 0, 0, dist, ysize, h1);
    case 3: return homogeneity<4, 8>(t, x, y, 4, 0, dist, ysize, h1);
    case 4: return homogeneity<4, 4>(t, x, y, 0, 0, dist, ysize, h1);
    case 5: return homogeneity<4, 4>(t, x, y, 4, 4, dist, ysize, h1);
    case 6: return homogeneity<4, 4>(t, x, y, 0, 4, dist, ysize, h1);
    default: return homogeneity<4, 4>(t, x, y, 4, 0, dist, ysize, h1);
  }
}

__device__ __forceinline__ float fmax_std(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float fmin_std(float a, float b) { return (b < a) ? b : a; }

__device__ __forceinline__ void similarity(const float* h, float& rh, float& rv, float& rd) {
  const float d1 = h[4] + h[5] / 2.0f;
  const float d2 = h[6] + h[7] / 2.0f;
  rh = fmax_std(h[0], h[1]) / fmin_std(h[0], h[1]);
  rv = fmax_std(h[2], h[3]) / fmin_std(h[2], h[3]);
  rd = fmax_std(d1, d2) / fmin_std(d1, d2);
}

__device__ __forceinline__ uint8_t partition_of(float rh, float rv, float rd, float dist) {
  float T = 1.60f;
  if ((double)dist > 10.0)
    T = 1.80f;
  else if ((double)dist <= 3.0)
    T = 1.50f;
  if (rd > T) return kDCT4X4;
  if (rh > rv && rh > T) return kDCT8X4;
  if (rv > rh && rv > T) return kDCT4X8;
  return kDCT8;
}

// ---------------------------------------------------------------------------
// 1-D DCT-II (out[0] = mean), fixed even/odd butterfly; op sequence and hex
// constants are those of oracle/front.c (dct8_1d / dct4_1d).
// ---------------------------------------------------------------------------
constexpr float kA = 0x1.63150cp-3f, kB = 0x1.2d062ep-3f, kC = 0x1.92469cp-4f,
                kD = 0x1.1a855ep-5f, kE1 = 0x1.4e7aeap-3f, kE3 = 0x1.1517a8p-4f,
                kF1 = 0x1.4e7aeap-2f, kF3 = 0x1.1517a8p-3f;

__device__ __forceinline__ void dct8_1d(float* v) {
  const float x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3], x4 = v[4], x5 = v[5], x6 = v[6],
              x7 = v[7];
  const float s0 = x0 + x7, s1 = x1 + x6, s2 = x2 + x5, s3 = x3 + x4;
  const float d0 = x0 - x7, d1 = x1 - x6, d2 = x2 - x5, d3 = x3 - x4;
  const float a0 = s0 + s3, a1 = s1 + s2, b0 = s0 - s3, b1 = s1 - s2;
  v[0] = (a0 + a1) * 0.125f;
  v[4] = (a0 - a1) * 0.125f;
  v[2] = fmaf(b1, kE3, b0 * kE1);
  v[6] = fmaf(b1, -kE1, b0 * kE3);
  v[1] = fmaf(d3, kD, fmaf(d2, kC, fmaf(d1, kB, d0 * kA)));
  v[3] = fmaf(d3, -kC, fmaf(d2, -kA, fmaf(d1, -kD, d0 * kB)));
  v[5] = fmaf(d3, kB, fmaf(d2, kD, fmaf(d1, -kA, d0 * kC)));
  v[7] = fmaf(d3, -kA, fmaf(d2, kB, fmaf(d1, -kC, d0 * kD)));
}
__device__ __forceinline__ void dct4_1d(float* v) {
  const float x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3];
  const float s0 = x0 + x3, s1 = x1 + x2, d0 = x0 - x3, d1 = x1 - x2;
  v[0] = (s0 + s1) * 0.25f;
  v[2] = (s0 - s1) * 0.25f;
  v[1] = fmaf(d1, kF3, d0 * kF1);
  v[3] = fmaf(d1, -kF1, d0 * kF3);
}

// working-array element p = prow*8 + pcol -> raster position in the
// coefficient layout of strategy T (oracle co_index)
template <int T>
__device__ __forceinline__ int co_index(int prow, int pcol) {
  if (T == kDCT8) return prow * 8 + pcol;
  if (T == kDCT4X4) return ((prow >> 2) + 2 * (prow & 3)) * 8 + (pcol >> 2) + 2 * (pcol & 3);
  if (T == kDCT8X4) return ((prow >> 2) + 2 * (prow & 3)) * 8 + pcol;
  return ((pcol >> 2) + 2 * (pcol & 3)) * 8 + prow;
}

template <int T>
constexpr int qkind() {
  return T == kDCT8 ? 0 : (T == kDCT4X4 ? 1 : 2);
}

__device__ __forceinline__ float adjust_bias_y(int q) {
  const float kBias1 = 1.0f - 0.07005449891748593f;
  if (q == 0) return 0.0f;
  if (q == 1) return kBias1;
  if (q == -1) return -kBias1;
  return (float)q - 0.145f / (float)q;
}
__device__ __forceinline__ int quant1(float v) {
  const float a = fabsf(v);
  if (a < 0.58f) return 0;
  int q = (int)(a + 0.5f);
  if (q > (1 << 24)) q = 1 << 24;
  return v < 0.0f ? -q : q;
}
__device__ __forceinline__ int bitlen(uint32_t v) { return v ? 32 - __clz(v) : 0; }

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// One 8-lane group quantizes one block under strategy T (channels Y, X, B).
//   src   : LDS address of the block's top-left pixel in plane X (planes are
//           kPlane floats apart), row stride kW
//   r     : lane within the group (0..7), g0 = lane index of the group's lane 0
//   xb    : the group's transpose scratch (kXbuf floats)
//   wts   : LDS copy of c_wts
//   out   : [X,Y,B][64 zigzag] ints of this block, or nullptr
// Returns the rate/distortion cost (identical in all 8 lanes).
constexpr int kPlane = kRows * kW;
template <int T>
__device__ float quantize_group(const float* src, int r, int g0, float* xb,
                                const float* wts, float scale, int32_t* out,
                                const uint8_t* inv_order) {
  constexpr int qk = qkind<T>();
  float yd[8];
  int bits = 0;
  float dist = 0.0f;
#pragma unroll
  for (int ci = 0; ci < 3; ci++) {
    const int c = ci == 0 ? 1 : (ci == 1 ? 0 : 2);
    float v[8];
    const float* row = src + c * kPlane + r * kW;
    const float4 lo = *reinterpret_cast<const float4*>(row);
    const float4 hi = *reinterpret_cast<const float4*>(row + 4);
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    // row pass
    if (T == kDCT8 || T == kDCT8X4) {
      dct8_1d(v);
    } else {
      dct4_1d(v);
      dct4_1d(v + 4);
    }
    // transpose: lane r gets working-array column r
#pragma unroll
    for (int x = 0; x < 8; x++) xb[r * 9 + x] = v[x];
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = xb[k * 9 + r];
    wave_lds_sync();
    // column pass
    if (T == kDCT8 || T == kDCT4X8) {
      dct8_1d(v);
    } else {
      dct4_1d(v);
      dct4_1d(v + 4);
    }
    // lowest-frequency combine (enc_transforms [ext]); slots per oracle
    if (T == kDCT4X4) {
      const float A = __shfl(v[0], g0), C = __shfl(v[4], g0);
      const float B = __shfl(v[0], g0 + 4), D = __shfl(v[4], g0 + 4);
      if (r == 0) {
        v[0] = (((A + B) + C) + D) * 0.25f;
        v[4] = (((A - B) + C) - D) * 0.25f;
      } else if (r == 4) {
        v[0] = (((A + B) - C) - D) * 0.25f;
        v[4] = (((A - B) - C) + D) * 0.25f;
      }
    } else if (T == kDCT8X4) {
      if (r == 0) {
        const float A = v[0], B = v[4];
        v[0] = (A + B) * 0.5f;
        v[4] = (A - B) * 0.5f;
      }
    } else if (T == kDCT4X8) {
      const float A = __shfl(v[0], g0), B = __shfl(v[0], g0 + 4);
      if (r == 0) v[0] = (A + B) * 0.5f;
      if (r == 4) v[0] = (A - B) * 0.5f;
    }
    // quantize the 8 coefficients of working column r
    int nz = 0;
    float part = 0.0f;
    int32_t q[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int co = co_index<T>(k, r);
      q[k] = 0;
      if (co == 0) continue;
      const float ws = wts[(qk * 3 + c) * 64 + co] * scale;
      float rv = v[k];
      if (c == 2) rv = rv - yd[k];
      const float vq = rv * ws;
      const int qq = quant1(vq);
      if (c == 1) yd[k] = adjust_bias_y(qq) / ws;
      const uint32_t aq = (uint32_t)(qq < 0 ? -qq : qq);
      const float e = fabsf(vq) - (float)aq;
      part += e * e;
      if (aq) {
        bits += 2 + 2 * bitlen(aq);
        nz++;
      }
      q[k] = qq;
    }
    // lane partials in lane order (oracle: dch += part for r = 0..7)
    float dch = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; i++) dch += __shfl(part, g0 + i);
    dist += dch;
    int nzc = nz;
#pragma unroll
    for (int i = 1; i < 8; i <<= 1) nzc += __shfl_xor(nzc, i);
    bits += bitlen((uint32_t)nzc) * (r == 0 ? 1 : 0);
    if (out) {
#pragma unroll
      for (int k = 0; k < 8; k++) out[c * 64 + inv_order[co_index<T>(k, r)]] = q[k];
    }
  }
  // bits: per-lane coefficient terms + lane 0's nz terms -> group total
#pragma unroll
  for (int i = 1; i < 8; i <<= 1) bits += __shfl_xor(bits, i);
  const float tmul = T == kDCT8 ? 1.0f : (T == kDCT4X4 ? 1.05f : 1.02f);
  return ((float)bits + 8.0f * dist) * tmul;
}

__device__ float hook_f(float ret, float rh, float rv, float rd) {
  const float avg_r = (rh + rv + rd) / 3.0f;
  return (float)((double)ret * 0.8 * (double)avg_r);
}

template <int T>
__device__ __forceinline__ float run_group(const float* sPix, int lbx, int lby, int r, int g0,
                                           float* xb, const float* wts, float scale,
                                           int32_t* out, const uint8_t* inv_order) {
  const float* src = sPix + (lby * 8 + 1) * kW + kOff + lbx * 8;
  return quantize_group<T>(src, r, g0, xb, wts, scale, out, inv_order);
}

__global__ __launch_bounds__(256) void front_kernel(FrontArgs a) {
  __shared__ __attribute__((aligned(16))) float sPix[3 * kPlane];  // X, Y, B planes
  __shared__ float sLut[256];
  __shared__ float sWts[3 * 3 * 64];
  __shared__ float sXb[32][kXbuf];  // one transpose scratch per 8-lane group
  __shared__ uint8_t sInv[64];
  __shared__ float sH[8][64];
  __shared__ float sR[64][3];
  __shared__ float sCost[4][64];
  __shared__ int sRaw[64];
  __shared__ int sAcs[64];
  const int tid = threadIdx.x;
  const int tx = blockIdx.x, ty = blockIdx.y;
  const int ox = tx * kTile - kOff, oy = ty * kTile - 1;
  sLut[tid] = c_lut[tid];
  for (int i = tid; i < 576; i += 256) sWts[i] = (&c_wts[0][0][0])[i];
  if (tid < 64) sInv[tid] = (uint8_t)c_inv_order_h(tid);
  __syncthreads();
  float* const sX = sPix;
  float* const sY = sPix + kPlane;
  float* const sB = sPix + 2 * kPlane;
  const float cb = cbrt_det(kOpsinBias);
  for (int i = tid; i < kRows * 66; i += 256) {
    const int ly = i / 66, lx = i - ly * 66 + (kOff - 1);
    const int gx = ox + lx, gy = oy + ly;
    float X = 0.0f, Y = 0.0f, B = 0.0f;
    if (gx >= 0 && gy >= 0 && gx < (int)a.xp && gy < (int)a.yp) {
      const int sx = gx < (int)a.w ? gx : (int)a.w - 1;
      const int sy = gy < (int)a.h ? gy : (int)a.h - 1;
      const uint8_t* p = a.rgb + (size_t)sy * a.stride + 3 * (size_t)sx;
      pixel_xyb(sLut, cb, p[0], p[1], p[2], X, Y, B);
    }
    sX[ly * kW + lx] = X;
    sY[ly * kW + lx] = Y;
    sB[ly * kW + lx] = B;
  }
  __syncthreads();
  const int nbx = min(8, (int)a.bxs - tx * 8), nby = min(8, (int)a.bys - ty * 8);
  const int wave = tid >> 6, lane = tid & 63;
  const size_t nb = (size_t)a.bxs * a.bys;
  const Tile tile{sX, sY, sB, ox, oy};
  // ---- phase A: thesis homogeneity (lane = block, wave-uniform region) ----
  if (a.proposals & 3u) {
    const int lbx = lane & 7, lby = lane >> 3;
    const bool valid = lbx < nbx && lby < nby;
    const int gx0 = tx * kTile + lbx * 8, gy0 = ty * kTile + lby * 8;
#pragma unroll 1
    for (int rr = 0; rr < 2; rr++) {
      const int r = wave + rr * 4;
      if (valid) sH[r][lane] = homog_region(tile, r, gx0, gy0, a.distance, (int)a.yp, a.h1_int);
    }
    __syncthreads();
    if (tid < 64 && valid) {
      float h[8];
#pragma unroll
      for (int r = 0; r < 8; r++) h[r] = sH[r][lane];
      float rh, rv, rd;
      similarity(h, rh, rv, rd);
      sR[lane][0] = rh;
      sR[lane][1] = rv;
      sR[lane][2] = rd;
      if (a.homog) {
        const size_t gb = (size_t)(ty * 8 + lby) * a.bxs + tx * 8 + lbx;
        a.homog[gb * 3 + 0] = rh;
        a.homog[gb * 3 + 1] = rv;
        a.homog[gb * 3 + 2] = rd;
      }
    }
  }
  // ---- phase B: block DC and adaptive quantization (lane = block) ----
  if (tid < 64) {
    const int lbx = lane & 7, lby = lane >> 3;
    if (lbx < nbx && lby < nby) {
      const size_t gb = (size_t)(ty * 8 + lby) * a.bxs + tx * 8 + lbx;
      const int base = (lby * 8 + 1) * kW + kOff + lbx * 8;
      float dc[3];
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const float* pl = sPix + c * kPlane + base;
        float s = 0.0f;
#pragma unroll
        for (int y = 0; y < 8; y++)
#pragma unroll
          for (int x = 0; x < 8; x++) s += pl[y * kW + x];
        dc[c] = s * (1.0f / 64.0f);
      }
      const float vy = dc[1] * a.dc_mul[1];
      const int qy = vy >= 0.0f ? (int)(vy + 0.5f) : -(int)(-vy + 0.5f);
      const float ydq = (float)qy * a.dc_step[1];
      const float xv = dc[0] * a.dc_mul[0];
      const float bv = (dc[2] - ydq) * a.dc_mul[2];
      a.dc[nb + gb] = qy;
      a.dc[gb] = xv >= 0.0f ? (int)(xv + 0.5f) : -(int)(-xv + 0.5f);
      a.dc[2 * nb + gb] = bv >= 0.0f ? (int)(bv + 0.5f) : -(int)(-bv + 0.5f);
      const float* Yp = sY + base;
      float act = 0.0f;
#pragma unroll
      for (int y = 0; y < 8; y++)
#pragma unroll
        for (int x = 0; x < 7; x++) act += fabsf(Yp[y * kW + x + 1] - Yp[y * kW + x]);
#pragma unroll
      for (int y = 0; y < 7; y++)
#pragma unroll
        for (int x = 0; x < 8; x++) act += fabsf(Yp[(y + 1) * kW + x] - Yp[y * kW + x]);
      const float am = act * (1.0f / 112.0f);
      float mult = 1.5f / sqrtf(1.0f + am * 40.0f);
      if (mult < 0.45f) mult = 0.45f;
      if (mult > 1.5f) mult = 1.5f;
      const float qff = a.qf_base * mult;
      int raw = (int)(qff * a.inv_g + 0.5f);
      raw = raw < 1 ? 1 : (raw > 256 ? 256 : raw);
      sRaw[lane] = raw;
    }
  }
  __syncthreads();
  // ---- phase C: candidate costs.  8-lane groups: group gi (0..7) of a wave
  // handles block column lbx = gi; the wave walks block rows. ----
  const int gi = lane >> 3, r = lane & 7, g0 = lane & ~7;
  float* xb = sXb[wave * 8 + gi];
  const int ncand = a.effort >= 5 ? 4 : 1;
  const int lbx = gi;
  // DCT8 is always evaluated; its coefficients are written right away (most
  // blocks keep it) and overwritten below for blocks that switch.
#pragma unroll 1
  for (int lby = wave; lby < 8; lby += 4) {
    const bool valid = lbx < nbx && lby < nby;
    if (!valid) continue;
    const int b = lby * 8 + lbx;
    const float scale = (float)a.G * (float)sRaw[b] / 65536.0f;
    const size_t gb = (size_t)(ty * 8 + lby) * a.bxs + tx * 8 + lbx;
    const float e = run_group<kDCT8>(sPix, lbx, lby, r, g0, xb, sWts, scale, a.ac + gb * 192, sInv);
    if (r == 0) sCost[0][b] = e;
    if (ncand > 1) {
      const float e1 = run_group<kDCT4X4>(sPix, lbx, lby, r, g0, xb, sWts, scale, nullptr, sInv);
      const float e2 = run_group<kDCT4X8>(sPix, lbx, lby, r, g0, xb, sWts, scale, nullptr, sInv);
      const float e3 = run_group<kDCT8X4>(sPix, lbx, lby, r, g0, xb, sWts, scale, nullptr, sInv);
      if (r == 0) {
        sCost[1][b] = e1;
        sCost[2][b] = e2;
        sCost[3][b] = e3;
      }
    }
  }
  __syncthreads();
  // ---- phase D: selection + hooks (lane = block) ----
  if (tid < 64) {
    const int bx_ = lane & 7, by_ = lane >> 3;
    if (bx_ < nbx && by_ < nby) {
      const int cand[4] = {kDCT8, kDCT4X4, kDCT4X8, kDCT8X4};
      int best_t = kDCT8;
      if (ncand > 1) {
        float best = FLT_MAX;
        for (int i = 0; i < ncand; i++) {
          float e = sCost[i][lane];
          if (a.proposals & 2u) e = hook_f(e, sR[lane][0], sR[lane][1], sR[lane][2]);
          if (e < best) {
            best = e;
            best_t = cand[i];
          }
        }
      }
      if ((a.proposals & 1u) && best_t == kDCT8)
        best_t = partition_of(sR[lane][0], sR[lane][1], sR[lane][2], a.distance);
      sAcs[lane] = best_t;
      const size_t gb = (size_t)(ty * 8 + by_) * a.bxs + tx * 8 + bx_;
      a.acs[gb] = (uint8_t)best_t;
      a.qf[gb] = (uint8_t)(sRaw[lane] - 1);
    }
  }
  __syncthreads();
  // ---- phase E: final coefficients for blocks that left DCT8 ----
#pragma unroll 1
  for (int lby = wave; lby < 8; lby += 4) {
    const bool valid = lbx < nbx && lby < nby;
    const int b = lby * 8 + lbx;
    const int t = valid ? sAcs[b] : kDCT8;
    if (t == kDCT8) continue;
    const float scale = (float)a.G * (float)sRaw[b] / 65536.0f;
    int32_t* out = a.ac + ((size_t)(ty * 8 + lby) * a.bxs + tx * 8 + lbx) * 192;
    if (t == kDCT4X4)
      run_group<kDCT4X4>(sPix, lbx, lby, r, g0, xb, sWts, scale, out, sInv);
    else if (t == kDCT4X8)
      run_group<kDCT4X8>(sPix, lbx, lby, r, g0, xb, sWts, scale, out, sInv);
    else
      run_group<kDCT8X4>(sPix, lbx, lby, r, g0, xb, sWts, scale, out, sInv);
  }
}

// standalone thesis selector over a given XYB frame (parity entry point)
__global__ __launch_bounds__(256) void homog_kernel(HomogArgs a) {
  __shared__ float sPix[3 * kPlane];
  __shared__ float sH[8][64];
  const int tid = threadIdx.x;
  const int tx = blockIdx.x, ty = blockIdx.y;
  const int ox = tx * kTile - kOff, oy = ty * kTile - 1;
  for (int i = tid; i < kRows * 66; i += 256) {
    const int ly = i / 66, lx = i - ly * 66 + (kOff - 1);
    const int gx = ox + lx, gy = oy + ly;
    const bool in = gx >= 0 && gy >= 0 && gx < (int)a.xsize && gy < (int)a.ysize;
    const size_t o = (size_t)gy * a.stride + gx;
    sPix[ly * kW + lx] = in ? a.xyb[o] : 0.0f;
    sPix[kPlane + ly * kW + lx] = in ? a.xyb[a.plane + o] : 0.0f;
    sPix[2 * kPlane + ly * kW + lx] = in ? a.xyb[2 * a.plane + o] : 0.0f;
  }
  __syncthreads();
  const int bxs = (int)a.xsize / 8, bys = (int)a.ysize / 8;
  const int wave = tid >> 6, lane = tid & 63;
  const int lbx = lane & 7, lby = lane >> 3;
  const bool valid = tx * 8 + lbx < bxs && ty * 8 + lby < bys;
  const Tile tile{sPix, sPix + kPlane, sPix + 2 * kPlane, ox, oy};
  const int gx0 = tx * kTile + lbx * 8, gy0 = ty * kTile + lby * 8;
#pragma unroll 1
  for (int rr = 0; rr < 2; rr++) {
    const int r = wave + rr * 4;
    if (valid) sH[r][lane] = homog_region(tile, r, gx0, gy0, a.distance, (int)a.ysize, a.h1_int);
  }
  __syncthreads();
  if (tid < 64 && valid) {
    float h[8];
#pragma unroll
    for (int r = 0; r < 8; r++) h[r] = sH[r][lane];
    float rh, rv, rd;
    similarity(h, rh, rv, rd);
    const size_t b = (size_t)(ty * 8 + lby) * bxs + tx * 8 + lbx;
    a.r3[b * 3 + 0] = rh;
    a.r3[b * 3 + 1] = rv;
    a.r3[b * 3 + 2] = rd;
    a.type[b] = partition_of(rh, rv, rd, a.distance);
  }
}

void set_front_constants(const float lut[256], const float wts[3][3][64], hipStream_t s) {
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(c_lut), lut, sizeof(float) * 256, 0,
                               hipMemcpyHostToDevice, s);
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(c_wts), wts, sizeof(float) * 576, 0,
                               hipMemcpyHostToDevice, s);
}
void launch_front(const FrontArgs& a, uint32_t tiles_x, uint32_t tiles_y, hipStream_t s) {
  hipLaunchKernelGGL(front_kernel, dim3(tiles_x, tiles_y), dim3(256), 0, s, a);
}
void launch_homog(const HomogArgs& a, uint32_t tiles_x, uint32_t tiles_y, hipStream_t s) {
  hipLaunchKernelGGL(homog_kernel, dim3(tiles_x, tiles_y), dim3(256), 0, s, a);
}

}  // namespace jxg
