// jxg_front.hip -- fused front end of the VarDCT encode on gfx950:
//   RGB8 -> linear -> XYB (LDS tile + 1 px halo, never written to HBM)
//   -> thesis homogeneity indices per 8x8 block (proposals/combined.diff:17-211)
//   -> block DC + adaptive quantization
//   -> AC-strategy search over the 8x8-class transforms with hooks F
//      (combined.diff:247-253) and P (:270-274)
//   -> forward transform, CfL residual, quantization -> int16 coefficients
//      ([block][X,Y,B][64 zigzag]), quantized DC, strategy, quant field.
//
// One 512-thread workgroup (8 waves) per 64x64 pixel tile; wave w owns block
// row w.  Within a wave, 8-lane group g owns block column g and lane r owns
// pixel row r for the row butterfly, then (after an in-register XOR-butterfly
// transpose) working-array column r for the column butterfly and the
// quantization of its 8 coefficients.  The candidate strategy is
// wave-uniform.  The LDS tile uses a one-dword skew per 8-pixel block column
// (row stride 75) so both the lane = block phase and the lane = row phase are
// (nearly) bank-conflict free.  Float op order == oracle/front.c.
#include <float.h>

#include <cstdio>

#include <type_traits>

#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

__constant__ float c_lut[256];
// per-lane quantization tables, built on the host from the weights
// (T: table index tindex -- DCT8, DCT4X4, DCT4X8, DCT8X4, DCT2X2, IDENTITY)
constexpr int kNT = 6;
__constant__ float c_wperm[kNT * 3 * 64];  // [T][c][lane r][row k] = w[qkind(T)][c][co_index(T,k,r)]
__constant__ float c_iwperm[kNT * 64];     // [T][r][k] = 1.0f / (Y weight) at the same slot
__constant__ float c_sdperm[kNT * 3 * 64]; // [T][c][r][k] distortion weight at the same slot
__constant__ float c_btab[256];            // [q] = AdjustQuantBias of a magnitude q < 256 (host table: 0, 1 - 0.0700..., q - 0.145 / q)
__constant__ uint8_t c_zz[kNT * 64];       // [T][r][k] = zigzag index of co_index(T,k,r)

constexpr int kTile = 64;
constexpr int kRows = 66;           // 64 + halo above/below
constexpr int kS = 75;              // LDS row stride (floats)
constexpr int kPlane = kRows * kS;  // floats per XYB plane
constexpr int kThreads = 512;

// LDS offset of tile-local pixel (lx, ly), lx/ly in [0, 66): one dword of
// skew per interior 8-pixel block column
// (round 6 measured a stride-67 layout without the skew, which the bank
// model gives conflict-free row reads: front kernel -1 %, e4 -0.6 %, but the
// lane = block reads of the thesis homogeneity phase become 8-way conflicted:
// not kept, profiles/r06h)
__device__ __forceinline__ int lds_at(int lx, int ly) { return ly * kS + lx + ((lx + 7) >> 3); }

// ---------------------------------------------------------------------------
// thesis homogeneity (combined.diff:17-181) on the LDS tile
// ---------------------------------------------------------------------------
struct Tile {
  const float* X;
  const float* Y;
  const float* B;
  int ox, oy;  // padded-frame coordinate of tile-local (0,0)
  __device__ __forceinline__ float at(const float* p, int gx, int gy) const {
    return p[lds_at(gx - ox, gy - oy)];
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

// edge threshold of CalculateHomogeneity (combined.diff:163-168)
__device__ __forceinline__ float edge_threshold(float dist) {
  float thr = 0.25f;
  if ((double)dist > 10.0)
    thr = 0.40f;
  else if ((double)dist <= 2.0)
    thr = 0.15f;
  return thr;
}

// The tile's (Laplacian > threshold) map, one 64-bit word per interior row
// (bit k = column k): wave w evaluates rows w, w + 8, ... with lane = column
// and one ballot per row.  Every region of every block then counts its zero
// crossings from these words instead of re-walking the Laplacian.
__device__ __forceinline__ void lap_bits(const Tile& t, float thr, uint64_t* bits) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int y = wave; y < 64; y += (int)(blockDim.x >> 6)) {
    const float v = lap(t, t.ox + 1 + lane, t.oy + 1 + y);
    const uint64_t b = __ballot(v > thr);
    if (lane == 0) bits[y] = b;
  }
}

// CalculateNumZeroCrossings (combined.diff:17-55) on the bit map: a crossing
// is an entry into L > t, i.e. a set bit whose predecessor along the row
// (column) inside the region is clear -- the walk's in_edge flag is exactly
// the previous entry's comparison (no NaN: L is a sum of finite samples).
template <int XS, int YS>
__device__ __forceinline__ float homogeneity(const Tile& t, const uint64_t* lbits, int x, int y,
                                             int bx, int by, float dist, int ysize, int h1_int) {
  (void)dist;
  const int x0 = x + bx, y0 = y + by;
  const int lx0 = x0 - (t.ox + 1), ly0 = y0 - (t.oy + 1);
  uint32_t nh = 0, nv = 0;
  uint32_t prev = 0;
#pragma unroll
  for (int i = 0; i < YS; i++) {
    const uint32_t r = (uint32_t)(lbits[ly0 + i] >> lx0) & ((1u << XS) - 1u);
    nh += __popc(r & ~(r << 1));
    nv += __popc(r & ~prev);
    prev = r;
  }
  const float avg_h = (float)nh / (float)YS;
  const float avg_v = (float)nv / (float)XS;
  const uint32_t nc = (uint32_t)(avg_h + avg_v);
  float sml = 0.0f;
#pragma unroll 1
  for (int i = 0; i < YS; i++)
#pragma unroll
    for (int j = 0; j < XS; j++) {
      const int px = x0 + j, py = y0 + i;
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
    for (int j = 0; j < XS; j++) mx += t.at(t.X, x0 + j, y0 + i);
  mx /= n;
#pragma unroll 1
  for (int i = 0; i < YS; i++)
#pragma unroll
    for (int j = 0; j < XS; j++) mb += t.at(t.B, x0 + j, y0 + i);
  mb /= n;
  float vx = 0.0f, vb = 0.0f;
#pragma unroll 1
  for (int i = 0; i < YS; i++)
#pragma unroll
    for (int j = 0; j < XS; j++) {
      const float diff = t.at(t.X, x0 + j, y0 + i) - mx;
      vx += diff * diff;
    }
  vx /= n;
#pragma unroll 1
  for (int i = 0; i < YS; i++)
#pragma unroll
    for (int j = 0; j < XS; j++) {
      const float diff = t.at(t.B, x0 + j, y0 + i) - mb;
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
// (one instantiation per region shape, the offsets at run time: r is
// wave-uniform, and eight inlined copies cost 9 KB of instruction cache)
__device__ __forceinline__ float homog_region(const Tile& t, const uint64_t* lb, int r, int x, int y,
                                              float dist, int ysize, int h1) {
  const int bx = (r == 3 || r == 5 || r == 7) ? 4 : 0;
  const int by = (r == 1 || r == 5 || r == 6) ? 4 : 0;
  if (r < 2) return homogeneity<8, 4>(t, lb, x, y, bx, by, dist, ysize, h1);
  if (r < 4) return homogeneity<4, 8>(t, lb, x, y, bx, by, dist, ysize, h1);
  return homogeneity<4, 4>(t, lb, x, y, bx, by, dist, ysize, h1);
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

// X and B go through the candidates together: f2 holds (X, B) of one
// element, and every float op of the pair is one packed VALU op (v_pk_*: each
// half is exactly the scalar op, no contraction) -- the per-channel float op
// sequence is unchanged, so the results stay bit-identical.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float vfma(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ f2 vfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
template <class V>
__device__ __forceinline__ V splat(float c) {
  if constexpr (std::is_same<V, float>::value) return c;
  else return f2{c, c};
}

template <class V>
__device__ __forceinline__ void dct8_1d(V* v) {
  const V x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3], x4 = v[4], x5 = v[5], x6 = v[6], x7 = v[7];
  const V s0 = x0 + x7, s1 = x1 + x6, s2 = x2 + x5, s3 = x3 + x4;
  const V d0 = x0 - x7, d1 = x1 - x6, d2 = x2 - x5, d3 = x3 - x4;
  const V a0 = s0 + s3, a1 = s1 + s2, b0 = s0 - s3, b1 = s1 - s2;
  const V cA = splat<V>(kA), cB = splat<V>(kB), cC = splat<V>(kC), cD = splat<V>(kD);
  v[0] = (a0 + a1) * splat<V>(0.125f);
  v[4] = (a0 - a1) * splat<V>(0.125f);
  v[2] = vfma(b1, splat<V>(kE3), b0 * splat<V>(kE1));
  v[6] = vfma(b1, splat<V>(-kE1), b0 * splat<V>(kE3));
  v[1] = vfma(d3, cD, vfma(d2, cC, vfma(d1, cB, d0 * cA)));
  v[3] = vfma(d3, -cC, vfma(d2, -cA, vfma(d1, -cD, d0 * cB)));
  v[5] = vfma(d3, cB, vfma(d2, cD, vfma(d1, -cA, d0 * cC)));
  v[7] = vfma(d3, -cA, vfma(d2, cB, vfma(d1, -cC, d0 * cD)));
}
template <class V>
__device__ __forceinline__ void dct4_1d(V* v) {
  const V x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3];
  const V s0 = x0 + x3, s1 = x1 + x2, d0 = x0 - x3, d1 = x1 - x2;
  v[0] = (s0 + s1) * splat<V>(0.25f);
  v[2] = (s0 - s1) * splat<V>(0.25f);
  v[1] = vfma(d1, splat<V>(kF3), d0 * splat<V>(kF1));
  v[3] = vfma(d1, splat<V>(-kF1), d0 * splat<V>(kF3));
}

// 8x8 transpose across the 8 lanes of a group (lane r: row r -> column r)
// by three XOR butterflies; pure data movement.  The lane-dependent choice is
// made with bit masks: a select between two array elements would be folded
// into a dynamically indexed (scratch) array access.
template <int D>
__device__ __forceinline__ void transpose_stage(float* v, int r) {
  const uint32_t m = (r & D) ? 0xFFFFFFFFu : 0u;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (i & D) continue;
    const int j = i | D;
    const uint32_t a = __float_as_uint(v[i]), b = __float_as_uint(v[j]);
    const uint32_t send = (a & m) | (b & ~m);
    const uint32_t recv = xor_lane_u<D>(send);
    v[i] = __uint_as_float((recv & m) | (a & ~m));
    v[j] = __uint_as_float((b & m) | (recv & ~m));
  }
}
__device__ __forceinline__ void transpose8(float* v, int r) {
  transpose_stage<4>(v, r);
  transpose_stage<2>(v, r);
  transpose_stage<1>(v, r);
}
__device__ __forceinline__ void transpose8(f2* v, int r) {  // each channel on its own
  float a[8], b[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a[i] = v[i].x;
    b[i] = v[i].y;
  }
  transpose8(a, r);
  transpose8(b, r);
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = f2{a[i], b[i]};
}
template <int D>
__device__ __forceinline__ f2 xor_lane(f2 v) {
  return f2{xor_lane<D>(v.x), xor_lane<D>(v.y)};
}
template <int K>
__device__ __forceinline__ f2 group_lane(f2 v) {
  return f2{group_lane<K>(v.x), group_lane<K>(v.y)};
}

template <int T>
constexpr int tindex() {
  return T == kDCT8 ? 0
                    : (T == kDCT4X4 ? 1
                                    : (T == kDCT4X8 ? 2 : (T == kDCT8X4 ? 3 : (T == kDCT2X2 ? 4 : 5))));
}
__device__ __forceinline__ int tindex_rt(int t) {
  return t == kDCT8 ? 0
                    : (t == kDCT4X4 ? 1
                                    : (t == kDCT4X8 ? 2 : (t == kDCT8X4 ? 3 : (t == kDCT2X2 ? 4 : 5))));
}

__device__ __forceinline__ int bitlen(uint32_t v) { return 32 - __clz(v); }  // __clz(0) = 32

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// tree sum over the 8 lanes of a group by XOR butterflies:
// ((0+1)+(2+3))+((4+5)+(6+7)) in every lane (float + is commutative), the
// order of oracle/front.c tree8
__device__ __forceinline__ float group_tree_sum(float v) {
  v += xor_lane<1>(v);
  v += xor_lane<2>(v);
  v += xor_lane<4>(v);
  return v;
}
__device__ __forceinline__ int group_int_sum(int v) {
  v += (int)xor_lane_u<1>((uint32_t)v);
  v += (int)xor_lane_u<2>((uint32_t)v);
  v += (int)xor_lane_u<4>((uint32_t)v);
  return v;
}

struct GroupCtx {
  const float* pix;    // LDS planes X, Y, B (kPlane apart)
  int ly0;             // tile-local row of the block's pixel row 0 (= lby*8 + 1)
  int lx0;             // tile-local column of pixel column 0 (= lbx*8 + 1)
  int r;
  const float* wperm;  // LDS [kNT T][3 c][8 r][8 k] weights per lane
  const float* iwperm; // LDS [kNT T][8 r][8 k] Y inverse weights per lane
  const float* btab;   // LDS [256] AdjustQuantBias of a magnitude q < 256 (c_btab)
  const float* sdperm; // LDS [kNT T][3 c][8 r][8 k] distortion weights per lane
  float kx, kb;        // chroma from luma of the tile: X - kx Yd, B - kb Yd
};

// Quantized values of one candidate: [channel X, Y, B][4 words of 2 x int16]
// (lane r: working-array column r, rows k = 0..7).
struct QVals {
  uint32_t w[12];  // [channel X, Y, B][4]
  uint32_t nz;  // non-zero AC counts of the block: X | Y << 8 | B << 16
};

// Row pass of one channel (lane r = pixel row r of the block): 8-point or
// two 4-point DCTs, then the 8x8 transpose, so lane r holds working-array
// column r.  Shared by the two candidates with the same row transform
// (DCT8 / DCT8X4: 8-point rows; DCT4X4 / DCT4X8: 4-point rows).
// C = kXB: X and B together (f2)
constexpr int kXB = 3;
template <int C, class V>
__device__ __forceinline__ void load_row8(const GroupCtx& G, V* v) {
  const int base = lds_at(G.lx0, G.ly0 + G.r);  // 8 contiguous dwords (same skew)
  if constexpr (C == kXB) {
    const float* px = G.pix + base;
    const float* pb = G.pix + 2 * kPlane + base;
#pragma unroll
    for (int x = 0; x < 8; x++) v[x] = f2{px[x], pb[x]};
  } else {
    const float* plane = G.pix + C * kPlane + base;
#pragma unroll
    for (int x = 0; x < 8; x++) v[x] = plane[x];
  }
}
template <bool ROW8, int C, class V>
__device__ __forceinline__ void row_pass_t(const GroupCtx& G, V* v) {
  load_row8<C>(G, v);
  if (ROW8) {
    dct8_1d(v);
  } else {
    dct4_1d(v);
    dct4_1d(v + 4);
  }
  transpose8(v, G.r);
}

// Candidate state accumulated over the channels Y, X, B (lane r = working
// column r): Y dequantized values for the B residual, rate bits, e*e
// partial, packed quantized values.
struct CandAcc {
  float yd[8];
  int bits;
  float part;
  QVals q;
};

// Column transform of strategy T (lane r: working-array column r) from the
// row-transformed, transposed values, with the lowest-frequency combine
// (enc_transforms [ext]; slots per oracle)
template <int T, class V>
__device__ __forceinline__ void col_transform(const GroupCtx& G, V* v) {
  if (T == kDCT8 || T == kDCT4X8) {
    dct8_1d(v);
  } else {
    dct4_1d(v);
    dct4_1d(v + 4);
  }
  const V q = splat<V>(0.25f), h = splat<V>(0.5f);
  if (T == kDCT4X4) {
    const V A0 = group_lane<0>(v[0]), Cc = group_lane<0>(v[4]);
    const V B0 = group_lane<4>(v[0]), D = group_lane<4>(v[4]);
    if (G.r == 0) {
      v[0] = (((A0 + B0) + Cc) + D) * q;
      v[4] = (((A0 - B0) + Cc) - D) * q;
    } else if (G.r == 4) {
      v[0] = (((A0 + B0) - Cc) - D) * q;
      v[4] = (((A0 - B0) - Cc) + D) * q;
    }
  } else if (T == kDCT8X4) {
    if (G.r == 0) {
      const V A0 = v[0], B0 = v[4];
      v[0] = (A0 + B0) * h;
      v[4] = (A0 - B0) * h;
    }
  } else if (T == kDCT4X8) {
    const V A0 = group_lane<0>(v[0]), B0 = group_lane<4>(v[0]);
    if (G.r == 0) v[0] = (A0 + B0) * h;
    if (G.r == 4) v[0] = (A0 - B0) * h;
  }
}

// The Haar-type candidates of channel C straight from the pixels (lane r =
// pixel row r), leaving lane r's 8 values in the slot order of co_index_rt
// (oracle jxo_transform, same float ops):
//   DCT2X2    three levels of 2x2 Haar steps; a level's cells pair lanes
//             r ^ 1 (level 1: all rows), r ^ 2 (level 2: the even lanes'
//             first four values), r ^ 4 (level 3: lanes 0 and 4, first two);
//             the top lane of a pair keeps (a_top +- a_bottom) / 4, the bottom
//             lane (b_top +- b_bottom) / 4;
//   IDENTITY  lane r = row iy = r & 3 of sub-block row r >> 2: residuals
//             against the sub-block's pixel (1, 1) (from lane 4y + 1), the
//             (0, 0) residual moved into the (1, 1) slot (from lane 4y), the
//             sub-block means (row sums, quad tree) in the (0, 0) slots and
//             combined over lanes 0 / 4 like DCT4X4's.
template <int T, int C, class V>
__device__ __forceinline__ void haar_lane(const GroupCtx& G, V* v) {
  V p[8];
  load_row8<C>(G, p);
  if constexpr (T == kDCT2X2) {
    const bool top1 = (G.r & 1) == 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const V a = p[2 * j] + p[2 * j + 1], b = p[2 * j] - p[2 * j + 1];
      const V ap = xor_lane<1>(a), bp = xor_lane<1>(b);
      v[j] = top1 ? (a + ap) * 0.25f : (bp + b) * 0.25f;
      v[4 + j] = top1 ? (a - ap) * 0.25f : (bp - b) * 0.25f;
    }
    const bool top2 = (G.r & 2) == 0, even = (G.r & 1) == 0;
    V n2[4];
#pragma unroll
    for (int x = 0; x < 2; x++) {
      const V a = v[2 * x] + v[2 * x + 1], b = v[2 * x] - v[2 * x + 1];
      const V ap = xor_lane<2>(a), bp = xor_lane<2>(b);
      n2[x] = top2 ? (a + ap) * 0.25f : (bp + b) * 0.25f;
      n2[2 + x] = top2 ? (a - ap) * 0.25f : (bp - b) * 0.25f;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = even ? n2[k] : v[k];
    const bool top3 = (G.r & 4) == 0, l3 = (G.r & 3) == 0;
    const V a = v[0] + v[1], b = v[0] - v[1];
    const V ap = xor_lane<4>(a), bp = xor_lane<4>(b);
    const V n30 = top3 ? (a + ap) * 0.25f : (bp + b) * 0.25f;
    const V n31 = top3 ? (a - ap) * 0.25f : (bp - b) * 0.25f;
    v[0] = l3 ? n30 : v[0];
    v[1] = l3 ? n31 : v[1];
  } else {  // kIDENTITY
    const V rs0 = ((p[0] + p[1]) + p[2]) + p[3], rs1 = ((p[4] + p[5]) + p[6]) + p[7];
    V s0 = rs0 + xor_lane<1>(rs0), s1 = rs1 + xor_lane<1>(rs1);
    s0 = s0 + xor_lane<2>(s0);
    s1 = s1 + xor_lane<2>(s1);
    const V dc0 = s0 * (1.0f / 16.0f), dc1 = s1 * (1.0f / 16.0f);
    const bool hi = (G.r & 4) != 0;
    const V p11a = group_lane<1>(p[1]), p11b = group_lane<5>(p[1]);
    const V p15a = group_lane<1>(p[5]), p15b = group_lane<5>(p[5]);
    const V q0 = hi ? p11b : p11a, q1 = hi ? p15b : p15a;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      v[k] = p[k] - q0;
      v[4 + k] = p[4 + k] - q1;
    }
    const V t0 = xor_lane<1>(v[0]), t1 = xor_lane<1>(v[4]);
    const int iy = G.r & 3;
    if (iy == 1) {
      v[1] = t0;
      v[5] = t1;
    }
    const V o0 = xor_lane<4>(dc0), o1 = xor_lane<4>(dc1);
    const V A = hi ? o0 : dc0, B = hi ? o1 : dc1, Cc = hi ? dc0 : o0, D = hi ? dc1 : o1;
    if (iy == 0) {
      v[0] = dc0;
      v[4] = dc1;
    }
    if (G.r == 0) {
      v[0] = (((A + B) + Cc) + D) * 0.25f;
      v[4] = (((A + B) - Cc) - D) * 0.25f;
    } else if (G.r == 4) {
      v[0] = (((A - B) + Cc) - D) * 0.25f;
      v[4] = (((A - B) - Cc) + D) * 0.25f;
    }
  }
}

// The signed quantized value of a coefficient: qf is the integer-valued
// magnitude (0 .. 32767), vq the scaled coefficient; (vq < 0 ? -(int)qf :
// (int)qf) is (int)sq, sq = copysign(qf, vq): one sign insert and one
// conversion (vq = -0 has qf = 0 and converts to 0 either way).  Two of them go into one word as int16 lo / hi
// (v_cvt_pk_i16_i32; its saturation never applies at |q| <= 32767).
// signed_err: the quantization error is taken on the signed values, (vq -
// sq) with sq = copysign(qf, vq): for vq < 0 that is (-|vq|) - (-qf) = -(|vq| -
// qf) exactly (round to nearest is symmetric in sign), for vq = +-0 it is +0,
// so e * e -- the only use of e -- is the oracle's (|vq| - qf)^2 bit for bit,
// with no |vq| pair to build for the packed subtraction.
// Non-zero count of eight quantized magnitudes from the sum of their biased
// exponents: a zero has E = 0, a non-zero qf in [1, 32767] has E = 127 + d
// with d = floor(log2 qf) in [0, 14], so the sum is 127 nz + (sum of d) with
// the second term at most 8 x 14 = 112 < 127: nz = sum / 127 exactly.
__device__ __forceinline__ int nz_of_esum(uint32_t esum) { return (int)(esum / 127u); }
__device__ __forceinline__ uint32_t pack_q(int lo, int hi) {
  const auto p = __builtin_amdgcn_cvt_pk_i16(lo, hi);
  return __builtin_bit_cast(uint32_t, p);
}

// Quantization of lane r's 8 values of channel C (0 X, 1 Y, 2 B) under
// strategy T: accumulate e*e (fmaf), rate bits and the non-zero count; Y
// records its dequantized values for the X / B residuals.  Float op order ==
// oracle jxo_quantize_block.  Coefficients go in pairs (k, k + 1): every
// float multiply / add / subtract of the pair is one packed op (f2: each half
// is exactly the scalar op, no contraction); the e*e chain stays in k order.
// qa is kept as an integer-valued float qf (the truncation of a positive value
// is its floor): the error needs no conversion, and the rate 2 + 2 bitlen(qa)
// of a non-zero is 2 E - 250, E = the biased exponent of qf.
template <int C>
__device__ __forceinline__ void quant_lane(const GroupCtx& G, int ti, float* v, float scale,
                                           float inv_scale, CandAcc& A) {
  if (G.r == 0) v[0] = 0.0f;  // DC slot: quantizes to 0, contributes nothing
  const float4* wp = reinterpret_cast<const float4*>(G.wperm + ((ti * 3 + C) * 8 + G.r) * 8);
  const float4 w0 = wp[0], w1 = wp[1];
  const f2 wk2[4] = {f2{w0.x, w0.y}, f2{w0.z, w0.w}, f2{w1.x, w1.y}, f2{w1.z, w1.w}};
  const float2* sdp = reinterpret_cast<const float2*>(G.sdperm + ((ti * 3 + C) * 8 + G.r) * 8);
  f2 iwk2[4];
  if (C == 1) {
    const float4* ip = reinterpret_cast<const float4*>(G.iwperm + (ti * 8 + G.r) * 8);
    const float4 i0 = ip[0], i1 = ip[1];
    iwk2[0] = f2{i0.x, i0.y};
    iwk2[1] = f2{i0.z, i0.w};
    iwk2[2] = f2{i1.x, i1.y};
    iwk2[3] = f2{i1.z, i1.w};
  }
  const f2 sc2 = f2{scale, scale}, isc2 = f2{inv_scale, inv_scale};
  uint32_t ebits = 0;
  int qs[8];
  int qmax = 0;  // (Y) magnitudes >= 256 take the division after the loop
#pragma unroll
  for (int kp = 0; kp < 4; kp++) {
    const int k = 2 * kp;
    const f2 ws = wk2[kp] * sc2;
    f2 rv = f2{v[k], v[k + 1]};
    if (C == 0) rv = rv - f2{G.kx, G.kx} * f2{A.yd[k], A.yd[k + 1]};
    if (C == 2) rv = rv - f2{G.kb, G.kb} * f2{A.yd[k], A.yd[k + 1]};
    const f2 vq = rv * ws;
    f2 qf;
    qf.x = fabsf(vq.x) < 0.58f ? 0.0f : floorf(fminf(fabsf(vq.x), 32767.0f) + 0.5f);
    qf.y = fabsf(vq.y) < 0.58f ? 0.0f : floorf(fminf(fabsf(vq.y), 32767.0f) + 0.5f);
    const f2 sq = f2{__builtin_copysignf(qf.x, vq.x), __builtin_copysignf(qf.y, vq.y)};
    if (C == 1) {
      f2 adj;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const float q = h ? qf.y : qf.x;
        const int qa = (int)q;
        float ad = G.btab[qa < 255 ? qa : 255];  // the tabulated bias below 256
        qmax = max(qmax, qa);
        // vq < 0 ? -ad : ad as one sign insert; at vq = -0 (ad = 0) it gives
        // -0, a dequantized Y of -0 whose only uses (the X / B residuals, every
        // quantity derived from them) see the same values for +-0
        ad = __builtin_copysignf(ad, h ? vq.y : vq.x);
        if (h) adj.y = ad;
        else adj.x = ad;
      }
      const f2 yd = adj * (iwk2[kp] * isc2);
      A.yd[k] = yd.x;
      A.yd[k + 1] = yd.y;
    }
    // quantization error in steps, times the distortion weight: the
    // coefficient's pixel-domain error (oracle jxo_dist_weight)
    // (signed_err: (vq - sq) sd = +-(|vq| - qf) sd exactly, same square)
    const float2 sd = sdp[kp];
    const f2 e = (vq - sq) * f2{sd.x, sd.y};
    A.part = fmaf(e.x, e.x, A.part);
    A.part = fmaf(e.y, e.y, A.part);
    ebits += (__float_as_uint(qf.x) >> 23) + (__float_as_uint(qf.y) >> 23);
    qs[k] = (int)sq.x;
    qs[k + 1] = (int)sq.y;
  }
  if (C == 1 && __any(qmax >= 256)) {
    // the bias of a magnitude >= 256, q - 0.145 / q (the table stops at 255),
    // and its dequantized value: the same float ops as below 256
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int qa = qs[k] < 0 ? -qs[k] : qs[k];
      if (qa >= 256) {
        const float q = (float)qa;
        float ad = q - 0.145f / q;
        if (qs[k] < 0) ad = -ad;
        A.yd[k] = ad * (((k & 1) ? iwk2[k >> 1].y : iwk2[k >> 1].x) * inv_scale);
      }
    }
  }
  // sum over k of [qa != 0] (2 + 2 bitlen) = 2 E-sum - 250 nz
  const int nz = nz_of_esum(ebits);
  A.bits += 2 * (int)ebits - 250 * nz;
  uint32_t pk[4];
#pragma unroll
  for (int i = 0; i < 4; i++) pk[i] = pack_q(qs[2 * i], qs[2 * i + 1]);
  const int nzc = group_int_sum(nz);
  A.bits += G.r == 0 ? bitlen((uint32_t)nzc) : 0;
  constexpr int slot = C == 1 ? 4 : (C == 0 ? 0 : 8);
#pragma unroll
  for (int i = 0; i < 4; i++) A.q.w[slot + i] = pk[i];
  const uint32_t sh = C == 1 ? 8 : (C == 0 ? 0 : 16);
  A.q.nz = (C == 1 ? 0u : A.q.nz) | ((uint32_t)nzc << sh);
}

// Quantization of lane r's 8 values of X and B together (f2 = (X, B) per
// coefficient k), each channel with its own weights, chroma-from-luma factor
// and distortion weights: every float op of the pair is one packed op.  The
// e*e chain keeps the scalar order (X's k = 0..7, then B's).
__device__ __forceinline__ void quant_xb(const GroupCtx& G, int ti, f2* v, float scale, CandAcc& A) {
  if (G.r == 0) v[0] = f2{0.0f, 0.0f};  // DC slots quantize to 0
  const float* wxp = G.wperm + ((ti * 3 + 0) * 8 + G.r) * 8;
  const float* wbp = G.wperm + ((ti * 3 + 2) * 8 + G.r) * 8;
  const float* sxp = G.sdperm + ((ti * 3 + 0) * 8 + G.r) * 8;
  const float* sbp = G.sdperm + ((ti * 3 + 2) * 8 + G.r) * 8;
  const float4 wx0 = reinterpret_cast<const float4*>(wxp)[0], wx1 = reinterpret_cast<const float4*>(wxp)[1];
  const float4 wb0 = reinterpret_cast<const float4*>(wbp)[0], wb1 = reinterpret_cast<const float4*>(wbp)[1];
  const f2 wk[8] = {f2{wx0.x, wb0.x}, f2{wx0.y, wb0.y}, f2{wx0.z, wb0.z}, f2{wx0.w, wb0.w},
                    f2{wx1.x, wb1.x}, f2{wx1.y, wb1.y}, f2{wx1.z, wb1.z}, f2{wx1.w, wb1.w}};
  const f2 sc2 = f2{scale, scale}, kxb = f2{G.kx, G.kb};
  uint32_t ebx = 0, ebb = 0;  // exponent sums of X's and of B's eight values
  float eb[8];
  int sx[8], sb[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const f2 ws = wk[k] * sc2;
    const f2 rv = v[k] - kxb * f2{A.yd[k], A.yd[k]};
    const f2 vq = rv * ws;
    f2 qf;
    qf.x = fabsf(vq.x) < 0.58f ? 0.0f : floorf(fminf(fabsf(vq.x), 32767.0f) + 0.5f);
    qf.y = fabsf(vq.y) < 0.58f ? 0.0f : floorf(fminf(fabsf(vq.y), 32767.0f) + 0.5f);
    const f2 sq = f2{__builtin_copysignf(qf.x, vq.x), __builtin_copysignf(qf.y, vq.y)};
    const f2 e = (vq - sq) * f2{sxp[k], sbp[k]};  // (signed_err)
    A.part = fmaf(e.x, e.x, A.part);  // X's chain
    eb[k] = e.y;
    ebx += __float_as_uint(qf.x) >> 23;
    ebb += __float_as_uint(qf.y) >> 23;
    sx[k] = (int)sq.x;
    sb[k] = (int)sq.y;
  }
#pragma unroll
  for (int k = 0; k < 8; k++) A.part = fmaf(eb[k], eb[k], A.part);  // then B's
  const int nzx = nz_of_esum(ebx), nzb = nz_of_esum(ebb);
  A.bits += 2 * (int)(ebx + ebb) - 250 * (nzx + nzb);
  const int nzcx = group_int_sum(nzx), nzcb = group_int_sum(nzb);
  A.bits += G.r == 0 ? bitlen((uint32_t)nzcx) + bitlen((uint32_t)nzcb) : 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    A.q.w[i] = pack_q(sx[2 * i], sx[2 * i + 1]);
    A.q.w[8 + i] = pack_q(sb[2 * i], sb[2 * i + 1]);
  }
  A.q.nz |= (uint32_t)nzcx | ((uint32_t)nzcb << 16);
}

// One candidate T (run-time, wave-uniform): Y, then X and B together (f2);
// only one candidate's state is live at a time, which keeps the kernel inside
// 128 VGPRs.  Round 6: the candidates share one transform dispatch and one
// quantization body per channel (the kernel evaluates them in two rolled
// loops, phase C) instead of six fully inlined instantiations -- 130 KB of
// machine code, twice the instruction cache a CU pair shares, and 31 % of the
// waves' cycles waiting on instruction fetch (profiles/r05zr/attr_front.json).
// The float ops of every candidate are unchanged.
// PRE (DCT8, DCT8X4): the fit's transposed 8-point row passes, y[k] and
// xb[k] = (X, B), are given; only the column transform is left.  Without PRE
// (DCT4X4, DCT4X8: 4-point rows; DCT2X2 / IDENTITY: Haar steps; hook P's
// re-evaluation of DCT8X4: 8-point rows) the transform starts from the pixels.
// Scan pruning (no effect on any result): the estimate's bits and e*e sum
// only grow from channel to channel (every non-zero adds 2 + 2 bitlen > 0,
// bitlen(nz) >= 0; fmaf(e, e, acc) >= acc and the tree sum of non-negative
// lane sums is monotone in each of them), so the estimate after Y alone is a
// lower bound of the final one, and so is hook F of it while hook F's factor
// 0.8 avg_r is not negative (a NaN factor makes both NaN: no pruning).  When
// that bound exceeds the best estimate so far for every block of the wave,
// the candidate cannot win the scan (`beats` needs e < best, or e == best with
// a lower index) and its X / B half is skipped: NaN is returned, which never
// wins.  The hook-P override re-evaluates its candidate in full.
struct Prune {
  bool on;          // a best estimate exists (not for the scan's first candidate)
  float best;       // the scan's best (after hook F)
  bool hookF;
  float rh, rv, rd;
};
template <bool PRE, int C, class V>
__device__ __forceinline__ void cand_transform(const GroupCtx& G, int T, V* v, const V* pre) {
  if constexpr (PRE) {
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = pre[k];
    if (T == kDCT8) col_transform<kDCT8>(G, v);
    else col_transform<kDCT8X4>(G, v);
  } else {
    if (T == kDCT4X4 || T == kDCT4X8) {
      row_pass_t<false, C>(G, v);
      if (T == kDCT4X4) col_transform<kDCT4X4>(G, v);
      else col_transform<kDCT4X8>(G, v);
    } else if (T == kDCT2X2) {
      haar_lane<kDCT2X2, C>(G, v);
    } else if (T == kIDENTITY) {
      haar_lane<kIDENTITY, C>(G, v);
    } else {  // kDCT8X4 without the fit's rows (hook P's re-evaluation)
      row_pass_t<true, C>(G, v);
      col_transform<kDCT8X4>(G, v);
    }
  }
}
template <bool PRE>
__device__ __forceinline__ float eval_cand(const GroupCtx& G, int T, float scale, float inv_scale,
                                           CandAcc& A, const float* pre_y, const f2* pre_xb,
                                           const Prune& pr) {
  // estimate multipliers (== oracle jxo_quantize_block tmul, JXO_TMUL_*)
  const float tm = T == kDCT8 ? 1.0f
                              : (T == kDCT4X4 ? 1.05f
                                              : (T == kDCT2X2 ? 1.05f
                                                              : (T == kIDENTITY ? 1.08f : 1.02f)));
  const int ti = tindex_rt(T);
  A.bits = 0;
  A.part = 0.0f;
  A.q.nz = 0;
  {
    float v[8];
    cand_transform<PRE, 1>(G, T, v, pre_y);
    quant_lane<1>(G, ti, v, scale, inv_scale, A);
  }
  if (pr.on) {
    float lb = ((float)group_int_sum(A.bits) + 8.0f * group_tree_sum(A.part)) * tm;
    bool out;
    if (pr.hookF) {
      const float avg_r = (pr.rh + pr.rv + pr.rd) / 3.0f;
      out = avg_r >= 0.0f && hook_f(lb, pr.rh, pr.rv, pr.rd) > pr.best;
    } else {
      out = lb > pr.best;
    }
    if (__all(out)) return __builtin_nanf("");
  }
  {
    f2 v[8];
    cand_transform<PRE, kXB>(G, T, v, pre_xb);
    quant_xb(G, ti, v, scale, A);
  }
  return ((float)group_int_sum(A.bits) + 8.0f * group_tree_sum(A.part)) * tm;
}

__device__ __forceinline__ void copy_q(QVals& d, const QVals& s, bool take) {
#pragma unroll
  for (int i = 0; i < 12; i++) d.w[i] = take ? s.w[i] : d.w[i];
  d.nz = take ? s.nz : d.nz;
}

// FindBest8x8Transform's scan (`e < best`, candidates in the order DCT8,
// DCT4X4, DCT2X2, DCT4X8, DCT8X4, IDENTITY, best starting at FLT_MAX) as a
// tournament: a
// candidate beats another when its estimate is below FLT_MAX and smaller, or
// equal with a lower scan index; NaN never wins.
__device__ __forceinline__ bool beats(float ea, int ia, float eb, int ib) {
  const bool va = ea < FLT_MAX, vb = eb < FLT_MAX;
  if (va && vb) return ea < eb || (ea == eb && ia < ib);
  if (va != vb) return va;
  return ia < ib;
}

// RGB8 -> XYB for the 66 x 66 tile (+1 px halo).  The tile's rows are read
// as 4-pixel chunks (12 bytes = 3 aligned dwords; the chunk grid is aligned
// to the frame's 4-pixel columns, 18 chunks per tile row); chunks that cross
// the frame's left/right edge (or an unaligned buffer) fall back to clamped
// byte loads.  All loads of a thread are issued before any conversion.
// Samples outside the block-padded frame read 0 (H2); padding inside it
// replicates the last column / row.
constexpr int kChunksX = 18;
constexpr int kChunks = kRows * kChunksX;
constexpr int kChunkIters = (kChunks + kThreads - 1) / kThreads;
constexpr int kRing = 2 * 68 + 2 * 66;  // Gaborish ring: tile-local rows / columns -1 and 66
// chunk i's 12 bytes (4 pixels), clamped to the image
__device__ __forceinline__ void load_chunk(const FrontArgs& a, bool al, int i, int ox, int oy,
                                           uint32_t d[3]) {
  const int ly = i / kChunksX, cx = i - ly * kChunksX;
  const int gy = oy + ly, gx0 = ox - 3 + 4 * cx;
  const int sy = min(max(gy, 0), (int)a.h - 1);
  const uint8_t* row = a.rgb + (size_t)sy * a.stride;
  if (al && gx0 >= 0 && gx0 + 4 <= (int)a.w) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(row + 3 * (size_t)gx0);
    d[0] = p[0];
    d[1] = p[1];
    d[2] = p[2];
  } else {
    uint32_t by[12];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int sx = min(max(gx0 + j, 0), (int)a.w - 1);
      const uint8_t* q = row + 3 * (size_t)sx;
      by[3 * j] = q[0];
      by[3 * j + 1] = q[1];
      by[3 * j + 2] = q[2];
    }
#pragma unroll
    for (int w = 0; w < 3; w++)
      d[w] = by[4 * w] | by[4 * w + 1] << 8 | by[4 * w + 2] << 16 | by[4 * w + 3] << 24;
  }
}
// The tile's global loads, issued all at once at the workgroup's start (before
// the table copies and their barrier): a thread's three chunks (12 bytes each)
// and, with Gaborish, its ring pixel.  Round 6: the per-phase clock profile
// (JXG_FRONT_PROFILE, profiles/r06p) put 29 % of an e7 workgroup's time (42 %
// at e4) in the tile load, which waited for one chunk's loads per iteration
// and then for the ring's: every wait a full memory latency.
struct TileLoads {
  uint32_t d[kChunkIters][3];  // chunks threadIdx.x + k * kThreads
  uint32_t ring;               // ring pixel threadIdx.x - kRingT0: r | g << 8 | b << 16
};
// the ring's pixels go to the threads the last chunk round leaves idle
// (threads kRingT0 .. kRingT0 + 267), so the ring costs no pass of its own
constexpr int kRingT0 = kChunks - (kChunkIters - 1) * kThreads;
static_assert(kRingT0 + kRing <= kThreads, "the ring fits the last round's idle threads");
__device__ __forceinline__ int ring_x(int i) { return i < 68 ? i - 1 : (i < 136 ? i - 69 : (i < 202 ? -1 : 66)); }
__device__ __forceinline__ int ring_y(int i) { return i < 68 ? -1 : (i < 136 ? 66 : (i < 202 ? i - 136 : i - 202)); }
__device__ __forceinline__ void issue_tile_loads(const FrontArgs& a, int ox, int oy, bool gab,
                                                 TileLoads& L) {
#ifdef JXG_EXP_NOLOAD  // (timing experiment only: no tile loads, hashed bytes)
#pragma unroll
  for (int k = 0; k < kChunkIters; k++)
#pragma unroll
    for (int w = 0; w < 3; w++)
      L.d[k][w] = ((uint32_t)threadIdx.x * 2654435761u + (uint32_t)(ox * 7919 + oy * 104729) + k * 31 + w) * 2246822519u;
  L.ring = ((uint32_t)threadIdx.x * 2246822519u + (uint32_t)(ox + oy)) & 0xFFFFFF;
  return;
#endif
  const bool al = ((a.stride | (size_t)a.rgb) & 3) == 0;
#pragma unroll
  for (int k = 0; k < kChunkIters; k++)
    load_chunk(a, al, min((int)threadIdx.x + k * kThreads, kChunks - 1), ox, oy, L.d[k]);
  L.ring = 0;
  const int ri = (int)threadIdx.x - kRingT0;
  if (gab && ri >= 0 && ri < kRing) {  // (the ring's pixels, clamped to the image)
    const int i = ri, lx = ring_x(i), ly = ring_y(i);
    const int sx = min(max(ox + lx, 0), (int)a.w - 1), sy = min(max(oy + ly, 0), (int)a.h - 1);
    const uint8_t* q = a.rgb + (size_t)sy * a.stride + 3 * (size_t)sx;
    L.ring = (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16;
  }
}
// rep (Gaborish): samples outside the block-padded frame hold the clamped
// image sample too (the inverse Gaborish reads every source at coordinates
// clamped to the padded frame, i.e. the image sample at coordinates clamped to
// the image); they are zeroed again after the sweep (zero_outside).
// The chunks are converted in a rolled loop (four inlined conversions; the
// chunk registers rotate, so every index stays static).
__device__ __forceinline__ void load_xyb_tile(const FrontArgs& a, const float* lut, float* sPix,
                                              int ox, int oy, bool rep, TileLoads& L,
                                              float* ring) {
  const float cb = cbrt_det(kOpsinBias);
#pragma unroll 1
  for (int k = 0; k < kChunkIters; k++) {
    const int i = threadIdx.x + k * kThreads;
    if (i >= kChunks) {  // (last round) the Gaborish ring's pixel instead
      const int ri = (int)threadIdx.x - kRingT0;
      if (ring && ri >= 0 && ri < kRing) {
        float X, Y, B;
        pixel_xyb(lut, cb, L.ring & 0xFF, (L.ring >> 8) & 0xFF, (L.ring >> 16) & 0xFF, X, Y, B);
        ring[ri] = X;
        ring[kRing + ri] = Y;
        ring[2 * kRing + ri] = B;
      }
    } else {
      const int ly = i / kChunksX, cx = i - ly * kChunksX;
      const int gy = oy + ly, gx0 = ox - 3 + 4 * cx;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int lx = 4 * cx - 3 + j;
        if (lx < 0 || lx >= 66) continue;
        const int gx = gx0 + j;
        const bool inside = rep || (gx >= 0 && gy >= 0 && gx < (int)a.xp && gy < (int)a.yp);
        float X = 0.0f, Y = 0.0f, B = 0.0f;
        if (inside) {
          const int b0 = 3 * j;
          const uint32_t r8 = (L.d[0][b0 >> 2] >> ((b0 & 3) * 8)) & 0xFF;
          const uint32_t g8 = (L.d[0][(b0 + 1) >> 2] >> (((b0 + 1) & 3) * 8)) & 0xFF;
          const uint32_t b8 = (L.d[0][(b0 + 2) >> 2] >> (((b0 + 2) & 3) * 8)) & 0xFF;
          pixel_xyb(lut, cb, r8, g8, b8, X, Y, B);
        }
        const int o = lds_at(lx, ly);
        sPix[o] = X;
        sPix[kPlane + o] = Y;
        sPix[2 * kPlane + o] = B;
      }
    }
#pragma unroll
    for (int q = 0; q + 1 < kChunkIters; q++)
#pragma unroll
      for (int w = 0; w < 3; w++) L.d[q][w] = L.d[q + 1][w];
  }
}
// samples outside the block-padded frame back to 0 (H2) after the sweep
__device__ __forceinline__ void zero_outside(const FrontArgs& a, float* sPix, int ox, int oy) {
  for (int i = threadIdx.x; i < 66 * 66; i += kThreads) {
    const int ly = i / 66, lx = i - ly * 66;
    const int gx = ox + lx, gy = oy + ly;
    if (gx >= 0 && gy >= 0 && gx < (int)a.xp && gy < (int)a.yp) continue;
    const int o = lds_at(lx, ly);
    sPix[o] = 0.0f;
    sPix[kPlane + o] = 0.0f;
    sPix[2 * kPlane + o] = 0.0f;
  }
}

// ---------------------------------------------------------------------------
// inverse Gaborish (JXG_FLAG_GABORISH; oracle/xyb.c jxo_gab_inverse): the
// 3x3 symmetric least-squares inverse of the decoder's Gaborish kernel, on
// the padded frame with edge replication, before every other stage.  The
// 66 x 66 LDS tile (1 px halo) is filtered in place; its outer ring (tile-local
// rows / columns -1 and 66: 268 pixels) is converted into a small LDS ring
// first.  Samples are read at coordinates clamped to the padded frame; pixels
// outside it stay 0 (H2).
// ---------------------------------------------------------------------------
constexpr float kGabK0 = 1.8012209f;
constexpr float kGabK1 = -0.15485205f;
constexpr float kGabK2 = -0.04545318f;
__device__ __forceinline__ int ring_index(int lx, int ly) {  // (lx, ly) on the ring
  if (ly == -1) return lx + 1;
  if (ly == 66) return 69 + lx;
  if (lx == -1) return 136 + ly;
  return 202 + ly;
}
// Sweep: thread = (row half, channel, column), 396 threads; a 3 x 3 window in
// registers, one new row per step, the 33 outputs of its column half kept in
// registers until every thread has read its inputs (one barrier), then
// stored in place.  (Round 4 stored each row after a barrier of its own: 33
// barriers per tile.)  Each source column is one LDS column at a per-thread
// base (row offsets become immediates), the two ring columns are read beside
// it and selected, and only the first row (half 0) and the last row (half 1)
// come from the ring rows.
//
// Round 6: every tile takes this form.  The edge tiles' clamped sweep (a
// second 33-step body with a clamp per sample: 28 KB of the kernel's code)
// is gone: an edge tile's LDS tile and ring hold the clamped image sample at
// every position (load_xyb_tile rep; the ring pixels are clamped to the image), which is
// what the clamped sweep read, so every in-frame output is the same float
// expression of the same values; the positions outside the padded frame are
// zeroed after it (zero_outside).
__device__ __forceinline__ void gab_sweep(float* sPix, const float* ring) {
  const int t = threadIdx.x;
  const bool act = t < 396;
  const int half = t >= 198 ? 1 : 0, c = (t - 198 * half) / 66, lx = t % 66;
  const int y0 = 33 * half;
  float* P = sPix + c * kPlane;
  const float* R = ring + c * kRing;
  float out[33];
  if (act) {
    const bool ringL = lx == 0, ringR = lx == 65;
    // column bases at row y0 (LDS) and the ring columns' bases at row y0
    const int bL = (ringL ? 0 : lds_at(lx - 1, 0)) + y0 * kS, bM = lds_at(lx, 0) + y0 * kS;
    const int bR = (ringR ? 0 : lds_at(lx + 1, 0)) + y0 * kS;
    const int cL = 136 + y0, cR = 202 + y0;
    // sample of column k at row y0 + d (d in [0, 33] for half 0, [-1, 32] for half 1)
#define GAB_L(d) (ringL ? R[cL + (d)] : P[bL + (d) * kS])
#define GAB_M(d) (P[bM + (d) * kS])
#define GAB_R(d) (ringR ? R[cR + (d)] : P[bR + (d) * kS])
    float n[3], m[3], sn[3];
    if (half == 0) {  // row -1: the ring's top row
      n[0] = R[lx];
      n[1] = R[lx + 1];
      n[2] = R[lx + 2];
    } else {
      n[0] = GAB_L(-1);
      n[1] = GAB_M(-1);
      n[2] = GAB_R(-1);
    }
    m[0] = GAB_L(0);
    m[1] = GAB_M(0);
    m[2] = GAB_R(0);
#pragma unroll
    for (int st = 0; st < 33; st++) {
      if (st == 32 && half == 1) {  // row 66: the ring's bottom row
        sn[0] = R[68 + lx];
        sn[1] = R[69 + lx];
        sn[2] = R[70 + lx];
      } else {
        sn[0] = GAB_L(st + 1);
        sn[1] = GAB_M(st + 1);
        sn[2] = GAB_R(st + 1);
      }
      const float s1 = (n[1] + sn[1]) + (m[0] + m[2]);
      const float s2 = (n[0] + n[2]) + (sn[0] + sn[2]);
      out[st] = (m[1] * kGabK0 + s1 * kGabK1) + s2 * kGabK2;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        n[k] = m[k];
        m[k] = sn[k];
      }
    }
#undef GAB_L
#undef GAB_M
#undef GAB_R
  }
  __syncthreads();
  if (act) {
#pragma unroll
    for (int st = 0; st < 33; st++) P[lds_at(lx, y0 + st)] = out[st];
  }
}
// chroma-from-luma factor as an int8 multiple of 1/84 (oracle cfl_quant)
__device__ __forceinline__ int cfl_quant(float k) {
  float v = k * 84.0f;
  v = fminf(fmaxf(v, -128.0f), 127.0f);
  const int q = v >= 0.0f ? (int)(v + 0.5f) : -(int)(-v + 0.5f);
  return q > 127 ? 127 : (q < -128 ? -128 : q);
}

// JXG_FRONT_PROFILE (experiment builds only): per-phase shader-clock sums of
// thread 0 of every workgroup (wave 0's view; the phases up to B end at
// workgroup barriers), printed by dump_front_profile() at context destroy
#ifdef JXG_FRONT_PROFILE
__device__ unsigned long long g_fprof[12];
#define FPROF(k)                                                     \
  do {                                                               \
    if (threadIdx.x == 0) {                                          \
      const unsigned long long now_ = __builtin_readcyclecounter();  \
      if ((k) > 0) atomicAdd(&g_fprof[(k)], now_ - fprof_t0);       \
      else atomicAdd(&g_fprof[0], 1ull);                             \
      fprof_t0 = now_;                                               \
    }                                                                \
  } while (0)
#else
#define FPROF(k) \
  do {           \
  } while (0)
#endif

// HOOKP: hook P compiled in (proposals bit 0); without it the kernel keeps
// no hook-P candidate aside (fewer live registers)
#ifndef JXG_FRONT_WPE  // (experiment builds override it: tools/build_variant.sh)
#define JXG_FRONT_WPE 4
#endif
template <bool HOOKP>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(JXG_FRONT_WPE))) void front_kernel(Batch<FrontArgs> bt_) {
  const FrontArgs& a = bt_.a[blockIdx.z];  // the batch's frame
  __shared__ __attribute__((aligned(16))) float sPix[3 * kPlane];
  // phase D's zigzag staging [wave][group][64] reuses the bytes of the sRGB
  // LUT (XYB load only) and of the phase-A / CfL scratch sH (a barrier
  // separates their last reads from the first staging store): 81 KB in all,
  // two workgroups per CU
  __shared__ __attribute__((aligned(16))) float sUnion[2048];
  int16_t(*sStage)[8][64] = reinterpret_cast<int16_t(*)[8][64]>(sUnion);
  float* sLut = sUnion;
  float(*sH)[64] = reinterpret_cast<float(*)[64]>(sUnion + 256);
  __shared__ __attribute__((aligned(16))) float sWperm[kNT * 3 * 64];
  __shared__ __attribute__((aligned(16))) float sIwperm[kNT * 64];
  __shared__ __attribute__((aligned(16))) float sSdperm[kNT * 3 * 64];
  __shared__ __attribute__((aligned(16))) uint8_t sZz[kNT * 64];
  __shared__ float sBtab[256];
  __shared__ float sR[64][3];
  __shared__ uint64_t sLapBits[64];
  const int tid = threadIdx.x;
  // a shard launches its own tiles through a list (1-D grid)
  // A whole frame's tiles go in an XCD-aware order (1-D grid of 8 x chunk
  // workgroups; workgroup w runs on XCD w % 8): XCD x takes the chunk
  // [x chunk, (x + 1) chunk) of the raster tile order, so the 128-byte lines
  // a tile's RGB8 rows share with its left / right / upper neighbours are L2
  // hits on the same XCD instead of fetches by another, and every XCD gets
  // the same number of tiles (a column-strip split left a 1080p frame's 510
  // tiles 68 per XCD on 64 workgroup slots: two rounds instead of one).
  int tx, ty;
  bool idle = false;
  if (a.tile_list) {
    const int tile_id = (int)a.tile_list[blockIdx.x];
    tx = tile_id % (int)a.tiles_x;
    ty = tile_id / (int)a.tiles_x;
  } else {
    const int ntiles = (int)a.ntiles_all, chunk = (ntiles + 7) >> 3;
    const int j = (int)(blockIdx.x >> 3), tile = (int)(blockIdx.x & 7) * chunk + j;
    idle = j >= chunk || tile >= ntiles;  // (the last XCD's chunk past the frame)
    tx = tile % (int)a.tiles_x;
    ty = tile / (int)a.tiles_x;
  }
  const int ox = tx * kTile - 1, oy = ty * kTile - 1;
  if (a.zero) {  // the frame's statistics arena (the statistics kernels add into it)
    const uint32_t nwg = gridDim.x, wg = blockIdx.x;
    const uint32_t per = (a.zero_quads + nwg - 1) / nwg;
    for (uint32_t i = wg * per + tid; i < min(a.zero_quads, (wg + 1) * per); i += kThreads)
      a.zero[i] = make_uint4(0, 0, 0, 0);
  }
  if (idle) return;
#ifdef JXG_FRONT_PROFILE
  unsigned long long fprof_t0 = 0;
#endif
  FPROF(0);
  // the table loads first, then the tile's (HBM) loads: a wave's loads
  // complete in order, so the table stores below wait for the tables (L2
  // hits) only, and the tile's loads stay in flight through them (round 6;
  // the other order made the table copy wait a memory latency)
  constexpr int kTabIt = (kNT * 3 * 64 + kThreads - 1) / kThreads;
  const bool t256 = tid < 256, t384 = tid < kNT * 64;
  const float lut_v = t256 ? c_lut[tid] : 0.0f, btab_v = t256 ? c_btab[tid] : 0.0f;
  const float iw_v = t384 ? c_iwperm[tid] : 0.0f;
  const uint8_t zz_v = t384 ? c_zz[tid] : 0;
  float w_v[kTabIt], sd_v[kTabIt];
#pragma unroll
  for (int k = 0; k < kTabIt; k++) {
    const int i = tid + k * kThreads;
#ifdef JXG_EXP_NOTAB  // (timing experiment only: no per-workgroup weight-table loads)
    w_v[k] = 0.25f + (float)(i & 63) * (1.0f / 64.0f);
    sd_v[k] = 1.0f + (float)(i & 31) * (1.0f / 32.0f);
#else
    w_v[k] = i < kNT * 3 * 64 ? c_wperm[i] : 0.0f;
    sd_v[k] = i < kNT * 3 * 64 ? c_sdperm[i] : 0.0f;
#endif
  }
  TileLoads TL;
  issue_tile_loads(a, ox, oy, a.gab, TL);  // in flight through the table copies
  if (t256) {
    sLut[tid] = lut_v;
    sBtab[tid] = btab_v;
  }
  if (t384) {
    sIwperm[tid] = iw_v;
    sZz[tid] = zz_v;
  }
#pragma unroll
  for (int k = 0; k < kTabIt; k++) {
    const int i = tid + k * kThreads;
    if (i < kNT * 3 * 64) {
      sWperm[i] = w_v[k];
      sSdperm[i] = sd_v[k];
    }
  }
  __syncthreads();
  FPROF(1);  // tables
  // (Gaborish: the ring beside the tile, 3 x 268 floats before phase A's sH)
  float* const ring = a.gab ? sUnion + 256 : nullptr;
  load_xyb_tile(a, sLut, sPix, ox, oy, a.gab, TL, ring);
  if (a.gab) {  // (uniform) the in-place sweep
    __syncthreads();
    FPROF(2);  // tile + ring load
    gab_sweep(sPix, ring);
    if (!(ox >= 0 && oy >= 0 && ox + 66 <= (int)a.xp && oy + 66 <= (int)a.yp)) {  // (uniform)
      __syncthreads();
      zero_outside(a, sPix, ox, oy);
    }
  }
  __syncthreads();
  FPROF(3);  // (Gaborish sweep; without it: the tile load)
  if (a.xyb_out) {
    // tile-major XYB copy for the merge stage: [tile][X, Y, B][64][64]
    float* dst = a.xyb_out + (size_t)(ty * a.tiles_x + tx) * (3 * 4096);
    // 16-byte stores; the 4 pixels lx+1..lx+4 (lx % 4 == 0) are contiguous
    // in LDS (they share a skew)
    for (int i = tid; i < 3 * 1024; i += kThreads) {
      const int c = i >> 10, ly = (i >> 4) & 63, lx = (i & 15) * 4;
      const float* q = sPix + c * kPlane + lds_at(lx + 1, ly + 1);
      reinterpret_cast<float4*>(dst)[i] = make_float4(q[0], q[1], q[2], q[3]);
    }
  }
  FPROF(4);  // XYB tile copy
  const int nbx = min(8, (int)a.bxs - tx * 8), nby = min(8, (int)a.bys - ty * 8);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const size_t nb = (size_t)a.bxs * a.bys;
  const Tile tile{sPix, sPix + kPlane, sPix + 2 * kPlane, ox, oy};
  // ---- phase A: thesis homogeneity; wave w = region w, lane = block ----
  if (a.proposals & 3u) {
    const int lbx = lane & 7, lby = lane >> 3;
    lap_bits(tile, edge_threshold(a.distance), sLapBits);
    __syncthreads();
    if (lbx < nbx && lby < nby)
      sH[wave][lane] = homog_region(tile, sLapBits, wave, tx * kTile + lbx * 8,
                                    ty * kTile + lby * 8, a.distance, (int)a.yp, a.h1_int);
    __syncthreads();
    if (tid < 64 && lbx < nbx && lby < nby) {
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
    __syncthreads();
  }
  FPROF(5);  // phase A
  // ---- phase B: wave w = block row, 8-lane group g = block column ----
  const int g = lane >> 3, r = lane & 7;
  const int lbx = g, lby = wave;
  const int b = lby * 8 + lbx;
  // chroma from luma (oracle jxo_cfl_tile): weighted least squares of X on Y
  // and of B - Y on Y over the tile's DCT8 AC coefficients; lane r of a block
  // accumulates its coefficient column, the block's 8 lanes tree-sum, the
  // tile sums its blocks in raster order (phase-A scratch sH reused)
  float kx = 0.0f, kb = 1.0f;
  // the fit's 8-point row passes (transposed: lane r = working column r) of
  // Y and (X, B) are those of the DCT8 and DCT8X4 candidates too: kept for
  // phase C, which only adds their column transforms
  float rty[8];  // Y
  f2 rtxb[8];    // (X, B)
  if (a.effort >= 5) {
    float* cs = &sH[0][0];  // [4 sums][64 blocks]
    {
      const GroupCtx G0{sPix, lby * 8 + 1, lbx * 8 + 1, r, sWperm, sIwperm, sBtab, sSdperm,
                        0.0f, 1.0f};
      row_pass_t<true, 1>(G0, rty);
      row_pass_t<true, kXB>(G0, rtxb);
      float vy[8], vx[8], vb[8];
      f2 cxb[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        vy[k] = rty[k];
        cxb[k] = rtxb[k];
      }
      dct8_1d(vy);
      dct8_1d(cxb);
#pragma unroll
      for (int k = 0; k < 8; k++) {
        vx[k] = cxb[k].x;
        vb[k] = cxb[k].y;
      }
      const float* wx = sWperm + (0 * 8 + r) * 8;  // DCT8 weights, X: [r][k]
      const float* wbp = sWperm + (2 * 8 + r) * 8; // DCT8 weights, B
      float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if (k == 0 && r == 0) continue;  // DC
        const float w2x = wx[k] * wx[k], w2b = wbp[k] * wbp[k];
        a0 = fmaf(w2x * vx[k], vy[k], a0);
        a1 = fmaf(w2x * vy[k], vy[k], a1);
        a2 = fmaf(w2b * (vb[k] - vy[k]), vy[k], a2);
        a3 = fmaf(w2b * vy[k], vy[k], a3);
      }
      a0 = group_tree_sum(a0);
      a1 = group_tree_sum(a1);
      a2 = group_tree_sum(a2);
      a3 = group_tree_sum(a3);
      if (r == 0) {
        cs[b] = a0;
        cs[64 + b] = a1;
        cs[128 + b] = a2;
        cs[192 + b] = a3;
      }
    }
    __syncthreads();
    if (tid < 4) {
      // the tile's sum in raster order, the same float adds; the partials come
      // in 16-byte loads, 16 at a time (a dependent LDS read per add before:
      // round 6), and a block outside a partial tile adds +0 instead of being
      // skipped -- the same sum: T starts at +0 and a sum is -0 only when both
      // of its terms are, so T + 0 = T at every step
      float T = 0.0f;
      const float4* row = reinterpret_cast<const float4*>(cs + tid * 64);
#pragma unroll
      for (int q0 = 0; q0 < 16; q0 += 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = row[q0 + u];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int bb = (q0 + u) * 4 + j;
            T = T + (((bb & 7) < nbx && (bb >> 3) < nby) ? e[j] : 0.0f);
          }
        }
      }
      cs[256 + tid] = T;
    }
    __syncthreads();
    const float T0 = cs[256], T1 = cs[257], T2 = cs[258], T3 = cs[259];
    __syncthreads();  // cs (sH) is phase D's staging from here on
    const int ytox = cfl_quant(T1 > 0.0f ? T0 / T1 : 0.0f);
    const int ytob = cfl_quant(T3 > 0.0f ? T2 / T3 : 0.0f);
    kx = (float)ytox * (1.0f / 84.0f);
    kb = 1.0f + (float)ytob * (1.0f / 84.0f);
    if (tid == 0 && a.cmap) {
      const size_t t = (size_t)ty * a.tiles_x + tx;
      a.cmap[t] = (int8_t)ytox;
      a.cmap[a.ntiles_all + t] = (int8_t)ytob;
    }
  } else {
    if (tid == 0 && a.cmap) {
      const size_t t = (size_t)ty * a.tiles_x + tx;
      a.cmap[t] = 0;
      a.cmap[a.ntiles_all + t] = 0;
    }
    // (no fit below effort 5: the DCT8 candidate's row passes alone)
    const GroupCtx G0{sPix, lby * 8 + 1, lbx * 8 + 1, r, sWperm, sIwperm, sBtab, sSdperm,
                      0.0f, 1.0f};
    row_pass_t<true, 1>(G0, rty);
    row_pass_t<true, kXB>(G0, rtxb);
  }
  FPROF(6);  // phase B (CfL fit / row passes)
  if (lbx >= nbx || lby >= nby) return;  // whole groups leave; no barrier follows
  // block index (recomputed where used: keeps a 64-bit value out of the
  // candidate search's live registers)
  auto gblock = [&]() { return (size_t)(ty * 8 + lby) * a.bxs + tx * 8 + lbx; };
  size_t gb = gblock();
  const GroupCtx G{sPix, lby * 8 + 1, lbx * 8 + 1, r, sWperm, sIwperm, sBtab, sSdperm, kx, kb};
  // block DC (row partials, tree over rows) and AQ activity
  float dc[3];
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const float* pl = sPix + c * kPlane + lds_at(G.lx0, G.ly0 + r);
    float rs = 0.0f;
#pragma unroll
    for (int x = 0; x < 8; x++) rs += pl[x];
    dc[c] = group_tree_sum(rs) * (1.0f / 64.0f);
  }
  const float* Yr = sPix + kPlane + lds_at(G.lx0, G.ly0 + r);
  const float* Yn = sPix + kPlane + lds_at(G.lx0, G.ly0 + r + 1);
  float hr = 0.0f, vr = 0.0f;
#pragma unroll
  for (int x = 0; x < 7; x++) hr += fabsf(Yr[x + 1] - Yr[x]);
  if (r < 7) {
#pragma unroll
    for (int x = 0; x < 8; x++) vr += fabsf(Yn[x] - Yr[x]);
  }
  const float act = group_tree_sum(hr + vr);
  const float am = act * (1.0f / 112.0f);
  float mult = 1.5f / sqrtf(1.0f + am * 40.0f);
  if (mult < 0.45f) mult = 0.45f;
  if (mult > 1.5f) mult = 1.5f;
  const float qff = a.qf_base * mult;
  int raw = (int)(qff * a.inv_g + 0.5f);
  raw = raw < 1 ? 1 : (raw > 256 ? 256 : raw);
  if (a.qf_in) raw = (int)a.qf_in[gb] + 1;  // the masking quant field (jxg_aq.hip)
  if (r == 0) {
    const float vy = dc[1] * a.dc_mul[1];
    const int qy = vy >= 0.0f ? (int)(vy + 0.5f) : -(int)(-vy + 0.5f);
    const float ydq = (float)qy * a.dc_step[1];
    const float xv = dc[0] * a.dc_mul[0];
    const float bv = (dc[2] - ydq) * a.dc_mul[2];
    a.dc[nb + gb] = qy;
    a.dc[gb] = xv >= 0.0f ? (int)(xv + 0.5f) : -(int)(-xv + 0.5f);
    a.dc[2 * nb + gb] = bv >= 0.0f ? (int)(bv + 0.5f) : -(int)(-bv + 0.5f);
  }
  if (r == 0) a.qf[gb] = (uint8_t)(raw - 1);
  const float scale = (float)a.G * (float)raw / 65536.0f;
  const float inv_scale = 1.0f / scale;
  FPROF(7);  // DC + AQ
  // ---- phase C: strategy search (FindBest8x8Transform [ext] + hooks) ----
  const int ncand = a.effort >= 5 ? 6 : 1;
  const bool hookF = (a.proposals & 2u) != 0 && ncand > 1;
#ifndef JXG_FRONT_PRUNE  // (A/B builds: -DJXG_FRONT_PRUNE=0)
#define JXG_FRONT_PRUNE 1
#endif
  const bool prune = JXG_FRONT_PRUNE != 0;
  // hook P target (combined.diff:270-274) is known before the search: it only
  // depends on the homogeneity indices; its coefficients are kept aside
  int pt = kDCT8;
  float rh = 0.0f, rv = 0.0f, rd = 0.0f;
  if (a.proposals & 3u) {
    rh = sR[b][0];
    rv = sR[b][1];
    rd = sR[b][2];
  }
  // hook P lives in FindBest8x8Transform, which libjxl does not run below
  // effort 5 (all-DCT8 speed tiers [ext]): no override there either
  if (HOOKP && (a.proposals & 1u) && ncand > 1) pt = partition_of(rh, rv, rd, a.distance);
  // scan indices: DCT8 0, DCT4X4 1, DCT2X2 2, DCT4X8 3, DCT8X4 4, IDENTITY 5.
  // `beats` is a strict total order on (estimate, scan index) in which every
  // estimate that is not below FLT_MAX ranks after the finite ones, so any
  // evaluation order finds the scan's winner.  Round 6: DCT8X4 and DCT8 first
  // (the fit's 8-point row passes, which die after them; DCT8X4 before DCT8
  // so that no winner's coefficients are held during the first evaluation),
  // then the others from the pixels in one rolled loop -- one transform
  // dispatch and one quantization body (eval_cand) for four candidates.
  // The best estimate is normalised to FLT_MAX when it is not finite, as the
  // scan's first candidate always was; pruning needs a finite best (then a
  // pruned candidate's NaN cannot win; with a non-finite best it could, by
  // its scan index).
  QVals best;
  int bt = kDCT8, bi = 0;
  float beste = FLT_MAX;
  if (ncand > 1) {
    CandAcc A;
    const Prune pr{false, beste, hookF, rh, rv, rd};
    float e = eval_cand<true>(G, kDCT8X4, scale, inv_scale, A, rty, rtxb, pr);
    if (hookF) e = hook_f(e, rh, rv, rd);
    copy_q(best, A.q, true);
    bt = kDCT8X4;
    bi = 4;
    beste = e < FLT_MAX ? e : FLT_MAX;
  }
  {
    CandAcc A;
    const Prune pr{ncand > 1 && prune && beste < FLT_MAX, beste, hookF, rh, rv, rd};
    float e = eval_cand<true>(G, kDCT8, scale, inv_scale, A, rty, rtxb, pr);
    if (hookF) e = hook_f(e, rh, rv, rd);
    if (ncand == 1 || beats(e, 0, beste, bi)) {
      copy_q(best, A.q, true);
      bt = kDCT8;
      bi = 0;
      beste = ncand > 1 && e < FLT_MAX ? e : FLT_MAX;
    }
  }
  // DCT4X4, DCT4X8, DCT2X2, IDENTITY; then (HOOKP) hook P's override
  // (combined.diff:270-274): when the scan kept DCT8, the partition's
  // candidate is evaluated again (keeping it aside through the search would
  // hold 13 more VGPRs; same inputs, same values) and replaces it
  const int n1 = ncand > 1 ? 4 : 0;
#pragma unroll 1
  for (int idx = 0;; idx++) {
    const bool over = idx == n1;  // past the scan: hook P's override, if any
    if (over && !(HOOKP && bt == kDCT8 && pt != kDCT8)) break;
    const int T = over ? pt : (idx == 0 ? kDCT4X4 : (idx == 1 ? kDCT4X8 : (idx == 2 ? kDCT2X2 : kIDENTITY)));
    const int si = idx == 0 ? 1 : (idx == 1 ? 3 : (idx == 2 ? 2 : 5));
    CandAcc A;
    const Prune pr{!over && prune && beste < FLT_MAX, beste, hookF, rh, rv, rd};
    float e = eval_cand<false>(G, T, scale, inv_scale, A, nullptr, nullptr, pr);
    if (over) {
      bt = pt;
      copy_q(best, A.q, true);
      break;
    }
    if (hookF) e = hook_f(e, rh, rv, rd);
    if (beats(e, si, beste, bi)) {
      copy_q(best, A.q, true);
      bt = T;
      bi = si;
      beste = e;
    }
  }
  gb = gblock();
  if (r == 0) {
    a.acs[gb] = (uint8_t)bt;
    // estimate summed by the merge stage: the search's best, stored before
    // the hook-P override (homogeneity-partitioning.diff:271 context)
    if (a.ent) a.ent[gb] = beste;
  }
  if (r < 3) a.nz[r * nb + gb] = (uint16_t)((best.nz >> (8 * r)) & 0xFFu);
  FPROF(8);  // phase C (the candidates)
  // ---- phase D: zigzag scatter through LDS, 16-byte stores ----
  const int bti = tindex_rt(bt);
  const uint2 zz2 = *reinterpret_cast<const uint2*>(sZz + bti * 64 + r * 8);
  const uint32_t zw[2] = {zz2.x, zz2.y};
  int16_t* stage = &sStage[wave][g][0];
  int16_t* out = a.ac + gb * 192;
#pragma unroll
  for (int c = 0; c < 3; c++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int pos = (zw[k >> 2] >> ((k & 3) * 8)) & 0xFF;
      stage[pos] = (int16_t)(best.w[c * 4 + (k >> 1)] >> ((k & 1) * 16));
    }
    wave_lds_sync();
    *reinterpret_cast<uint4*>(out + c * 64 + 8 * r) =
        *reinterpret_cast<const uint4*>(stage + 8 * r);
    wave_lds_sync();
  }
  FPROF(9);  // phase D
}


// standalone thesis selector over a given XYB frame (parity entry point)
__global__ __launch_bounds__(kThreads) void homog_kernel(HomogArgs a) {
  __shared__ float sPix[3 * kPlane];
  __shared__ float sH[8][64];
  __shared__ uint64_t sLapBits[64];
  const int tid = threadIdx.x;
  const int tx = blockIdx.x, ty = blockIdx.y;
  const int ox = tx * kTile - 1, oy = ty * kTile - 1;
  for (int i = tid; i < kRows * 66; i += kThreads) {
    const int ly = i / 66, lx = i - ly * 66;
    const int gx = ox + lx, gy = oy + ly;
    const bool in = gx >= 0 && gy >= 0 && gx < (int)a.xsize && gy < (int)a.ysize;
    const size_t o = (size_t)gy * a.stride + gx;
    const int l = lds_at(lx, ly);
    sPix[l] = in ? a.xyb[o] : 0.0f;
    sPix[kPlane + l] = in ? a.xyb[a.plane + o] : 0.0f;
    sPix[2 * kPlane + l] = in ? a.xyb[2 * a.plane + o] : 0.0f;
  }
  __syncthreads();
  const int bxs = (int)a.xsize / 8, bys = (int)a.ysize / 8;
  const int wave = tid >> 6, lane = tid & 63;
  const int lbx = lane & 7, lby = lane >> 3;
  const bool valid = tx * 8 + lbx < bxs && ty * 8 + lby < bys;
  const Tile tile{sPix, sPix + kPlane, sPix + 2 * kPlane, ox, oy};
  lap_bits(tile, edge_threshold(a.distance), sLapBits);
  __syncthreads();
  if (valid)
    sH[wave][lane] = homog_region(tile, sLapBits, wave, tx * kTile + lbx * 8, ty * kTile + lby * 8,
                                  a.distance, (int)a.ysize, a.h1_int);
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

#ifdef JXG_FRONT_PROFILE
void dump_front_profile() {
  unsigned long long h[12];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_fprof), sizeof(h)) != hipSuccess) return;
  static const char* kNames[10] = {"workgroups", "tables", "tile+ring load", "gab sweep",
                                   "xyb copy", "phase A", "phase B", "dc+aq", "phase C",
                                   "phase D"};
  std::fprintf(stderr, "front_kernel thread-0 shader cycles (Mcycles summed over workgroups):\n");
  for (int k = 0; k < 10; k++)
    std::fprintf(stderr, "  %-16s %12.3f\n", kNames[k], k ? h[k] / 1e6 : (double)h[0]);
}
#else
void dump_front_profile() {}
#endif

hipError_t set_front_constants(const float lut[256], const float wts[5][3][64], hipStream_t s) {
  static float wperm[kNT * 3 * 64], iwperm[kNT * 64], btab[256], sdperm[kNT * 3 * 64];
  static uint8_t zz[kNT * 64];
  const int types[kNT] = {kDCT8, kDCT4X4, kDCT4X8, kDCT8X4, kDCT2X2, kIDENTITY};
  // quant kinds (host quant_weights): DCT8 0, DCT4 1, DCT4X8 2, IDENTITY 3, DCT2X2 4
  const int qks[kNT] = {0, 1, 2, 2, 4, 3};
  for (int ti = 0; ti < kNT; ti++) {
    const int T = types[ti];
    const int qk = qks[ti];
    for (int r = 0; r < 8; r++)
      for (int k = 0; k < 8; k++) {
        const int co = co_index_rt(T, k, r);
        // area a coefficient's basis spans: the lowest-frequency combine slots
        // the whole block, other DCT4X4 coefficients a 4x4 sub-block, other
        // DCT4X8 / DCT8X4 ones a 4x8 half, DCT2X2 level-2 / level-1 ones a 4x4
        // quarter / 2x2 cell, IDENTITY residuals one pixel (oracle
        // jxo_frame_init)
        const int row = co >> 3, col = co & 7;
        int area = 64;
        if (ti == 1 && !(row < 2 && col < 2)) area = 16;
        if ((ti == 2 || ti == 3) && !(row < 2 && col == 0)) area = 32;
        if (ti == 4 && !(row < 2 && col < 2)) area = row < 4 && col < 4 ? 16 : 4;
        if (ti == 5 && !(row < 2 && col < 2)) area = 1;
        for (int c = 0; c < 3; c++) {
          wperm[((ti * 3 + c) * 8 + r) * 8 + k] = wts[qk][c][co];
          sdperm[((ti * 3 + c) * 8 + r) * 8 + k] = dist_weight(c, area, wts[qk][c][co]);
        }
        iwperm[(ti * 8 + r) * 8 + k] = 1.0f / wts[qk][1][co];
        zz[(ti * 8 + r) * 8 + k] = (uint8_t)c_inv_order_h(co);
      }
  }
  // AdjustQuantBias of a magnitude q: 0 -> 0, 1 -> kBias1, else q - 0.145 / q
  // (the same single-precision division and subtraction the kernel did per
  // coefficient before round 5; SSE rounds them as the GPU does, no
  // contraction is involved)
  btab[0] = 0.0f;
  btab[1] = 1.0f - 0.07005449891748593f;
  for (int q = 2; q < 256; q++) btab[q] = (float)q - 0.145f / (float)q;
  hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_lut), lut, sizeof(float) * 256, 0,
                                        hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_wperm), wperm, sizeof(wperm), 0,
                               hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_iwperm), iwperm, sizeof(iwperm), 0,
                               hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_sdperm), sdperm, sizeof(sdperm), 0,
                               hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_btab), btab, sizeof(btab), 0,
                               hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_zz), zz, sizeof(zz), 0, hipMemcpyHostToDevice, s);
  // the static host tables must outlive the copies
  const hipError_t e2 = hipStreamSynchronize(s);
  return e != hipSuccess ? e : e2;
}
// (the frames of a batch share their size and parameters)
void launch_front(const FrontArgs* a, uint32_t k, uint32_t tiles_x, uint32_t tiles_y, hipStream_t s) {
  if (!k) return;
  const Batch<FrontArgs> b = make_batch(a, k);
  const uint32_t nwg = 8 * ((tiles_x * tiles_y + 7) / 8);  // XCD-aware order (front_kernel)
  if (a[0].proposals & 1u)
    hipLaunchKernelGGL(front_kernel<true>, dim3(nwg, 1, k), dim3(kThreads), 0, s, b);
  else
    hipLaunchKernelGGL(front_kernel<false>, dim3(nwg, 1, k), dim3(kThreads), 0, s, b);
}
void launch_front_list(const FrontArgs* a, uint32_t k, uint32_t ntiles, hipStream_t s) {
  if (!ntiles || !k) return;
  const Batch<FrontArgs> b = make_batch(a, k);
  if (a[0].proposals & 1u)
    hipLaunchKernelGGL(front_kernel<true>, dim3(ntiles, 1, k), dim3(kThreads), 0, s, b);
  else
    hipLaunchKernelGGL(front_kernel<false>, dim3(ntiles, 1, k), dim3(kThreads), 0, s, b);
}
void launch_homog(const HomogArgs& a, uint32_t tiles_x, uint32_t tiles_y, hipStream_t s) {
  hipLaunchKernelGGL(homog_kernel, dim3(tiles_x, tiles_y), dim3(kThreads), 0, s, a);
}

}  // namespace jxg
