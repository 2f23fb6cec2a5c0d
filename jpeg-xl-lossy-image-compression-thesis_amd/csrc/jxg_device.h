// jxg_device.h -- gfx950 device math for the VarDCT encode path.
//
// Every float operation here follows the op order fixed in DESIGN.md §3 (and
// restated by oracle/front.c, oracle/homog.c, oracle/xyb.c) so the HIP path is
// bit-identical to the CPU oracle.  Built with -ffp-contract=off; fmaf is
// used only where written explicitly; division/sqrt are IEEE (hipcc default
// correctly-rounded f32 div/sqrt).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jxg {

// raw AcStrategy ids returned by the thesis selector
// (proposals/combined.diff:227-233)
enum : int { kDCT8 = 0, kDCT4X4 = 3, kDCT4X8 = 12, kDCT8X4 = 13 };
// the two Haar-type 8x8 candidates of the strategy search [ext AcStrategy]
enum : int { kIDENTITY = 1, kDCT2X2 = 2 };

// opsin absorbance [ext libjxl opsin_params.h]
constexpr float kM00 = 0.30f, kM01 = 0.622f, kM02 = 0.078f;
constexpr float kM10 = 0.23f, kM11 = 0.692f, kM12 = 0.078f;
constexpr float kM20 = 0.24342268924547819f, kM21 = 0.20476744424496821f,
                kM22 = 0.55180986650955360f;
constexpr float kOpsinBias = 0.0037930732552754493f;

// multiply/fma-only cube root == oracle/xyb.c jxo_cbrtf (bit-identical)
__device__ __forceinline__ float cbrt_det(float x) {
  if (!(x > 0.0f)) return 0.0f;
  const uint32_t i = 0x54a2fa8cu - __float_as_uint(x) / 3u;
  float r = __uint_as_float(i);
#pragma unroll
  for (int it = 0; it < 3; it++) {
    const float r3 = (r * r) * r;
    const float e = fmaf(-x, r3, 1.0f);
    r = fmaf(r * e, 0x1.555556p-2f, r);
  }
  return (x * r) * r;
}

__device__ __forceinline__ void pixel_xyb(const float* lut, float cb, uint32_t r8,
                                          uint32_t g8, uint32_t b8, float& X,
                                          float& Y, float& B) {
  const float r = lut[r8], g = lut[g8], b = lut[b8];
  float m0 = ((kM00 * r + kM01 * g) + kM02 * b) + kOpsinBias;
  float m1 = ((kM10 * r + kM11 * g) + kM12 * b) + kOpsinBias;
  float m2 = ((kM20 * r + kM21 * g) + kM22 * b) + kOpsinBias;
  m0 = cbrt_det(m0) - cb;
  m1 = cbrt_det(m1) - cb;
  m2 = cbrt_det(m2) - cb;
  X = 0.5f * (m0 - m1);
  Y = 0.5f * (m0 + m1);
  B = m2;
}

// Two pixels at once: every float multiply / add / fma is one packed op
// (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32), each half exactly the scalar
// op, so the results are cbrt_det's / pixel_xyb's bit for bit at about half
// the float instructions.  A half whose input is not > 0 runs the iterations
// on a meaningless seed and is replaced by 0 at the end (no traps on the GPU).
typedef float pf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf2 cbrt_det2(pf2 x) {
  pf2 r = {__uint_as_float(0x54a2fa8cu - __float_as_uint(x.x) / 3u),
           __uint_as_float(0x54a2fa8cu - __float_as_uint(x.y) / 3u)};
  const pf2 one = {1.0f, 1.0f}, third = {0x1.555556p-2f, 0x1.555556p-2f};
#pragma unroll
  for (int it = 0; it < 3; it++) {
    const pf2 r3 = (r * r) * r;
    const pf2 e = __builtin_elementwise_fma(-x, r3, one);
    r = __builtin_elementwise_fma(r * e, third, r);
  }
  pf2 y = (x * r) * r;
  y.x = x.x > 0.0f ? y.x : 0.0f;
  y.y = x.y > 0.0f ? y.y : 0.0f;
  return y;
}
// linear RGB of two pixels -> opsin (m0, m1, m2) before the cube roots
__device__ __forceinline__ void opsin2(pf2 r, pf2 g, pf2 b, pf2& m0, pf2& m1, pf2& m2) {
  const pf2 bias = {kOpsinBias, kOpsinBias};
  m0 = ((kM00 * r + kM01 * g) + kM02 * b) + bias;
  m1 = ((kM10 * r + kM11 * g) + kM12 * b) + bias;
  m2 = ((kM20 * r + kM21 * g) + kM22 * b) + bias;
}
__device__ __forceinline__ void pixel_xyb2(const float* lut, float cb, const uint32_t* r8,
                                           const uint32_t* g8, const uint32_t* b8, pf2& X,
                                           pf2& Y, pf2& B) {
  const pf2 r = {lut[r8[0]], lut[r8[1]]}, g = {lut[g8[0]], lut[g8[1]]},
            b = {lut[b8[0]], lut[b8[1]]};
  pf2 m0, m1, m2;
  opsin2(r, g, b, m0, m1, m2);
  const pf2 cb2 = {cb, cb};
  m0 = cbrt_det2(m0) - cb2;
  m1 = cbrt_det2(m1) - cb2;
  m2 = cbrt_det2(m2) - cb2;
  X = 0.5f * (m0 - m1);
  Y = 0.5f * (m0 + m1);
  B = m2;
}

// thesis hook F (combined.diff:247-253): ret * 0.8 * avg_r in double, stored
// to float
__device__ __forceinline__ float hook_f(float ret, float rh, float rv, float rd) {
  const float avg_r = (rh + rv + rd) / 3.0f;
  return (float)((double)ret * 0.8 * (double)avg_r);
}

// DC quantization of one block == oracle jxo_quant_dc: Y first, B residual
// against the dequantized Y (base correlation b = 1.0, x = 0.0) [ext]
__device__ __forceinline__ void quant_dc3(const float* dc, const float* dc_mul,
                                          const float* dc_step, int32_t* q) {
  const float vy = dc[1] * dc_mul[1];
  const int qy = vy >= 0.0f ? (int)(vy + 0.5f) : -(int)(-vy + 0.5f);
  const float ydq = (float)qy * dc_step[1];
  const float xv = dc[0] * dc_mul[0];
  const float bv = (dc[2] - ydq) * dc_mul[2];
  q[1] = qy;
  q[0] = xv >= 0.0f ? (int)(xv + 0.5f) : -(int)(-xv + 0.5f);
  q[2] = bv >= 0.0f ? (int)(bv + 0.5f) : -(int)(-bv + 0.5f);
}

// [ext] AC context model tables (libjxl ac_context.h)
__device__ __constant__ static const uint8_t kStrategyOrder[27] = {
    0, 1, 1, 1, 2, 3, 4, 4, 5, 5, 6, 6, 1, 1, 1, 1, 1, 1, 7, 8, 8, 9, 10, 10, 11, 12, 12};
__device__ __constant__ static const uint8_t kDefaultCtxMap[39] = {
    0, 1, 2, 2, 3,  3,  4,  5,  6,  6,  6,  6,  6,  7, 8, 9, 9, 10, 11, 12,
    13, 14, 14, 14, 14, 14, 7, 8, 9, 9, 10, 11, 12, 13, 14, 14, 14, 14, 14};
__device__ __constant__ static const uint8_t kFreqCtx[64] = {
    0,  0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 15, 16, 16, 17, 17,
    18, 18, 19, 19, 20, 20, 21, 21, 22, 22, 23, 23, 23, 23, 24, 24, 24, 24, 25, 25, 25, 25,
    26, 26, 26, 26, 27, 27, 27, 27, 28, 28, 28, 28, 29, 29, 29, 29, 30, 30, 30, 30};
__device__ __constant__ static const uint16_t kNnzCtx[64] = {
    0,   0,   31,  62,  62,  93,  93,  93,  93,  123, 123, 123, 123, 152, 152, 152,
    152, 152, 152, 152, 152, 180, 180, 180, 180, 180, 180, 180, 180, 180, 180, 180,
    180, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206,
    206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206};

constexpr int kBlockCtx = 15, kNzBuckets = 37, kZdCtx = 458;
constexpr int kAcCtx = kBlockCtx * (kNzBuckets + kZdCtx);  // 7425
constexpr int kMaxClusters = 132;
constexpr int kAlpha = 128;

__host__ __device__ __forceinline__ int bclass(int bctx) {
  if (bctx < 7) return bctx == 0 ? 0 : (bctx == 1 ? 1 : 2);
  return bctx == 7 ? 3 : (bctx == 8 ? 4 : 5);
}
// static clustering of the 7425 AC contexts (the map is transmitted)
__host__ __device__ __forceinline__ int ac_cluster(int ctx) {
  if (ctx < kBlockCtx * kNzBuckets) {
    int bucket = ctx / kBlockCtx, bctx = ctx % kBlockCtx;
    int nb = bucket == 0 ? 0 : (bucket <= 2 ? 1 : (bucket <= 8 ? 2 : 3));
    return bclass(bctx) * 4 + nb;
  }
  int z = ctx - kBlockCtx * kNzBuckets;
  int bctx = z / kZdCtx, zz = z % kZdCtx;
  int prev = zz & 1, base = zz >> 1;
  int bi = base >= 206 ? 7 : base >= 180 ? 6 : base >= 152 ? 5 : base >= 123 ? 4
         : base >= 93 ? 3 : base >= 62 ? 2 : base >= 31 ? 1 : 0;
  const int nzb_base = bi == 7 ? 206 : bi == 6 ? 180 : bi == 5 ? 152 : bi == 4 ? 123
                     : bi == 3 ? 93 : bi == 2 ? 62 : bi == 1 ? 31 : 0;
  int fc = base - nzb_base;
  int nzg = bi < 2 ? 0 : (bi < 4 ? 1 : 2);
  int fg = fc < 4 ? 0 : (fc < 12 ? 1 : 2);
  return 24 + ((bclass(bctx) * 3 + nzg) * 3 + fg) * 2 + prev;
}

__host__ __device__ __forceinline__ uint32_t pack_signed(int32_t v) {
  return v >= 0 ? (uint32_t)v * 2u : (uint32_t)(-(int64_t)v) * 2u - 1u;
}

// hybrid-uint (split_exponent 4, msb_in_token 2, lsb_in_token 0)
__host__ __device__ __forceinline__ void hybrid420(uint32_t v, uint32_t& tok, uint32_t& nb,
                                                   uint32_t& bits) {
  if (v < 16u) {
    tok = v;
    nb = 0;
    bits = 0;
    return;
  }
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t n = 31u - (uint32_t)__clz(v);
#else
  uint32_t n = 31u - (uint32_t)__builtin_clz(v);
#endif
  uint32_t m = v - (1u << n);
  tok = 16u + ((n - 4u) << 2) + (m >> (n - 2u));
  nb = n - 2u;
  bits = v & ((1u << nb) - 1u);
}

// natural coefficient order of an 8x8 varblock [ext coeff_order.cc]:
// zigzag index -> raster position, computable at compile time
struct Order64 {
  uint8_t v[64];
};
__host__ __device__ constexpr Order64 make_order64() {
  Order64 o{};
  int cur = 1;
  o.v[0] = 0;
  for (int i = 0; i < 8; i++)
    for (int j = 0; j <= i; j++) {
      int x = j, y = i - j;
      if (i & 1) {
        int t = x;
        x = y;
        y = t;
      }
      if (x == 0 && y == 0) continue;
      o.v[cur++] = (uint8_t)(y * 8 + x);
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
      o.v[cur++] = (uint8_t)(y * 8 + x);
    }
  }
  return o;
}
__host__ __device__ constexpr int c_order_h(int j) { return make_order64().v[j]; }
__host__ __device__ constexpr int c_inv_order_h(int k) {
  const Order64 o = make_order64();
  for (int j = 0; j < 64; j++)
    if (o.v[j] == k) return j;
  return 0;
}
// transform working-array element (prow, pcol) -> raster position in the
// 8x8 coefficient layout of strategy T (oracle/front.c co_index); only
// (0, 0) maps to the DC slot
__host__ __device__ __forceinline__ int co_index_rt(int T, int prow, int pcol) {
  if (T == kDCT8) return prow * 8 + pcol;
  // IDENTITY / DCT2X2: lane pcol's value prow (front kernel haar_lane)
  if (T == kIDENTITY) return ((pcol >> 2) + 2 * (pcol & 3)) * 8 + (prow >> 2) + 2 * (prow & 3);
  if (T == kDCT2X2) {
    const int q = pcol >> 1;
    const int row = (pcol & 1) ? 4 + q : (prow >= 4 ? q : ((q & 1) ? 2 + (q >> 1) : (q >> 1)));
    return row * 8 + prow;
  }
  if (T == kDCT4X4) return ((prow >> 2) + 2 * (prow & 3)) * 8 + (pcol >> 2) + 2 * (pcol & 3);
  if (T == kDCT8X4) return ((prow >> 2) + 2 * (prow & 3)) * 8 + pcol;
  return ((pcol >> 2) + 2 * (pcol & 3)) * 8 + prow;  // kDCT4X8
}

__device__ __forceinline__ int nz_bucket(int n) {
  if (n >= 64) n = 64;
  return n < 8 ? n : 4 + n / 2;
}

// Lane exchange inside 8-lane groups with DPP (no LDS traffic, no address
// VGPRs): xor 1 / 2 are quad permutes; xor 4 = quad_perm(3,2,1,0) followed by
// row_half_mirror (i -> 7 - i), since (i ^ 3) ^ 7 = i ^ 4.  Every source lane
// is in the caller's (fully active) group.
template <int D>
__device__ __forceinline__ uint32_t xor_lane_u(uint32_t v) {
  static_assert(D == 1 || D == 2 || D == 4, "xor distance");
  if (D == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  if (D == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  const int t = __builtin_amdgcn_mov_dpp((int)v, 0x1B, 0xF, 0xF, false);
  return (uint32_t)__builtin_amdgcn_mov_dpp(t, 0x141, 0xF, 0xF, false);
}
template <int D>
__device__ __forceinline__ float xor_lane(float v) {
  return __uint_as_float(xor_lane_u<D>(__float_as_uint(v)));
}
// value of lane K of this lane's 8-lane group (ds_swizzle bitmask mode:
// and 0x18, or K, within 32-lane halves)
template <int K>
__device__ __forceinline__ float group_lane(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x18 | (K << 5)));
}

// bit sink writing into a zero-initialised word buffer with atomicOr
struct BitSink {
  uint32_t* buf;
  uint64_t pos;  // absolute bit position of acc's bit 0
  uint64_t acc;
  int n;
  __device__ __forceinline__ void flush_word(uint32_t lo, int nb) {
    if (nb == 0) return;
    const uint64_t w = pos >> 5;
    const int sh = (int)(pos & 31);
    atomicOr(&buf[w], lo << sh);
    if (sh && (sh + nb > 32)) atomicOr(&buf[w + 1], lo >> (32 - sh));
  }
  __device__ __forceinline__ void put(uint32_t nbits, uint32_t v) {
    if (nbits == 0) return;
    acc |= (uint64_t)v << n;
    n += (int)nbits;
    if (n >= 32) {
      flush_word((uint32_t)acc, 32);
      pos += 32;
      acc >>= 32;
      n -= 32;
    }
  }
  __device__ __forceinline__ void finish() { flush_word((uint32_t)acc, n); }
};

}  // namespace jxg
