// jxg_aq.hip -- the libjxl-shaped masking quant field on gfx950
// (JXG_FLAG_AQ_MASKING; oracle/aq.c jxo_aq_masking, bit for bit).
//
// [ext] libjxl InitialQuantField / AdaptiveQuantizationMap restated as
// recalled (parity with libjxl unpinned; oracle/aq.c lists the stages).  The
// field is what ACSConfig carries into the AC-strategy search
// (proposals/combined.diff:412-418 context).  One 256-thread workgroup per
// 64x64 tile, launched before the front kernel, which takes the block's raw
// quant field from it instead of its activity heuristic:
//   1. RGB8 -> X, Y (two cube roots; B is not needed) of the tile and a 5 px
//      ring, coordinates clamped to the padded frame, into LDS;
//   2. the pre-erosion cells (4x4) of the tile and a one-cell ring: thread =
//      (cell, pixel column), its 4 gamma-weighted, masked neighbour
//      differences, then a thread per cell sums the 4 columns;
//   3. fuzzy erosion, thread = cell: the 4 smallest of the clamped 3 x 3
//      neighbourhood, weighted;
//   4. per block, 8 lanes = its pixel columns: HF and gamma sums over the
//      rows, 8-lane tree sums, then the mask, the modulations and FastPow2f
//      -> raw quant field.
// Every float op in oracle/aq.c's order (explicit fmaf, IEEE division and
// square root).
#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

constexpr int kAqThreads = 256;
constexpr int kAqRing = 5;                 // pixels beside the tile
constexpr int kAqR = 64 + 2 * kAqRing;     // 74 region rows / columns
constexpr int kAqS = kAqR + 1;             // LDS row stride
constexpr int kAqC = 18;                   // cells of the tile and its one-cell ring

__device__ __forceinline__ float aq_fast_log2f(float x) {
  const float p0 = -1.8503833400518310E-06f, p1 = 1.4287160470083755E+00f,
              p2 = 7.4245873327820566E-01f;
  const float q0 = 9.9032814277590719E-01f, q1 = 1.0096718572241148E+00f,
              q2 = 1.7409343003366853E-01f;
  const int32_t xb = (int32_t)__float_as_uint(x);
  const int32_t es = (xb - 0x3f2aaaab) >> 23;
  const float m = __uint_as_float((uint32_t)(xb - (int32_t)((uint32_t)es << 23)));
  const float t = m - 1.0f;
  float yp = p2, yq = q2;
  yp = fmaf(yp, t, p1);
  yq = fmaf(yq, t, q1);
  yp = fmaf(yp, t, p0);
  yq = fmaf(yq, t, q0);
  return yp / yq + (float)es;
}
__device__ __forceinline__ float aq_fast_pow2f(float x) {
  const float fl = floorf(x);
  const float e = __uint_as_float((uint32_t)(((int32_t)fl + 127) << 23));
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

// RatioOfDerivativesOfCubicRootToSimpleGamma (== oracle jxo_aq_ratio)
constexpr float kAqSgMul = 226.77216153508914f;
constexpr float kAqSgMul2 = 1.0f / 73.377132366608819f;
constexpr float kAqLog2 = 0.693147181f;
constexpr float kAqSgRetMul = kAqSgMul2 * 18.6580932135f * kAqLog2;
constexpr float kAqSgVOffset = 7.7825991679894591f;
constexpr float kAqEps = 1e-2f;
template <bool INVERT>
__device__ __forceinline__ float aq_ratio(float v) {
  constexpr float num_mul = kAqSgRetMul * 3.0f * kAqSgMul;
  constexpr float num_off = kAqEps;
  constexpr float den_off = kAqSgVOffset * kAqLog2 + kAqEps;
  constexpr float den_mul = kAqLog2 * kAqSgMul;
  if (!(v > 0.0f)) v = 0.0f;
  const float v2 = v * v;
  const float num = fmaf(num_mul, v2, num_off);
  const float den = fmaf(den_mul * v, v2, den_off);
  return INVERT ? num / den : den / num;
}

__device__ __forceinline__ float aq_masking_sqrt(float v) {
  constexpr float mul = (float)((double)211.50759899638012f * 1e8);
  return 0.25f * sqrtf(fmaf(v, sqrtf(mul), 28.0f));
}

__device__ __forceinline__ void swap_gt(float& a, float& b) {
  const float lo = a > b ? b : a, hi = a > b ? a : b;
  a = lo;
  b = hi;
}
// StoreMin4 (oracle store_min4: insert v into m0 <= m1 <= m2 <= m3, dropping
// the largest) as selects -- the same results, no branches (a branchy form
// was lowered to a scratch array)
__device__ __forceinline__ void store_min4(float v, float& m0, float& m1, float& m2, float& m3) {
  const bool c0 = v < m0, c1 = v < m1, c2 = v < m2, c3 = v < m3;
  m3 = c2 ? m2 : (c3 ? v : m3);
  m2 = c1 ? m1 : (c2 ? v : m2);
  m1 = c0 ? m0 : (c1 ? v : m1);
  m0 = c0 ? v : m0;
}

__global__ __launch_bounds__(kAqThreads) void aq_kernel(Batch<AqArgs> bt_) {
  const AqArgs& a = bt_.a[blockIdx.z];
  __shared__ float sY[kAqR * kAqS];  // Y of the tile and its 5 px ring
  __shared__ float sX[64 * 65];      // X of the tile
  __shared__ float sCell[kAqC * kAqC];
  __shared__ float sCol[kAqC * kAqC * 4];  // per cell: its 4 column sums
  __shared__ float sEro[16 * 16];
  __shared__ float sLut[256];
  const int tid = threadIdx.x;
  // a whole frame: the front kernel's XCD-aware order (XCD x = workgroup % 8
  // takes the chunk [x chunk, (x + 1) chunk) of the raster tile order), so the
  // lines of RGB8 rows neighbouring tiles share are L2 hits
  int tx, ty;
  if (a.tile_list) {
    const int tile = (int)a.tile_list[blockIdx.x];
    tx = tile % (int)a.tiles_x;
    ty = tile / (int)a.tiles_x;
  } else {
    const int ntiles = (int)a.tiles_x * (((int)a.bys + 7) >> 3), chunk = (ntiles + 7) >> 3;
    const int j = (int)(blockIdx.x >> 3), tile = (int)(blockIdx.x & 7) * chunk + j;
    if (j >= chunk || tile >= ntiles) return;
    tx = tile % (int)a.tiles_x;
    ty = tile / (int)a.tiles_x;
  }
  const int ox = tx * 64, oy = ty * 64;  // padded-frame coordinate of tile-local (0, 0)
  const int xp = (int)a.xp, yp = (int)a.yp;
  sLut[tid] = a.lut[tid];
  __syncthreads();
  // 1. X, Y of the region (padded-frame coordinates clamped; the padded
  // frame replicates the image's last column / row)
  // (pixel pairs of a row -- 74 is even -- through packed float ops,
  // cbrt_det2: the same values as one pixel at a time)
  const float cb = cbrt_det(kOpsinBias);
  const pf2 cb2 = {cb, cb};
  // Round 6: the pairs go kAqBatch at a time, every byte load of a batch
  // issued before its first conversion (the strided loop waited one memory
  // latency per pair); a pair index past the region is clamped for the loads
  // and its stores skipped.
#ifndef JXG_AQ_BATCH
#define JXG_AQ_BATCH 4
#endif
  constexpr int kPairs = kAqR * kAqR / 2, kAqBatch = JXG_AQ_BATCH;
  constexpr int kPairIt = (kPairs + kAqThreads - 1) / kAqThreads;
#pragma unroll 1
  for (int it0 = 0; it0 < kPairIt; it0 += kAqBatch) {
    uint32_t px[kAqBatch][2][3];
#pragma unroll
    for (int u = 0; u < kAqBatch; u++) {
      const int i = min(tid + (it0 + u) * kAqThreads, kPairs - 1);
      const int ly = (2 * i) / kAqR, lx0 = 2 * i - ly * kAqR;
      const int gy = min(max(oy - kAqRing + ly, 0), yp - 1);
      const uint8_t* row = a.rgb + (size_t)min(gy, (int)a.h - 1) * a.stride;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int gx = min(max(ox - kAqRing + lx0 + h, 0), xp - 1);
        const uint8_t* q = row + 3 * (size_t)min(gx, (int)a.w - 1);
        px[u][h][0] = q[0];
        px[u][h][1] = q[1];
        px[u][h][2] = q[2];
      }
    }
#pragma unroll
    for (int u = 0; u < kAqBatch; u++) {
      const int i = tid + (it0 + u) * kAqThreads;
      if (it0 + u >= kPairIt || i >= kPairs) break;  // (i grows with u)
      const int ly = (2 * i) / kAqR, lx0 = 2 * i - ly * kAqR;
      pf2 r, g, b;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        r[h] = sLut[px[u][h][0]];
        g[h] = sLut[px[u][h][1]];
        b[h] = sLut[px[u][h][2]];
      }
      pf2 m0, m1, m2;
      opsin2(r, g, b, m0, m1, m2);
      m0 = cbrt_det2(m0) - cb2;
      m1 = cbrt_det2(m1) - cb2;
      const pf2 Y = 0.5f * (m0 + m1), X = 0.5f * (m0 - m1);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int lx = lx0 + h;
        sY[ly * kAqS + lx] = Y[h];
        const int tlx = lx - kAqRing, tly = ly - kAqRing;
        if (tlx >= 0 && tlx < 64 && tly >= 0 && tly < 64) sX[tly * 65 + tlx] = X[h];
      }
    }
  }
  __syncthreads();
  // Y at padded-frame coordinate (gx, gy), clamped to the frame (inside the region)
  auto Yat = [&](int gx, int gy) {
    gx = min(max(gx, 0), xp - 1);
    gy = min(max(gy, 0), yp - 1);
    return sY[(gy - (oy - kAqRing)) * kAqS + gx - (ox - kAqRing)];
  };
  auto diff = [&](int x, int y) {
    const float c = Yat(x, y);
    const float base = 0.25f * (((Yat(x, y + 1) + Yat(x, y - 1)) + Yat(x - 1, y)) + Yat(x + 1, y));
    const float gammac = aq_ratio<false>(c + 0.019f);
    float d = gammac * (c - base);
    d = d * d;
    if (d >= 0.2f) d = 0.2f;
    return aq_masking_sqrt(d);
  };
  // 2. pre-erosion cells: local (ci, cj) = global cell (16 tx - 1 + ci, 16 ty - 1 + cj);
  // item = (cell, pixel column j): the column's 4 diffs from a vertical window
  // (the sums in the oracle's order), then one thread per cell adds its columns.
  // Tiles whose cells and their 1 px ring lie inside the padded frame read the
  // region without clamps.
  const int ncx = xp / 4, ncy = yp / 4, cx0 = 16 * tx - 1, cy0 = 16 * ty - 1;
  const bool inner = tx >= 1 && ty >= 1 && 16 * tx + 17 <= ncx && 16 * ty + 17 <= ncy &&
                     64 * tx + 69 <= xp && 64 * ty + 69 <= yp;
  for (int i = tid; i < kAqC * kAqC * 4; i += kAqThreads) {
    const int cell = i >> 2, j = i & 3;
    const int gcx = cx0 + cell % kAqC, gcy = cy0 + cell / kAqC;
    if (gcx < 0 || gcy < 0 || gcx >= ncx || gcy >= ncy) continue;
    const int x = 4 * gcx + j, y = 4 * gcy;
    float s;
    if (inner) {  // (uniform) region-local rows y - 1 .. y + 4 of column x
      const float* c0 = sY + (y - (oy - kAqRing)) * kAqS + x - (ox - kAqRing);
      float up = c0[-kAqS], cc = c0[0];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const float* cr = c0 + r * kAqS;
        const float dn = cr[kAqS];
        const float base = 0.25f * (((dn + up) + cr[-1]) + cr[1]);
        const float gammac = aq_ratio<false>(cc + 0.019f);
        float d = gammac * (cc - base);
        d = d * d;
        if (d >= 0.2f) d = 0.2f;
        const float dv = aq_masking_sqrt(d);
        s = r == 0 ? dv : s + dv;
        up = cc;
        cc = dn;
      }
    } else {
      s = diff(x, y);
#pragma unroll
      for (int r = 1; r < 4; r++) s += diff(x, y + r);
    }
    sCol[i] = s;
  }
  __syncthreads();
  for (int i = tid; i < kAqC * kAqC; i += kAqThreads) {
    const float* c = sCol + 4 * i;
    sCell[i] = (((c[0] + c[1]) + c[2]) + c[3]) * 0.25f;
  }
  __syncthreads();
  // 3. fuzzy erosion of the tile's cells (neighbours clamped to the cell grid)
  {
    const int gcx = 16 * tx + (tid & 15), gcy = 16 * ty + (tid >> 4);
    if (gcx < ncx && gcy < ncy) {
      auto C = [&](int x, int y) {
        x = min(max(x, 0), ncx - 1);
        y = min(max(y, 0), ncy - 1);
        return sCell[(y - cy0) * kAqC + x - cx0];
      };
      float m0 = C(gcx, gcy), m1 = C(gcx - 1, gcy), m2 = C(gcx + 1, gcy), m3 = C(gcx - 1, gcy - 1);
      swap_gt(m0, m1);
      swap_gt(m0, m2);
      swap_gt(m0, m3);
      swap_gt(m1, m2);
      swap_gt(m1, m3);
      swap_gt(m2, m3);
      store_min4(C(gcx, gcy - 1), m0, m1, m2, m3);
      store_min4(C(gcx + 1, gcy - 1), m0, m1, m2, m3);
      store_min4(C(gcx - 1, gcy + 1), m0, m1, m2, m3);
      store_min4(C(gcx, gcy + 1), m0, m1, m2, m3);
      store_min4(C(gcx + 1, gcy + 1), m0, m1, m2, m3);
      sEro[tid] = ((a.ew[0] * m0 + a.ew[1] * m1) + a.ew[2] * m2) + a.ew[3] * m3;
    }
  }
  __syncthreads();
  // 4. per block: lane j of an 8-lane group = pixel column j
  const int nbx = min(8, (int)a.bxs - tx * 8), nby = min(8, (int)a.bys - ty * 8);
  constexpr float valmin = 0.020602694503245016f;
#pragma unroll 1
  for (int it = 0; it < 2; it++) {
    const int item = tid + it * kAqThreads;
    const int blk = item >> 3, j = item & 7, lbx = blk & 7, lby = blk >> 3;
    if (lbx >= nbx || lby >= nby) continue;  // whole 8-lane groups
    float s = 0.0f, g = 0.0f;
#pragma unroll
    for (int dy = 0; dy < 8; dy++) {
      const int px = lbx * 8 + j, py = lby * 8 + dy;
      const float* yr = sY + (py + kAqRing) * kAqS + px + kAqRing;
      const float p = yr[0];
      s += j < 7 ? fminf(valmin, fabsf(p - yr[1])) : 0.0f;
      s += fminf(valmin, fabsf(p - (dy < 7 ? yr[kAqS] : p)));
      const float iny = p + 0.16f, inx = sX[py * 65 + px];
      const float rr = aq_ratio<true>(iny - inx), rg = aq_ratio<true>(iny + inx);
      g += 0.5f * (rr + rg);
    }
    s = s + xor_lane<1>(s);
    s = s + xor_lane<2>(s);
    s = s + xor_lane<4>(s);
    g = g + xor_lane<1>(g);
    g = g + xor_lane<2>(g);
    g = g + xor_lane<4>(g);
    if (j == 0) {
      const float* e = sEro + (2 * lby) * 16 + 2 * lbx;
      float v = ((e[0] + e[1]) + e[16]) + e[17];
      // ComputeMask (== oracle jxo_aq_mask)
      const float v1 = fmaxf(v * 0.74760422233706747f, 1e-3f);
      const float v2 = 1.0f / (v1 + 305.04035728311436f);
      const float v3 = 1.0f / fmaf(v1, v1, 2.1925739705298404f);
      const float v4 = 1.0f / fmaf(v1, v1, 0.25f * 2.1925739705298404f);
      v = -0.74174993f +
          fmaf(3.2353257320940401f, v4, fmaf(12.906028311180409f, v2, 5.0220313103171232f * v3));
      // HfModulation, GammaModulation (== oracle jxo_aq_modulate)
      const float hf = (s + -1.110929106987477f) * -0.38078920620238305f;
      v = hf + v;
      const float ratio = g * (1.0f / 64.0f);
      v = fmaf(-0.15526878023684174f * 0.693147180559945f, aq_fast_log2f(ratio), v);
      const float qf = aq_fast_pow2f(v * 1.442695041f) * a.mul + a.add;
      int raw = (int)(qf * a.inv_g + 0.5f);
      raw = raw < 1 ? 1 : (raw > 256 ? 256 : raw);
      a.qf[(size_t)(ty * 8 + lby) * a.bxs + tx * 8 + lbx] = (uint8_t)(raw - 1);
    }
  }
}

void launch_aq(const AqArgs* a, uint32_t k, uint32_t ntiles, hipStream_t s) {
  if (!ntiles || !k) return;
  // a list: one workgroup per listed tile; a whole frame: the XCD-aware grid
  const uint32_t tiles_y = (a[0].bys + 7) / 8;
  const uint32_t nwg = a[0].tile_list ? ntiles : 8 * ((a[0].tiles_x * tiles_y + 7) / 8);
  hipLaunchKernelGGL(aq_kernel, dim3(nwg, 1, k), dim3(kAqThreads), 0, s, make_batch(a, k));
}

}  // namespace jxg
