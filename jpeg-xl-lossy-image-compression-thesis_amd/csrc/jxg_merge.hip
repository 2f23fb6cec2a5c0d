// jxg_merge.hip -- merge stage of the AC-strategy search on gfx950:
// 8x8-class decisions -> 16x8 ... 64x64 varblocks, and the transform,
// quantization and LLF-derived DC of every merged varblock.
//
// Three launches over the 64x64 tiles (the unit of libjxl's ProcessRectACS,
// combined.diff:346 context):
//   merge_eval    one 256-thread workgroup per (tile, candidate shape): the
//                 shape's varblocks tile the 64x64 area, so every workgroup
//                 does the same amount of work whatever the shape -- no idle
//                 lanes at barriers.  The tile's XYB planes (written once by
//                 the front kernel) are copied into an LDS coefficient image
//                 (48 KB, 3 workgroups per CU) and transformed in place:
//                   rows    lane = (channel, varblock, row), C-point DCT in
//                           registers (64-point: two lanes, Lee's even / odd
//                           halves, wave-uniform);
//                   columns lane = (channel, varblock, column), same;
//                   quant   lane = (channel, 16-row chunk, varblock, column):
//                           Y first (its dequantized values replace its
//                           coefficients for the B residual), then X and B;
//                   reduce  lane = (varblock, column): chunk partials,
//                           (Y + X) + B, C-lane XOR tree -> estimate (+hook F).
//                 The nine shape workgroups of a tile get workgroup ids
//                 congruent mod 8, so they land on one XCD and share its L2.
//   merge_resolve one wave per tile: per level (16, 32, 64 px) and region,
//                 keep / full / two tall / two wide halves with the
//                 TryMergeAcs comparison (`candidate >= current` keeps: NaN
//                 estimates are accepted, combined.diff:294 context).
//   merge_write   one workgroup per (tile, shape) that holds chosen varblocks:
//                 the same transform + quantization, coefficients scattered to
//                 natural-order slices of the covered blocks, non-zero counts,
//                 quant field, and the DC of each covered block from the LLF.
// Float op order == oracle/merge.c (jxo_varblock, jxo_llf_dc, jxo_merge_tile).
#include <float.h>

#include <cstdio>
#include <type_traits>

#include "jxg_device.h"
#include "jxg_kernels.h"
#include "jxg_lee_tables.h"

namespace jxg {

__constant__ float c_llf_p[4 * 8];   // [log2 M][k]
__constant__ float c_llf_ib[4 * 64]; // [log2 M][n][k]

constexpr int kMThreads = 256;
#ifndef JXG_MERGE_WPE
#define JXG_MERGE_WPE 4  // waves per SIMD the eval kernel is register-capped for (4 WGs / CU)
#endif
#ifndef JXG_MERGE_WRITE_WPE
// write: 3 waves / SIMD (168 VGPRs, 8 B of scratch since round 6's column
// halves; 2: 195 VGPRs, no scratch, merge stage 1.94 vs 1.85 ms in round 5,
// profiles/r05zp).  4 (128 VGPRs, 120 B = 39 spilled VGPRs, past
// tests/test_isa_lint.py's 32) ran 0.301 vs 0.308 ms (profiles/r06mw): not
// worth the spill traffic it hides
#define JXG_MERGE_WRITE_WPE 3
#endif
constexpr int kMS = 65;  // LDS row stride (floats)
constexpr int kMPlane = 64 * kMS;

template <int N>
constexpr int ilog2c() {
  return N <= 1 ? 0 : 1 + ilog2c<N / 2>();
}

// Two independent transforms per lane: f2 holds the same element of two rows
// (or columns), so every butterfly is one packed op (v_pk_add_f32 /
// v_pk_mul_f32) with no operand shuffles; each half sees exactly the float ops
// of the scalar transform (no contraction), so results are bit-identical.
typedef float f2 __attribute__((ext_vector_type(2)));

// unnormalized DCT-II in registers, Lee's recursive even/odd split
// (== oracle/merge.c lee); T = float or f2
template <int N, class T>
__device__ __forceinline__ void lee(T* x) {
  if constexpr (N > 1) {
    constexpr int h = N / 2, l = ilog2c<N>();
    T a[h], b[h];
#pragma unroll
    for (int i = 0; i < h; i++) {
      a[i] = x[i] + x[N - 1 - i];
      b[i] = (x[i] - x[N - 1 - i]) * kLeeC[l][i];
    }
    lee<h>(a);
    lee<h>(b);
#pragma unroll
    for (int k = 0; k < h; k++) x[2 * k] = a[k];
#pragma unroll
    for (int k = 0; k < h - 1; k++) x[2 * k + 1] = b[k] + b[k + 1];
    x[N - 1] = b[h - 1];
  }
}
// normalized N-point DCT (N <= 32) of src[k * st] into x (registers)
template <int N>
__device__ __forceinline__ void dct_from(const float* src, int st, float* x) {
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = src[k * st];
  lee<N>(x);
  constexpr int l = ilog2c<N>();
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = x[k] * kLeeS[l][k];
}
// half h of the normalized N-point DCT (Lee's first split: h = 0 the even
// outputs 2k from the sums, h = 1 the odd outputs 2k+1 from the scaled
// differences) -- the same float ops as lee<N>, spread over two lanes.
// dctN_first: t[i] from x[i] and its mirror x[N - 1 - i]; dctN_rest: the
// N/2-point transform of t and the output scaling, out(k, value) for output
// 2k + h.  T = f2: two independent rows / columns with the same h.
template <int N, class T>
__device__ __forceinline__ T dctN_first(T xi, T xm, int i, int h) {
  return h == 0 ? xi + xm : (xi - xm) * kLeeC[ilog2c<N>()][i];
}
template <int N, class T, class Out>
__device__ __forceinline__ void dctN_rest(T* t, int h, Out out) {
  constexpr int l = ilog2c<N>(), H = N / 2;
  lee<H>(t);
  if (h == 0) {
#pragma unroll
    for (int k = 0; k < H; k++) out(k, t[k] * kLeeS[l][2 * k]);
  } else {
#pragma unroll
    for (int k = 0; k < H - 1; k++) out(k, (t[k] + t[k + 1]) * kLeeS[l][2 * k + 1]);
    out(H - 1, t[H - 1] * kLeeS[l][N - 1]);
  }
}
template <class T>
__device__ __forceinline__ T dct64_first(T xi, T xm, int i, int h) {
  return dctN_first<64>(xi, xm, i, h);
}
template <class T, class Out>
__device__ __forceinline__ void dct64_rest(T* t, int h, Out out) {
  dctN_rest<64>(t, h, out);
}

// JXG_MERGE_PROFILE (experiment builds only): per (shape, phase) cycle sums
// of thread 0 of every eval workgroup, printed by dump_merge_profile()
#ifdef JXG_MERGE_PROFILE
__device__ unsigned long long g_mprof[16][8];
#define MPROF_MARK(k)                                                 \
  do {                                                                \
    if (!WRITE && threadIdx.x == 0) {                                 \
      const unsigned long long now_ = __builtin_readcyclecounter();   \
      if ((k) > 0) atomicAdd(&g_mprof[P.si][(k)], now_ - mprof_t0);   \
      mprof_t0 = now_;                                                \
    }                                                                 \
  } while (0)
#else
#define MPROF_MARK(k) \
  do {                \
  } while (0)
#endif

// merged shapes (== oracle jxo_shapes): raw id, blocks down / across (log2),
// cost multiplier
struct ShapeDesc {
  int type, lcy, lcx;
  float tmul;
};
constexpr ShapeDesc kShapes[kNumShapes] = {
    {6, 1, 0, 1.0f},   {7, 0, 1, 1.0f},   {4, 1, 1, 1.0f},
    {10, 2, 1, 1.02f}, {11, 1, 2, 1.02f}, {5, 2, 2, 1.03f},
    {19, 3, 2, 1.05f}, {20, 2, 3, 1.05f}, {18, 3, 3, 1.05f}};

__device__ __forceinline__ int bitlen_u(uint32_t v) { return 32 - __clz(v); }

// Two coefficient planes (37.9 KB: four workgroups per CU -- gfx950
// allocates LDS in 1280-byte granules, 31 granules = 39680 B is the most that
// fits four; three planes, 53.7 KB, allowed three): plane 0 holds Y (its
// dequantized values after the Y quantization, for the X / B residuals),
// plane 1 X, then B -- B is transformed into plane 1 once X is quantized.
struct MergeLds {
  float co[2 * kMPlane];  // coefficient image of the tile's varblocks
  float llf[3][64];       // write mode: the LLF of covered block b, per channel
  float qsum[3][4][32];   // [Y, X, B][chunk][varblock]: column-tree chunk sums
  float btab[256];        // AdjustQuantBias of a magnitude q < 256 (setup_varblocks)
  float vr3[32][3];       // hook F: similarity indices of each top-left block
  int vbits[32];          // per varblock: rate bits
  int vnz[32][3];         //               non-zeros per channel
  int vraw[32];           //               max quant field
  int valid[32];
  uint8_t braw[64];       // front-kernel quant field (raw) of the tile's blocks
  int any;
};
__device__ __forceinline__ float& llf_at(MergeLds& S, int c, int b) { return S.llf[c][b]; }
// the two transform passes of a tile: pass 0 = Y (plane 0) and X (plane 1),
// pass 1 = B (plane 1); local channel lc of a pass -> frame channel (X 0, Y 1,
// B 2) and LDS plane
__device__ __forceinline__ int pass_src(int pass, int lc) { return pass ? 2 : 1 - lc; }
__device__ __forceinline__ int pass_plane(int pass, int lc) { return pass ? 1 : lc; }
__device__ __forceinline__ constexpr int chan_plane(int ch) { return ch == 1 ? 0 : 1; }

// one (tile, shape) workgroup: all index math is shifts and masks
struct Pass {
  int si, type, lcy, lcx, soff, ls, tx, ty, tile;
  float tmul;
  __device__ __forceinline__ int cy() const { return 1 << lcy; }
  __device__ __forceinline__ int cx() const { return 1 << lcx; }
  __device__ __forceinline__ int R() const { return 8 << lcy; }
  __device__ __forceinline__ int C() const { return 8 << lcx; }
  __device__ __forceinline__ int lR() const { return 3 + lcy; }
  __device__ __forceinline__ int lC() const { return 3 + lcx; }
  __device__ __forceinline__ int lGX() const { return 3 - lcx; }
  __device__ __forceinline__ int lNV() const { return 6 - lcx - lcy; }
  __device__ __forceinline__ int NV() const { return 1 << lNV(); }
  __device__ __forceinline__ int bx0(int v) const { return (v & ((1 << lGX()) - 1)) << lcx; }
  __device__ __forceinline__ int by0(int v) const { return (v >> lGX()) << lcy; }
  __device__ __forceinline__ int off(int v, int plane) const {
    return plane * kMPlane + by0(v) * 8 * kMS + bx0(v) * 8;
  }
};

// workgroup id -> (tile, shape): the nine shapes of a tile share b % 8 (XCD);
// per XCD the tiles go in chunks of JXG_MERGE_CHUNK, shape-major inside a
// chunk, so the workgroups resident on a CU at a time mostly run one shape's
// code (the kernel is 53 KB of code; interleaved shapes, chunk 1, took 1.595
// ms at 8K, chunk 64 1.545 ms: profiles/r02s4_merge_chunk) while a chunk's
// tiles are still in the XCD's L2: chunk 32 (1.5 MB of XYB per XCD) fetches
// 448 MB per 8K launch, chunk 64 650 MB (the nine shape passes no longer
// find the tiles in L2), at the same merge-stage time (1.81 ms;
// chunk 16: 435 MB, 1.84 ms -- profiles/r04p/merge_chunk).
// (a shard's tiles come through a list: tile = list[index])
#ifndef JXG_MERGE_CHUNK
#define JXG_MERGE_CHUNK 32
#endif
__device__ __forceinline__ bool decode_wg(const MergeArgs& a, int& tile, int& si) {
  constexpr int T = JXG_MERGE_CHUNK;
  const int b = blockIdx.x, x = b & 7, q = b >> 3;
  const int r = q % (kNumShapes * T);
  si = r / T;
  tile = ((q / (kNumShapes * T)) * T + r % T) * 8 + x;
  if (tile >= (int)a.ntiles) return false;
  if (a.tile_list) tile = (int)a.tile_list[tile];
  return true;
}

__device__ __forceinline__ Pass make_pass(const MergeArgs& a, int tile, int si) {
  Pass P;
  P.si = si;
  const ShapeDesc& D = kShapes[si];
  P.type = D.type;
  P.lcy = D.lcy;
  P.lcx = D.lcx;
  P.tmul = D.tmul;
  P.soff = kShapeOff[si];
  P.ls = max(D.lcy, D.lcx);  // level: the s x s region (log2 blocks) of the shape
  P.tile = tile;
  P.tx = tile % (int)a.tiles_x;
  P.ty = tile / (int)a.tiles_x;
  return P;
}

// rows: C-point DCT of every row of every valid varblock, read straight
// from the tile-major XYB copy (16-byte loads; a thread issues all its rows'
// loads before the first transform) into the LDS coefficient image.  For
// C = 64 two lanes share a row (Lee halves), each reading the whole row.
template <int C>
__device__ __forceinline__ void load_row(const float* src, float* d) {
#pragma unroll
  for (int q = 0; q < C / 4; q++) {
    const float4 u = reinterpret_cast<const float4*>(src)[q];
    d[4 * q] = u.x;
    d[4 * q + 1] = u.y;
    d[4 * q + 2] = u.z;
    d[4 * q + 3] = u.w;
  }
}
template <int C, int NCH>
__device__ __forceinline__ void row_pass(const MergeArgs& a, const Pass& P, MergeLds& S, int pass) {
  const float* tsrc = a.xyb + (size_t)P.tile * (3 * 4096);
  const int R = P.R(), lvr = P.lNV() + P.lR();
  if constexpr (C == 64) {
    // item = (row pair, half h): rows r and r + 1 of one varblock and channel
    // (R >= 32: pairs never straddle a varblock); h is wave-uniform: waves
    // alternate h over 64-pair chunks
    const int npairs = NCH * P.NV() * R / 2;  // 64 / 32
    const int n = ((npairs + 63) >> 6) << 7;
    for (int i = threadIdx.x; i < n; i += kMThreads) {
      const int h = (i >> 6) & 1, pp = ((i >> 7) << 6) | (i & 63), r = pp * 2;
      if (pp >= npairs) continue;
      const int c = r >> lvr, v = (r >> P.lR()) & (P.NV() - 1), y = r & (R - 1);
      if (!S.valid[v]) continue;
      const float4* s0 =
          reinterpret_cast<const float4*>(tsrc + pass_src(pass, c) * 4096 + (P.by0(v) * 8 + y) * 64);
      const float4* s1 = s0 + 16;  // row y + 1
      f2 t[32];
      // 16-byte loads of x[4q..4q+3] and of its mirror x[60-4q..63-4q]
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const float4 a0 = s0[q], b0 = s0[15 - q], a1 = s1[q], b1 = s1[15 - q];
        const float fa0[4] = {a0.x, a0.y, a0.z, a0.w}, fb0[4] = {b0.x, b0.y, b0.z, b0.w};
        const float fa1[4] = {a1.x, a1.y, a1.z, a1.w}, fb1[4] = {b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int j = 0; j < 4; j++)
          t[4 * q + j] = dct64_first(f2{fa0[j], fa1[j]}, f2{fb0[3 - j], fb1[3 - j]}, 4 * q + j, h);
      }
      const int off = P.off(v, pass_plane(pass, c)) + y * kMS;
      dct64_rest(t, h, [&](int k, f2 o) {
        S.co[off + 2 * k + h] = o.x;
        S.co[off + kMS + 2 * k + h] = o.y;
      });
    }
  } else {
    // thread: row pairs (r, r + 256) -- two rows per transform (f2 lanes).
    // Row r of a channel: the varblock column is the fastest index, so the
    // lanes of a wave read whole 256-byte tile rows (coalesced) instead of
    // one C-float chunk per cache line
    constexpr int PER = (NCH * 4096 / C + kMThreads - 1) / kMThreads;  // 2 ch: 4, 2, 1
    const int nrows = NCH * P.NV() * R;
    const int lgx = P.lGX();
    auto row_of = [&](int rr, int& c, int& v, int& y) {
      c = rr >> lvr;
      const int i = rr & ((1 << lvr) - 1);
      y = (i >> lgx) & (R - 1);
      v = ((i >> (lgx + P.lR())) << lgx) | (i & ((1 << lgx) - 1));
    };
    float buf[PER][C];
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int r = threadIdx.x + k * kMThreads;
      if (r < nrows) {
        int c, v, y;
        row_of(r, c, v, y);
        load_row<C>(tsrc + pass_src(pass, c) * 4096 + (P.by0(v) * 8 + y) * 64 + P.bx0(v) * 8,
                    buf[k]);
      } else {
#pragma unroll
        for (int q = 0; q < C; q++) buf[k][q] = 0.0f;
      }
    }
    constexpr int l = ilog2c<C>();
#pragma unroll
    for (int k = 0; k < PER; k += 2) {
      const int r0 = threadIdx.x + k * kMThreads, r1 = r0 + kMThreads;
      if (r0 >= nrows) continue;
      int c0, v0, y0, c1, v1, y1;
      row_of(r0, c0, v0, y0);
      row_of(r1, c1, v1, y1);
      const bool ok0 = S.valid[v0], ok1 = k + 1 < PER && r1 < nrows && S.valid[v1];
      if (!ok0 && !ok1) continue;
      if (k + 1 < PER) {
        f2 x[C];
#pragma unroll
        for (int q = 0; q < C; q++) x[q] = f2{buf[k][q], buf[k + 1][q]};
        lee<C>(x);
        const int off0 = P.off(v0, pass_plane(pass, c0)) + y0 * kMS,
                  off1 = P.off(v1, pass_plane(pass, c1)) + y1 * kMS;
#pragma unroll
        for (int q = 0; q < C; q++) {
          const f2 o = x[q] * kLeeS[l][q];
          if (ok0) S.co[off0 + q] = o.x;
          if (ok1) S.co[off1 + q] = o.y;
        }
      } else {
        float* x = buf[k];
        lee<C>(x);
        const int off0 = P.off(v0, pass_plane(pass, c0)) + y0 * kMS;
#pragma unroll
        for (int q = 0; q < C; q++) S.co[off0 + q] = x[q] * kLeeS[l][q];
      }
    }
  }
}

// columns: R-point DCT of every column, in place.  A lane transforms the
// columns X and X + 32 (X < 32) of one band of R rows and one channel (f2
// lanes; any two columns of a band have the same length, whatever varblocks
// they belong to): the two LDS reads of a pair are one ds_read2 and the 32
// lanes of a band read 64 consecutive columns.  64-point: item = (pair, h).
template <int R, int NCH>
__device__ __forceinline__ void col_pass(const Pass& P, MergeLds& S, int pass) {
  constexpr int lR = ilog2c<R>(), nb = 64 / R, lnb = 6 - lR;
  constexpr int npairs = NCH * nb * 32;  // (channel, band, X)
  const int lGX = P.lGX(), lC = P.lC();
  auto col_of = [&](int pidx, int& off, bool& okA, bool& okB) {
    const int X = pidx & 31, band = (pidx >> 5) & (nb - 1), c = pidx >> (5 + lnb);
    off = pass_plane(pass, c) * kMPlane + band * R * kMS + X;
    okA = S.valid[(band << lGX) | (X >> lC)];
    okB = S.valid[(band << lGX) | ((X + 32) >> lC)];
  };
  // Two lanes per column pair (Lee halves, h wave-uniform: waves alternate h
  // over 64 pairs) for 64-point columns, and (round 6) for 16 / 32-point
  // columns whenever one lane per pair would leave threads idle (<= 128
  // pairs: R = 32, and the B pass at R = 16) -- each lane then runs half the
  // transform, every thread busy; a barrier separates the column reads from
  // the in-place writes.
  if constexpr (R == 64 || (R >= 16 && npairs <= kMThreads / 2)) {
    constexpr int H = R / 2;
    constexpr int n = ((npairs + 63) >> 6) << 7;
    for (int i0 = 0; i0 < n; i0 += kMThreads) {
      const int i = i0 + threadIdx.x;
      const int h = (i >> 6) & 1, p = ((i >> 7) << 6) | (i & 63);
      int off = 0;
      bool okA = false, okB = false;
      if (p < npairs) col_of(p, off, okA, okB);
      const bool act = okA || okB;
      f2 o[H];
      if (act) {
        const float* q0 = S.co + off;
        f2 t[H];
#pragma unroll
        for (int j = 0; j < H; j++)
          t[j] = dctN_first<R>(f2{q0[j * kMS], q0[j * kMS + 32]},
                               f2{q0[(R - 1 - j) * kMS], q0[(R - 1 - j) * kMS + 32]}, j, h);
        dctN_rest<R>(t, h, [&](int k, f2 u) { o[k] = u; });
      }
      __syncthreads();
      if (act) {
#pragma unroll
        for (int k = 0; k < H; k++) {
          if (okA) S.co[off + (2 * k + h) * kMS] = o[k].x;
          if (okB) S.co[off + 32 + (2 * k + h) * kMS] = o[k].y;
        }
      }
    }
  } else {
    for (int p = threadIdx.x; p < npairs; p += kMThreads) {
      int off;
      bool okA, okB;
      col_of(p, off, okA, okB);
      if (!okA && !okB) continue;
      float* col = S.co + off;
      f2 o[R];
#pragma unroll
      for (int k = 0; k < R; k++) o[k] = f2{col[k * kMS], col[k * kMS + 32]};
      lee<R>(o);
#pragma unroll
      for (int k = 0; k < R; k++) {
        const f2 u = o[k] * kLeeS[lR][k];
        if (okA) col[k * kMS] = u.x;
        if (okB) col[k * kMS + 32] = u.y;
      }
    }
  }
}

// quantization, phase 0 = Y, phase 1 = X and B; lane = (channel, chunk of
// RPC rows, varblock, column).  Chunk partial: fmaf(e, e) over its rows
// ascending.  The lane's weights, inverse Y weights and natural positions
// come in 16-byte loads of four rows each (row-quad tables, load_qtab).
// Rate bits and non-zeros are summed over the varblock's C lanes in-wave and
// added to LDS by one lane.  WRITE: coefficients to their natural-order
// slices, LLF to LDS.
template <int N>
__device__ __forceinline__ void load_f(const float* p, float* d) {
#pragma unroll
  for (int i = 0; i < N / 4; i++) {
    const float4 v = reinterpret_cast<const float4*>(p)[i];
    d[4 * i] = v.x;
    d[4 * i + 1] = v.y;
    d[4 * i + 2] = v.z;
    d[4 * i + 3] = v.w;
  }
}
// A thread's quantization tables for one channel: its NIT items' weights,
// distortion weights and (Y) inverse weights.  They are loaded before the
// barrier that precedes the channel's pass (load_qtab), so their L2 latency
// overlaps the barrier wait (-1 % measured; a build without any table loads
// ran 13 % faster, so the loads' issue, not their latency, is what costs).
template <int RPC>
struct QTab {
  static constexpr int NIT = RPC == 8 ? 2 : 1;  // items per thread: 512 or 256 / 256
  float w[NIT][RPC], sd[NIT][RPC], iw[NIT][RPC];
};
// Tables in row quads ([ky / 4][kx][ky % 4], host quant tables): one 16-byte
// load per lane and four rows, the wave's 64 lanes 1 KB contiguous.
__device__ __forceinline__ int qtab_index(const Pass& P, int ky, int x) {
  return P.soff + ((ky >> 2) * P.C() + x) * 4;
}
template <int RPC, bool WRITE, int CH>
__device__ __forceinline__ void load_qtab(const MergeArgs& a, const Pass& P, QTab<RPC>& T) {
  constexpr int STOT = kShapeOff[kNumShapes];
#pragma unroll
  for (int it = 0; it < QTab<RPC>::NIT; it++) {
    const int j = threadIdx.x + it * kMThreads;
    const int ch = j >> (P.lNV() + P.lC()), x = j & (P.C() - 1);
#pragma unroll
    for (int kk = 0; kk < RPC; kk += 4) {
      const int ti = qtab_index(P, ch * RPC + kk, x);
      load_f<4>(a.wk + (size_t)CH * STOT + ti, &T.w[it][kk]);
      if (!WRITE) load_f<4>(a.sdk + (size_t)CH * STOT + ti, &T.sd[it][kk]);
      if (CH == 1) load_f<4>(a.iwy + ti, &T.iw[it][kk]);
    }
  }
}
// All-reduce over an aligned group of C lanes (C = 8 .. 64, the group fully
// active) as the XOR butterfly v += v(lane ^ m), m = 1, 2, 4, ...: every
// step's partner value comes from DPP / ds_swizzle / readlane instead of a
// ds_bpermute chain (round 6).  Exactness: each step adds the partner's
// value, which is what lane ^ m holds -- xor 1 / 2 / 4 are exact lane
// permutations (quad_perm, quad_perm + row_half_mirror), xor 8 is
// row_half_mirror + row_mirror ((i ^ 7) ^ 15 = i ^ 8), xor 16 a ds_swizzle
// xor mask; for xor 32 the two 32-lane halves are uniform by then, so the
// partner is the other half's lane 0 / 32, and a + b = b + a.
template <int M>
__device__ __forceinline__ uint32_t grp_xor(uint32_t v) {
  if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  if constexpr (M == 4) {
    const int t = __builtin_amdgcn_mov_dpp((int)v, 0x1B, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_mov_dpp(t, 0x141, 0xF, 0xF, false);
  }
  if constexpr (M == 8) {
    const int t = __builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_mov_dpp(t, 0x140, 0xF, 0xF, false);
  }
  if constexpr (M == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
  if constexpr (M == 32) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
    return (threadIdx.x & 32) ? lo : hi;
  }
}
template <int M>
__device__ __forceinline__ void grp_step(float& cp, int& packed) {
  cp += __uint_as_float(grp_xor<M>(__float_as_uint(cp)));
  packed += (int)grp_xor<M>((uint32_t)packed);
}
__device__ __forceinline__ void group_all_reduce(float& cp, int& packed, int C) {
  grp_step<1>(cp, packed);
  grp_step<2>(cp, packed);
  grp_step<4>(cp, packed);
  if (C > 8) grp_step<8>(cp, packed);
  if (C > 16) grp_step<16>(cp, packed);
  if (C > 32) grp_step<32>(cp, packed);
}

template <int RPC, bool WRITE, int CH>
__device__ __forceinline__ void quant_pass(const MergeArgs& a, const Pass& P, MergeLds& S, const QTab<RPC>& T) {
  constexpr int cidx = CH == 1 ? 0 : (CH == 0 ? 1 : 2);  // 0 Y, 1 X, 2 B
  const int C = P.C(), NV = P.NV();
  // chroma from luma of the tile (front kernel): X - kx Yd, B - kb Yd
  float kc = 0.0f;
  if (CH != 1) {
    const float f = (float)a.cmap[(CH == 0 ? 0u : a.ntiles_all) + (uint32_t)P.tile];
    kc = CH == 0 ? f * (1.0f / 84.0f) : 1.0f + f * (1.0f / 84.0f);
  }
#pragma unroll
  for (int it = 0; it < QTab<RPC>::NIT; it++) {
    const int j = threadIdx.x + it * kMThreads;
    const int ch = j >> (P.lNV() + P.lC()), v = (j >> P.lC()) & (NV - 1), x = j & (C - 1);
    if (!S.valid[v]) continue;  // the varblock's C lanes leave together
    const int bx0 = P.bx0(v), by0 = P.by0(v);
    const float scale = (float)a.G * (float)S.vraw[v] / 65536.0f;
    float* cplane = S.co + P.off(v, chan_plane(CH)) + x;
    const float* yd = S.co + P.off(v, 0) + x;
    const float* w = T.w[it];
    const float* sd = T.sd[it];
    float iw[RPC];
    if (CH == 1) {
      const float inv_scale = 1.0f / scale;
#pragma unroll
      for (int kk = 0; kk < RPC; kk++) iw[kk] = T.iw[it][kk] * inv_scale;
    }
    uint16_t nat[RPC];
    if (WRITE) {
#pragma unroll
      for (int kk = 0; kk < RPC; kk += 4) {
        const uint2 u = *reinterpret_cast<const uint2*>(a.nat + qtab_index(P, ch * RPC + kk, x));
        nat[kk] = (uint16_t)u.x;
        nat[kk + 1] = (uint16_t)(u.x >> 16);
        nat[kk + 2] = (uint16_t)u.y;
        nat[kk + 3] = (uint16_t)(u.y >> 16);
      }
    }
    // the LLF (first cy rows x cx columns) only occurs in chunk 0
    const bool llf_col = ch == 0 && x < P.cx();
    float cp = 0.0f;
    // exponent sums of the rows below 8 and from 8 on: non-zeros from each
    // (nz = sum / 127, exact for eight values: jxg_front.hip nz_of_esum)
    uint32_t eb8[2] = {0u, 0u};
    // rows in pairs: the float multiplies / adds of the two rows are one
    // packed op each (f2, no contraction: each half is the scalar op order);
    // the distortion chain stays in row order
#pragma unroll
    for (int kk = 0; kk < RPC; kk += 2) {
      const int ky = ch * RPC + kk;
      const f2 coef = f2{cplane[ky * kMS], cplane[(ky + 1) * kMS]};
      if (WRITE && llf_col) {
        if (kk < P.cy()) llf_at(S, CH, (by0 + ky) * 8 + bx0 + x) = coef.x;
        if (kk + 1 < P.cy()) llf_at(S, CH, (by0 + ky + 1) * 8 + bx0 + x) = coef.y;
      }
      f2 rv = coef;
      if (CH != 1) rv = rv - f2{kc, kc} * f2{yd[ky * kMS], yd[(ky + 1) * kMS]};
      // LLF positions carry weight 0 (host tables): vq = +-0 quantizes to 0
      // and contributes nothing
      const f2 vq = rv * (f2{w[kk], w[kk + 1]} * f2{scale, scale});
      float sqs[2], qfs[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const float vqh = h ? vq.y : vq.x;
        const float av = fabsf(vqh);
        // qa = (int)(min(av, 32767) + 0.5) as an integer-valued float (the
        // truncation of a positive value is its floor): no conversions
        // needed for the error and the rate
        qfs[h] = av < 0.58f ? 0.0f : floorf(fminf(av, 32767.0f) + 0.5f);
        sqs[h] = __builtin_copysignf(qfs[h], vqh);
      }
      if (CH == 1) {
        // AdjustQuantBias from the table below 256; one wave vote per row pair
        // for the (rare) larger magnitudes
        float adj[2];
#pragma unroll
        for (int h = 0; h < 2; h++) adj[h] = S.btab[min((int)qfs[h], 255)];
        if (__builtin_expect(__any(fmaxf(qfs[0], qfs[1]) >= 256.0f), 0)) {
#pragma unroll
          for (int h = 0; h < 2; h++)
            if (qfs[h] >= 256.0f) adj[h] = qfs[h] - 0.145f / qfs[h];
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
          // (vq = -0: a -0 that no result sees; jxg_front.hip)
          const float a1 = __builtin_copysignf(adj[h], h ? vq.y : vq.x);
          cplane[(ky + h) * kMS] = a1 * iw[kk + h];  // LLF: 0 (its value lives in llf_at)
        }
      }
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const float qf = qfs[h];
        // 2 + 2 bitlen(qa) per non-zero = 2 E - 250, E = biased exponent of
        // qf (qf = 0 has E = 0 and is not counted in nzc)
        eb8[kk >= 8] += __float_as_uint(qf) >> 23;
        if (WRITE) {
          const int qq = (int)sqs[h];  // (vq < 0 ? -qa : qa)
          const int p = nat[kk + h];
          const int sl = p >> 6;
          const int lbx = bx0 + (sl & (P.cx() - 1)), lby = by0 + (sl >> P.lcx);
          const size_t gb = (size_t)(P.ty * 8 + lby) * a.bxs + P.tx * 8 + lbx;
          a.ac[(gb * 3 + CH) * 64 + (p & 63)] = (int16_t)qq;
        }
      }
      // error in steps times the distortion weight (oracle jxo_dist_weight);
      // the write pass needs no estimate
      // (the signed error: (vq - sq) sd = +-(|vq| - qf) sd exactly, the same
      // square; jxg_front.hip signed_err)
      if (!WRITE) {
        const f2 e = (vq - f2{sqs[0], sqs[1]}) * f2{sd[kk], sd[kk + 1]};
        cp = fmaf(e.x, e.x, cp);
        cp = fmaf(e.y, e.y, cp);
      }
    }
    const int nzc = (int)(eb8[0] / 127u) + (int)(eb8[1] / 127u);
    const int bits = 2 * (int)(eb8[0] + eb8[1]) - 250 * nzc;
    // the chunk's column partials, tree-summed over the varblock's C lanes
    // (an aligned group inside one wave); bits | non-zeros << 20 likewise
    int packed = bits | nzc << 20;
    group_all_reduce(cp, packed, C);
    if (x == 0) {
      S.qsum[cidx][ch][v] = cp;
      if (packed & 0xFFFFF) atomicAdd(&S.vbits[v], packed & 0xFFFFF);
      if (packed >> 20) atomicAdd(&S.vnz[v][CH], packed >> 20);
    }
  }
}

// transform + quantize every valid varblock of the pass; leaves per-varblock
// bits / non-zeros and the chunk sums in LDS
template <bool WRITE>
__device__ __forceinline__ void transform_quant(const MergeArgs& a, const Pass& P, MergeLds& S) {
#ifdef JXG_MERGE_PROFILE
  unsigned long long mprof_t0 = 0;
#endif
  MPROF_MARK(0);
  auto transform = [&](auto nch_tag, int pass) {
    constexpr int NCH = decltype(nch_tag)::value;
    switch (P.lcx) {
      case 0: row_pass<8, NCH>(a, P, S, pass); break;
      case 1: row_pass<16, NCH>(a, P, S, pass); break;
      case 2: row_pass<32, NCH>(a, P, S, pass); break;
      default: row_pass<64, NCH>(a, P, S, pass); break;
    }
    __syncthreads();
    switch (P.lcy) {
      case 0: col_pass<8, NCH>(P, S, pass); break;
      case 1: col_pass<16, NCH>(P, S, pass); break;
      case 2: col_pass<32, NCH>(P, S, pass); break;
      default: col_pass<64, NCH>(P, S, pass); break;
    }
  };
  transform(std::integral_constant<int, 2>(), 0);  // Y -> plane 0, X -> plane 1
  MPROF_MARK(1);
  // Y first: its dequantized values replace its coefficients (X / B
  // residuals); then X; then B is transformed into X's plane.  Every pass's
  // tables are in flight across the barrier before it.  A lane's X / B items
  // read the Y values its own Y item wrote (same item map).
  auto quant_yx = [&](auto rpc_tag) {
    constexpr int RPC = decltype(rpc_tag)::value;
    {
      QTab<RPC> ty;
      load_qtab<RPC, WRITE, 1>(a, P, ty);
      __syncthreads();
      MPROF_MARK(2);
      quant_pass<RPC, WRITE, 1>(a, P, S, ty);
    }
    QTab<RPC> tx;
    load_qtab<RPC, WRITE, 0>(a, P, tx);
    quant_pass<RPC, WRITE, 0>(a, P, S, tx);
  };
  auto quant_b = [&](auto rpc_tag) {
    constexpr int RPC = decltype(rpc_tag)::value;
    QTab<RPC> tb;
    load_qtab<RPC, WRITE, 2>(a, P, tb);
    __syncthreads();
    quant_pass<RPC, WRITE, 2>(a, P, S, tb);
  };
  if (P.lcy == 0) quant_yx(std::integral_constant<int, 8>());
  else quant_yx(std::integral_constant<int, 16>());
  __syncthreads();  // plane 1 (X) fully read
  MPROF_MARK(3);
  transform(std::integral_constant<int, 1>(), 1);  // B -> plane 1
  if (P.lcy == 0) quant_b(std::integral_constant<int, 8>());
  else quant_b(std::integral_constant<int, 16>());
  __syncthreads();
  MPROF_MARK(4);
}

// distortion of varblock v: chunk sums in order per channel, (Y + X) + B
__device__ __forceinline__ float varblock_dist(const Pass& P, const MergeLds& S, int v) {
  const int nch = P.lcy == 0 ? 1 : P.R() >> 4;
  float pc[3];
#pragma unroll
  for (int ci = 0; ci < 3; ci++) {
    float t = S.qsum[ci][0][v];
    for (int ch = 1; ch < nch; ch++) t = t + S.qsum[ci][ch][v];
    pc[ci] = t;
  }
  return (pc[0] + pc[1]) + pc[2];
}

// per-varblock setup, before the tile-load barrier: validity (eval: the
// level region lies inside the frame's blocks; write: the resolved map holds
// the shape there), hook-F indices, sums reset; the blocks' quant field goes
// to LDS (the varblock maxima are taken after the barrier: vraw_pass)
template <bool WRITE>
__device__ __forceinline__ void setup_varblocks(const MergeArgs& a, const Pass& P, MergeLds& S,
                                                int nbx, int nby) {
  const int t = threadIdx.x;
  if (t < 64) {
    const int lbx = t & 7, lby = t >> 3;
    const bool in = lbx < nbx && lby < nby;
    const size_t gb = (size_t)(P.ty * 8 + lby) * a.bxs + P.tx * 8 + lbx;
    S.braw[t] = in ? a.qf[gb] : 0;
  }
  if (t < 32) {
    const int v = t;
    bool ok = false;
    if (v < P.NV()) {
      const int bx0 = P.bx0(v), by0 = P.by0(v);
      const size_t gb0 = (size_t)(P.ty * 8 + by0) * a.bxs + P.tx * 8 + bx0;
      if (WRITE) {
        ok = bx0 < nbx && by0 < nby && a.acs[gb0] == (uint8_t)P.type;
      } else {
        ok = (((bx0 >> P.ls) + 1) << P.ls) <= nbx && (((by0 >> P.ls) + 1) << P.ls) <= nby;
        if (ok && (a.proposals & 2u)) {
          S.vr3[v][0] = a.homog[gb0 * 3 + 0];
          S.vr3[v][1] = a.homog[gb0 * 3 + 1];
          S.vr3[v][2] = a.homog[gb0 * 3 + 2];
        }
      }
    }
    S.valid[v] = ok;
    S.vraw[v] = 0;  // (vraw_pass: atomic max over the covered blocks)
    S.vbits[v] = 0;
    S.vnz[v][0] = S.vnz[v][1] = S.vnz[v][2] = 0;
  }
  // AdjustQuantBias of q: 0 -> 0, 1 -> 1 - 0.0700..., else q - 0.145 / q (the
  // per-coefficient expression, tabulated)
  for (int i = t; i < 256; i += kMThreads)
    S.btab[i] = i == 0 ? 0.0f : (i == 1 ? 1.0f - 0.07005449891748593f : (float)i - 0.145f / (float)i);
}
// varblock quant field = max raw over its covered blocks (after a barrier):
// one thread per block, an LDS atomic max into its varblock (round 6: one
// thread per varblock walked up to 64 blocks in a row of dependent LDS reads
// while its wave's row pass waited; max is order-free, so the result is the
// same); visible to the quantization after the row pass's barrier
__device__ __forceinline__ void vraw_pass(const MergeArgs& a, const Pass& P, MergeLds& S) {
  (void)a;
  const int b = threadIdx.x;
  if (b < 64) {
    const int lbx = b & 7, lby = b >> 3;
    const int v = ((lby >> P.lcy) << P.lGX()) | (lbx >> P.lcx);
    if (v < P.NV() && S.valid[v]) atomicMax(&S.vraw[v], (int)S.braw[b] + 1);
  }
}

__device__ __forceinline__ int max_level(const MergeArgs& a) {
  return a.max_s >= 8 ? 3 : (a.max_s >= 4 ? 2 : 1);
}

__global__ __launch_bounds__(kMThreads) __attribute__((amdgpu_waves_per_eu(JXG_MERGE_WPE)))
void merge_eval_kernel(Batch<MergeArgs> bt_) {
  const MergeArgs& a = bt_.a[blockIdx.z];  // the batch's frame
  __shared__ __attribute__((aligned(16))) MergeLds S;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.work[0] = 0;  // merge_resolve's work-list count
  int tile, si;
  if (!decode_wg(a, tile, si)) return;
  const Pass P = make_pass(a, tile, si);
  if (P.ls > max_level(a)) return;  // level not searched at this effort
  const int nbx = min(8, (int)a.bxs - P.tx * 8), nby = min(8, (int)a.bys - P.ty * 8);
  if ((1 << P.ls) > nbx || (1 << P.ls) > nby) return;  // no region of this level fits
#ifdef JXG_MERGE_PROFILE
  const unsigned long long t_setup = __builtin_readcyclecounter();
#endif
  setup_varblocks<false>(a, P, S, nbx, nby);
  __syncthreads();
  vraw_pass(a, P, S);
#ifdef JXG_MERGE_PROFILE
  if (threadIdx.x == 0) atomicAdd(&g_mprof[P.si][5], __builtin_readcyclecounter() - t_setup);
#endif
  transform_quant<false>(a, P, S);
  const int v = threadIdx.x;
  if (v < P.NV() && S.valid[v]) {
    const float dist = varblock_dist(P, S, v);
    const int tb = bitlen_u((uint32_t)S.vnz[v][0]) + bitlen_u((uint32_t)S.vnz[v][1]) +
                   bitlen_u((uint32_t)S.vnz[v][2]);
    float e = ((float)(S.vbits[v] + tb) + 8.0f * dist) * P.tmul;
    if (a.proposals & 2u) e = hook_f(e, S.vr3[v][0], S.vr3[v][1], S.vr3[v][2]);
    a.cost[((size_t)tile * kNumShapes + si) * 32 + v] = e;
  }
}

// one wave per tile (16 tiles per workgroup): levels in order, one lane per
// region; then the tile's chosen shapes go to the merge_write work list (one
// global atomic per workgroup)
constexpr int kResolveWaves = 16;
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__global__ __launch_bounds__(64 * kResolveWaves) void merge_resolve_kernel(Batch<MergeArgs> bt_) {
  const MergeArgs& a = bt_.a[blockIdx.z];
  __shared__ float sEntW[kResolveWaves][64];
  __shared__ uint8_t sAcsW[kResolveWaves][64];
  __shared__ uint32_t sCnt[kResolveWaves];
  __shared__ uint32_t sBase;
  const int wv = threadIdx.x >> 6, t = threadIdx.x & 63;
  float* sEnt = sEntW[wv];
  uint8_t* sAcs = sAcsW[wv];
  const int idx = blockIdx.x * kResolveWaves + wv;
  uint32_t has = 0;
  int tile = 0;
  if (idx < (int)a.ntiles) {
    tile = a.tile_list ? (int)a.tile_list[idx] : idx;
    const int tx = tile % (int)a.tiles_x, ty = tile / (int)a.tiles_x;
    const int nbx = min(8, (int)a.bxs - tx * 8), nby = min(8, (int)a.bys - ty * 8);
    const int lbx = t & 7, lby = t >> 3;
    const bool in = lbx < nbx && lby < nby;
    const size_t gb = (size_t)(ty * 8 + lby) * a.bxs + tx * 8 + lbx;
    sEnt[t] = in ? a.ent[gb] : 0.0f;
    sAcs[t] = in ? a.acs[gb] : 0;
    wave_sync_lds();
    const float* cost = a.cost + (size_t)tile * kNumShapes * 32;
    for (int s = 2; s <= a.max_s && s <= nbx && s <= nby; s *= 2) {
      const int nr = 8 / s;
      const int full = s == 2 ? 2 : (s == 4 ? 5 : 8);
      const int tall = s == 2 ? 0 : (s == 4 ? 3 : 6);
      if (t < nr * nr) {
        const int rx = t % nr, ry = t / nr;
        if ((rx + 1) * s <= nbx && (ry + 1) * s <= nby) {
          float cur = 0.0f;
          for (int iy = 0; iy < s; iy++)
            for (int ix = 0; ix < s; ix++) cur += sEnt[(ry * s + iy) * 8 + rx * s + ix];
          // varblock grid indices: full (8/s per row), tall (16/s), wide (8/s)
          const int vf = ry * nr + rx, vl = ry * (16 / s) + 2 * rx, vt = (2 * ry) * nr + rx;
          const float e0 = cost[full * 32 + vf];
          const float el = cost[tall * 32 + vl], er = cost[tall * 32 + vl + 1];
          const float etop = cost[(tall + 1) * 32 + vt], ebot = cost[(tall + 1) * 32 + vt + nr];
          const float et = el + er, ew = etop + ebot;
          float best = cur;
          int choice = 0;
          if (!(e0 >= best)) {
            best = e0;
            choice = 1;
          }
          if (!(et >= best)) {
            best = et;
            choice = 2;
          }
          if (!(ew >= best)) {
            best = ew;
            choice = 3;
          }
          for (int j = 0; choice && j < (choice == 1 ? 1 : 2); j++) {
            int sh, bx, by;
            float e;
            if (choice == 1) {
              sh = full, bx = rx * s, by = ry * s, e = e0;
            } else if (choice == 2) {
              sh = tall, bx = rx * s + j * (s / 2), by = ry * s, e = j ? er : el;
            } else {
              sh = tall + 1, bx = rx * s, by = ry * s + j * (s / 2), e = j ? ebot : etop;
            }
            const int cy = 1 << kShapes[sh].lcy, cx = 1 << kShapes[sh].lcx;
            for (int iy = 0; iy < cy; iy++)
              for (int ix = 0; ix < cx; ix++) {
                const int b = (by + iy) * 8 + bx + ix;
                sAcs[b] = (uint8_t)(kShapes[sh].type | ((iy | ix) ? 0x80 : 0));
                sEnt[b] = (iy | ix) ? 0.0f : e;
              }
          }
        }
      }
      wave_sync_lds();
    }
    if (in) {
      a.acs[gb] = sAcs[t];
      a.ent[gb] = sEnt[t];  // the decisions' estimates: the 128 / 256 px levels' "current"
    }
    // the shapes chosen somewhere in this tile
    if (in && !(sAcs[t] & 0x80)) {
#pragma unroll
      for (int si = 0; si < kNumShapes; si++) has |= sAcs[t] == kShapes[si].type ? 1u << si : 0u;
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) has |= __shfl_xor(has, m, 64);
  }
  if (t == 0) sCnt[wv] = (uint32_t)__popc(has);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int w = 0; w < kResolveWaves; w++) tot += sCnt[w];
    sBase = tot ? atomicAdd(a.work, tot) : 0u;
  }
  __syncthreads();
  uint32_t base = sBase;
  for (int w = 0; w < wv; w++) base += sCnt[w];
  if (t < kNumShapes && ((has >> t) & 1u))
    a.work[1 + base + __popc(has & ((1u << t) - 1u))] = (uint32_t)tile << 4 | (uint32_t)t;
}

// one (tile, shape) entry of the work list; returns after its last LDS use
__device__ __forceinline__ void write_entry(const MergeArgs& a, int tile, int si, MergeLds& S) {
  const Pass P = make_pass(a, tile, si);
  const int nbx = min(8, (int)a.bxs - P.tx * 8), nby = min(8, (int)a.bys - P.ty * 8);
  setup_varblocks<true>(a, P, S, nbx, nby);
  __syncthreads();
  vraw_pass(a, P, S);
  transform_quant<true>(a, P, S);
  // per covered block: non-zero counts, quant field, LLF-derived DC
  const int cb = P.cy() * P.cx(), lcb = P.lcy + P.lcx;
  const size_t nb = (size_t)a.bxs * a.bys;
  const int ly = P.lcy, lx = P.lcx;
  for (int i = threadIdx.x; i < P.NV() * cb; i += kMThreads) {
    const int v = i >> lcb, k = i & (cb - 1);
    if (!S.valid[v]) continue;
    const int iy = k >> P.lcx, ix = k & (P.cx() - 1);
    const int bx0 = P.bx0(v), by0 = P.by0(v);
    const size_t gb = (size_t)(P.ty * 8 + by0 + iy) * a.bxs + P.tx * 8 + bx0 + ix;
    for (int c = 0; c < 3; c++) {
      const int n = S.vnz[v][c];
      a.nz[c * nb + gb] = (uint16_t)(k == 0 ? n : (n + cb - 1) >> lcb);
    }
    // the LLF -> DC tables of this block in registers (static indices, loop
    // bounds cx, cy <= 8 as predicates): no dependent constant loads
    float px[8], py[8], ibx[8], iby[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      px[k] = c_llf_p[lx * 8 + k];
      py[k] = c_llf_p[ly * 8 + k];
      ibx[k] = c_llf_ib[lx * 64 + ix * 8 + k];
      iby[k] = c_llf_ib[ly * 64 + iy * 8 + k];
    }
    const int cx = P.cx(), cy = P.cy();
    float dc[3];
#pragma unroll 1
    for (int c = 0; c < 3; c++) {
      float acc = 0.0f;
#pragma unroll
      for (int ky = 0; ky < 8; ky++) {
        if (ky < cy) {
          float u = 0.0f;
#pragma unroll
          for (int kx = 0; kx < 8; kx++) {
            if (kx < cx) {
              const float tt = (llf_at(S, c, (by0 + ky) * 8 + bx0 + kx) * py[ky]) * px[kx];
              u = fmaf(tt, ibx[kx], u);
            }
          }
          acc = fmaf(u, iby[ky], acc);
        }
      }
      dc[c] = acc;
    }
    int32_t q[3];
    quant_dc3(dc, a.dc_mul, a.dc_step, q);
    a.dc[gb] = q[0];
    a.dc[nb + gb] = q[1];
    a.dc[2 * nb + gb] = q[2];
    a.qf[gb] = (uint8_t)(S.vraw[v] - 1);
  }
}

// persistent workgroups over the (tile, shape) entries the resolve kernel
// listed: only (tile, shape) pairs holding a chosen varblock cost anything
__global__ __launch_bounds__(kMThreads) __attribute__((amdgpu_waves_per_eu(JXG_MERGE_WRITE_WPE)))
void merge_write_kernel(Batch<MergeArgs> bt_) {
  const MergeArgs& a = bt_.a[blockIdx.z];
  __shared__ __attribute__((aligned(16))) MergeLds S;
  const uint32_t n = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)a.work);
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
    const uint32_t e = a.work[1 + w];
    write_entry(a, (int)(e >> 4), (int)(e & 15u), S);
    __syncthreads();  // LDS reuse by the next entry
  }
}

// ---------------------------------------------------------------------------
// varblock lists of the LF groups (AC metadata channel of size count x 2):
// block indices of the varblocks' first blocks in LF-group raster order
// ---------------------------------------------------------------------------
// Varblock list of one LF group: the frame-raster block index of every
// varblock's first block, in raster order inside the LF group.  Thread t
// holds the first-block flags of blocks t, t + 1024, ... (all 64 loads in
// flight at once); per-(chunk, wave) counts -> one workgroup scan -> stores.
__global__ __launch_bounds__(1024) void vb_list_kernel(Batch<VbArgs> bt_) {
  const VbArgs& a = bt_.a[blockIdx.z];
  __shared__ uint32_t sCnt[64 * 16];
  __shared__ uint32_t sWave[16];
  const uint32_t lg = blockIdx.x;
  if (a.lf_mine && !a.lf_mine[lg]) return;  // LF group of another shard
  const uint32_t bx0 = (lg % a.lfxs) * 256, by0 = (lg / a.lfxs) * 256;
  const uint32_t bw = min(256u, a.bxs - bx0), bh = min(256u, a.bys - by0);
  const uint32_t n = bw * bh;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  // (row, column) of element i = k * 1024 + threadIdx.x in the group, stepped
  // by (1024 / bw, 1024 % bw) with a carry: no integer division per element
  const uint32_t dq = 1024u / bw, dr = 1024u % bw;
  const uint32_t y0 = threadIdx.x / bw, x0 = threadIdx.x % bw;
  auto step = [&](uint32_t& y, uint32_t& x) {
    x += dr;
    y += dq;
    if (x >= bw) {
      x -= bw;
      y++;
    }
  };
  uint64_t fl = 0;  // bit k: block k * 1024 + threadIdx.x starts a varblock
  {
    uint32_t y = y0, x = x0;
#pragma unroll 16
    for (int k = 0; k < 64; k++) {
      const uint32_t i = (uint32_t)k * 1024 + threadIdx.x;
      if (i < n && !(a.acs[(size_t)(by0 + y) * a.bxs + bx0 + x] & 0x80)) fl |= 1ull << k;
      step(y, x);
    }
  }
  for (int k = 0; k < 64; k++) {
    const uint64_t bal = __ballot((fl >> k) & 1);
    if (lane == 0) sCnt[k * 16 + wv] = (uint32_t)__popcll(bal);
  }
  __syncthreads();
  // exclusive scan of the 1024 (chunk, wave) counts in (chunk, wave) order
  const uint32_t v = sCnt[threadIdx.x];
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  if (lane == 63) sWave[wv] = incl;
  __syncthreads();
  uint32_t before = 0, total = 0;
  for (int w = 0; w < 16; w++) {
    before += w < wv ? sWave[w] : 0u;
    total += sWave[w];
  }
  sCnt[threadIdx.x] = before + incl - v;
  __syncthreads();
  uint32_t y = y0, x = x0;
  for (int k = 0; k < 64; k++) {
    const bool f = (fl >> k) & 1;
    const uint64_t bal = __ballot(f);
    if (f)
      a.vb[(size_t)lg * 65536 + sCnt[k * 16 + wv] + (uint32_t)__popcll(bal & lt)] =
          (uint32_t)((size_t)(by0 + y) * a.bxs + bx0 + x);
    step(y, x);
  }
  if (threadIdx.x == 0) a.count[lg] = total;
}

#ifdef JXG_MERGE_PROFILE
void dump_merge_profile() {
  unsigned long long h[16][8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_mprof), sizeof(h)) != hipSuccess) return;
  std::fprintf(stderr, "merge_eval cycles (thread 0 sums, Mcycles): shape setup rows+cols(Y,X) "
                       "qtab quantY+X B(rows,cols,quant)\n");
  for (int si = 0; si < kNumShapes; si++)
    std::fprintf(stderr, "  %dx%d %8.1f %8.1f %8.1f %8.1f %8.1f\n", 8 << kShapes[si].lcy,
                 8 << kShapes[si].lcx, h[si][5] / 1e6, h[si][1] / 1e6, h[si][2] / 1e6,
                 h[si][3] / 1e6, h[si][4] / 1e6);
}
#else
void dump_merge_profile() {}
#endif

hipError_t set_merge_constants(const float* llf_p, const float* llf_ib, hipStream_t s) {
  hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_llf_p), llf_p, sizeof(float) * 4 * 8, 0,
                                        hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_llf_ib), llf_ib, sizeof(float) * 4 * 64, 0,
                               hipMemcpyHostToDevice, s);
  const hipError_t e2 = hipStreamSynchronize(s);
  return e != hipSuccess ? e : e2;
}
// k frames of one size (same tile count): one launch of each kernel
hipError_t launch_merge(const MergeArgs* a, uint32_t k, hipStream_t s) {
  if (!k || !a[0].ntiles) return hipSuccess;
  const Batch<MergeArgs> b = make_batch(a, k);
  const uint32_t ntiles = a[0].ntiles;
  constexpr uint32_t T = JXG_MERGE_CHUNK;
  const uint32_t nwg = (((ntiles + 7) / 8 + T - 1) / T) * T * 8 * kNumShapes;
  hipLaunchKernelGGL(merge_eval_kernel, dim3(nwg, 1, k), dim3(kMThreads), 0, s, b);
  hipLaunchKernelGGL(merge_resolve_kernel, dim3((ntiles + kResolveWaves - 1) / kResolveWaves, 1, k),
                     dim3(64 * kResolveWaves), 0, s, b);
  // the persistent write workgroups: nwrite over the whole launch
  const uint32_t nw = max(1u, min(a[0].nwrite / k, ntiles * (uint32_t)kNumShapes));
  hipLaunchKernelGGL(merge_write_kernel, dim3(nw, 1, k), dim3(kMThreads), 0, s, b);
  return hipGetLastError();
}
void launch_vb_list(const VbArgs* a, uint32_t k, uint32_t nlf, hipStream_t s) {
  if (k) hipLaunchKernelGGL(vb_list_kernel, dim3(nlf, 1, k), dim3(1024), 0, s, make_batch(a, k));
}

}  // namespace jxg
