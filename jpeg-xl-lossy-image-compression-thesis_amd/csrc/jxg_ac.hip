// jxg_ac.hip -- pass-group AC token statistics and bit emission on gfx950.
//
// One 1024-thread workgroup per 256x256-pixel pass group: thread = 8x8 block
// = one 64-coefficient slice of a varblock (an 8x8-class block is a varblock
// of one slice; a merged varblock covering cb blocks keeps slice i of its
// natural-order coefficients in covered block i, raster order).  A slice's
// walk state at its first coefficient -- non-zeros left and the
// previous-coefficient flag -- follows from the per-slice non-zero counts of
// the earlier slices (LDS), so every slice of a 64x64 varblock is independent.
// The token walk is wave-parallel: a wave takes the tasks (slice, channel) of
// its 64 threads one at a time, lane = coefficient; ballot + popcount give
// each coefficient its non-zeros-left context, so a task costs one pass
// whatever its token count and its records are stored contiguously.
//   ac_hist : non-zero counts -> predicted-nz + zero-density contexts ->
//             clustered histograms (LDS, one global atomic per non-empty bin),
//             exact per-group token counts, per-group bit upper bound; then a
//             workgroup scan over varblocks (stream order: varblocks by first
//             block raster, channels Y, X, B, slices) and the wave-parallel
//             walk that writes every token as a 32-bit record (cluster | token << 8 |
//             raw-bit count << 14 | raw bits << 18) at its stream position.
//   ac_emit : prefix codes from the records alone (no coefficient walk):
//             a contiguous record range per wave, coalesced reads, wave scans
//             of the code lengths -> LDS bit buffer (ds_or), copied out with
//             plain 4-byte stores (global atomics only for groups larger than
//             the buffer).
//   ans_*   : the rANS coder over the same records.
// Token order / contexts are those of oracle/encode.c group_tokens, [ext]
// libjxl dec_group DecodeACVarBlock.
#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

// context -> static cluster id (padded to whole 16-byte words: ac_hist copies
// it to LDS with 16-byte loads; the pad stays 0)
constexpr int kAcCtxPad = (kAcCtx + 15) & ~15;
__constant__ __attribute__((aligned(16))) uint8_t c_cluster[kAcCtxPad];

constexpr int kAcThreads = 1024;

struct GroupGeom {
  int bx0, by0, gw, gh;
};
// pass group of launch slot i: a shard's group list, or the range g0 + i
__device__ __forceinline__ uint32_t slot_group(const uint32_t* glist, uint32_t g0, uint32_t i) {
  return glist ? glist[i] : g0 + i;
}
__device__ __forceinline__ GroupGeom group_geom(const AcArgs& a, int g) {
  GroupGeom r;
  const int gx = g % (int)a.gxs, gy = g / (int)a.gxs;
  r.bx0 = gx * 32;
  r.by0 = gy * 32;
  r.gw = min(32, (int)a.bxs - r.bx0);
  r.gh = min(32, (int)a.bys - r.by0);
  return r;
}

__device__ __forceinline__ void load_coefs(const int16_t* q, uint32_t* w) {
  const uint4* p = reinterpret_cast<const uint4*>(q);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint4 t = p[i];
    w[4 * i + 0] = t.x;
    w[4 * i + 1] = t.y;
    w[4 * i + 2] = t.z;
    w[4 * i + 3] = t.w;
  }
}
// coefficient k (zigzag) of a register-resident block; k must be static
__device__ __forceinline__ int32_t coef(const uint32_t* w, int k) {
  return (int32_t)(int16_t)(w[k >> 1] >> ((k & 1) * 16));
}

// kFreqCtx / kNnzCtx as arithmetic (lane-varying indices; no constant-table
// gathers in the walk)
__device__ __forceinline__ int freq_ctx(int k) {
  return k < 16 ? max(k - 1, 0) : (k < 32 ? 15 + ((k - 16) >> 1) : 23 + ((k - 32) >> 2));
}
__device__ __forceinline__ int nnz_ctx(int n) {
  return n < 2 ? 0 : n < 3 ? 31 : n < 5 ? 62 : n < 9 ? 93 : n < 13 ? 123 : n < 21 ? 152
       : n < 33 ? 180 : 206;
}

__device__ __forceinline__ int block_ctx_of(int c, int acs) {
  return kDefaultCtxMap[(c < 2 ? c ^ 1 : 2) * 13 + kStrategyOrder[acs]];
}

// AC tokens are < 64: |q| <= 32767 -> packed value <= 65534 -> hybrid token
// <= 63; the non-zero count (<= 4032) token is <= 47.  Device tables use 64 columns.
constexpr int kAcTok = 64;
// LDS bit buffer of ac_emit / ans_emit (groups whose exact size exceeds it
// fall back to global atomics): 96 KiB = 786432 bits = 12 bpp over a full
// 256x256 group, so only near-incompressible groups take the slow path
// (ac_emit: 96 KiB + 33 KiB of code tables, one 1024-thread workgroup per CU)
constexpr int kEmitLdsWords = 24576;

__device__ __forceinline__ int channel_of(int ci) { return ci == 0 ? 1 : (ci == 1 ? 0 : 2); }

// covered blocks of a raw strategy id: log2 and blocks across / down
__device__ __forceinline__ void varblock_dims(int type, int& lcb, int& cx, int& cy) {
  switch (type) {
    case 6: lcb = 1, cx = 1, cy = 2; break;   // 16x8
    case 7: lcb = 1, cx = 2, cy = 1; break;   // 8x16
    case 4: lcb = 2, cx = 2, cy = 2; break;   // 16x16
    case 10: lcb = 3, cx = 2, cy = 4; break;  // 32x16
    case 11: lcb = 3, cx = 4, cy = 2; break;  // 16x32
    case 5: lcb = 4, cx = 4, cy = 4; break;   // 32x32
    case 19: lcb = 5, cx = 4, cy = 8; break;  // 64x32
    case 20: lcb = 5, cx = 8, cy = 4; break;  // 32x64
    case 18: lcb = 6, cx = 8, cy = 8; break;  // 64x64
    case 22: lcb = 7, cx = 8, cy = 16; break;   // 128x64 (effort >= 8)
    case 23: lcb = 7, cx = 16, cy = 8; break;   // 64x128
    case 21: lcb = 8, cx = 16, cy = 16; break;  // 128x128
    case 25: lcb = 9, cx = 16, cy = 32; break;  // 256x128
    case 26: lcb = 9, cx = 32, cy = 16; break;  // 128x256
    case 24: lcb = 10, cx = 32, cy = 32; break; // 256x256
    default: lcb = 0, cx = 1, cy = 1; break;  // 8x8 class
  }
}

// ac_hist runs one 256-thread workgroup per BAND of a pass group: 8 block
// rows (one row of 64x64 tiles) x 32 block columns.  Varblocks up to 64x64
// are aligned to their size inside 64x64 tiles, so a band holds whole
// varblocks, and the group's token stream (varblocks by first block raster)
// is the concatenation of its four bands' streams: band j writes its records
// at [j * kBandTokStride, ...) of the group's record space and its token
// count to bandtok[g][j]; the coders read the group's stream through
// rec_index (a 4-entry prefix).  Four workgroups per group give small frames
// (1080p: 40 groups) 160 workgroups instead of 40.  At effort >= 8 varblocks
// of 128 / 256 px span bands: the kernel then runs with BR = 32 (one
// 1024-thread workgroup = one band = the whole group; bands 1-3 empty).
constexpr int kBands = 4;  // bandtok entries per group (the coders' view)
static_assert(kBands * kBandTokStride == kGroupTokStride, "band record spaces tile the group's");

// record space index of stream position k of a group whose band counts are bt[4]
// (band j holds stream positions [c_j, c_j+1), c_j = bt[0] + ... + bt[j-1];
// the bounds are cumulative, so k >= c_j holds for a prefix of the bands)
__device__ __forceinline__ uint32_t rec_index(const uint32_t* bt, uint32_t k) {
  uint32_t j = 0, lo = 0, cum = 0;
#pragma unroll
  for (int i = 0; i < kBands - 1; i++) {
    cum += bt[i];
    const bool past = k >= cum;
    lo = past ? cum : lo;
    j += past ? 1u : 0u;
  }
  return j * (uint32_t)kBandTokStride + (k - lo);
}

// One thread per block of the band: slice `sl` of the varblock whose first
// block is (obx, oby) (group-local rows; varblocks are aligned to their size).
struct SliceTask {
  bool valid;
  int bx, by, obx, oby, sl, lcb, cx, type;
  size_t gb, ogb;
};
// (BR: the band's block rows, 8 or 32; thread = block of the band)
__device__ __forceinline__ SliceTask slice_task(const AcArgs& a, const GroupGeom& G, int y0) {
  SliceTask t;
  const int b = threadIdx.x;
  t.bx = b & 31;
  t.by = y0 + (b >> 5);
  t.valid = t.bx < G.gw && t.by < G.gh;
  if (!t.valid) t.bx = t.by = 0;
  t.gb = (size_t)(G.by0 + t.by) * a.bxs + G.bx0 + t.bx;
  t.type = t.valid ? (a.acs[t.gb] & 0x7F) : 0;
  int cy;
  varblock_dims(t.type, t.lcb, t.cx, cy);
  t.obx = t.bx & ~(t.cx - 1);
  t.oby = t.by & ~(cy - 1);
  t.sl = (t.by - t.oby) * t.cx + (t.bx - t.obx);
  t.ogb = (size_t)(G.by0 + t.oby) * a.bxs + G.bx0 + t.obx;
  return t;
}
// band-local index of slice j of t's varblock
__device__ __forceinline__ int block_of_slice(const SliceTask& t, int j, int y0) {
  return (t.oby - y0 + j / t.cx) * 32 + t.obx + j % t.cx;
}

template <int BR>
struct AcLds {
  uint8_t nz[3][(BR + 1) * 32];  // predicted-nz image, band rows and the row above
  uint8_t snz[3][BR * 32];   // non-zeros of each slice (positions >= cb)
  uint8_t last[3][BR * 32];  // last coefficient of the slice != 0
  int8_t lastk[3][BR * 32];  // highest slice-local index >= cb - 64 sl holding a non-zero, or -1
};
// predicted non-zeros of group-local block (bx, by) from the band's nz image
// (row 0 = the row above the band); neighbours inside the group only
__device__ __forceinline__ int predict_nz(const uint8_t* nzc, int bx, int by, int y0) {
  const int r = by - y0 + 1;
  if (bx == 0) return by == 0 ? 32 : nzc[(r - 1) * 32 + bx];
  if (by == 0) return nzc[r * 32 + bx - 1];
  return (nzc[(r - 1) * 32 + bx] + nzc[r * 32 + bx - 1] + 1) / 2;
}

// tokens of task (t, c) without walking it: the walk runs from the slice's
// first position >= cb up to the varblock's last non-zero K (1 + K for an
// 8x8-class block), plus the non-zero count token on slice 0
template <int BR>
__device__ __forceinline__ uint32_t task_token_count(const AcArgs& a, const SliceTask& t,
                                                     const AcLds<BR>& L, int c, int y0) {
  if (t.lcb == 0) {
    uint32_t w[32];
    load_coefs(a.ac + (t.gb * 3 + c) * 64, w);
    int last = 0;
#pragma unroll
    for (int kk = 1; kk < 64; kk++) last = coef(w, kk) != 0 ? kk : last;
    return 1u + (uint32_t)last;
  }
  const int cb = 1 << t.lcb;
  int K = -1;
  for (int j = 0; j < cb; j++) {
    const int lk = L.lastk[c][block_of_slice(t, j, y0)];
    K = lk >= 0 ? j * 64 + lk : K;
  }
  const int lo = max(t.sl * 64, cb), hi = min(t.sl * 64 + 63, K);
  return (t.sl == 0 ? 1u : 0u) + (hi >= lo ? (uint32_t)(hi - lo + 1) : 0u);
}

// predicted-nz image (the band and the row above) and per-slice non-zero counts.
// Round 6: every position's loads (its strategy byte, three counts) are
// issued before the first LDS store -- the strided loop waited a memory
// latency per position and channel (the phase clock put ~90 K cycles per band
// workgroup here, a third of its time).
template <int BR>
__device__ __forceinline__ void fill_slices(const AcArgs& a, const GroupGeom& G,
                                            const SliceTask& t, AcLds<BR>& L, int y0) {
  const size_t nb = (size_t)a.bxs * a.bys;
  constexpr int kPos = (BR + 1) * 32, kNT = BR * 32, kIt = (kPos + kNT - 1) / kNT;
  uint32_t acsv[kIt], nzv[kIt][3];
  bool in[kIt];
#pragma unroll
  for (int it = 0; it < kIt; it++) {
    const int i = threadIdx.x + it * kNT, r = i >> 5, bx = i & 31, by = y0 - 1 + r;
    in[it] = i < kPos && bx < G.gw && by >= 0 && by < G.gh;
    const size_t gb = in[it] ? (size_t)(G.by0 + by) * a.bxs + G.bx0 + bx : 0;
    acsv[it] = in[it] ? a.acs[gb] : 0u;
#pragma unroll
    for (int c = 0; c < 3; c++) nzv[it][c] = in[it] ? a.nz[c * nb + gb] : 0u;
  }
#pragma unroll
  for (int it = 0; it < kIt; it++) {
    if (!in[it]) continue;
    const int i = threadIdx.x + it * kNT;
    int l, cx, cy;
    varblock_dims((int)acsv[it], l, cx, cy);  // covered blocks (flag set) hold scaled counts
#pragma unroll
    for (int c = 0; c < 3; c++) L.nz[c][i] = (uint8_t)((nzv[it][c] + (1u << l) - 1) >> l);
  }
  if (t.valid && t.lcb > 0) {
    const int cb = 1 << t.lcb, me = threadIdx.x;
#pragma unroll 1
    for (int c = 0; c < 3; c++) {
      uint32_t w[32];
      load_coefs(a.ac + (t.gb * 3 + c) * 64, w);
      int n = 0, lk = -1;
#pragma unroll
      for (int kk = 0; kk < 64; kk++) {
        const bool on = (t.sl * 64 + kk >= cb) && coef(w, kk) != 0;
        n += on;
        lk = on ? kk : lk;
      }
      L.snz[c][me] = (uint8_t)n;
      L.last[c][me] = coef(w, 63) != 0;
      L.lastk[c][me] = (int8_t)lk;
    }
  }
}

// walk state of task (t, c) at its first coefficient; nz = varblock count
template <int BR>
__device__ __forceinline__ void slice_state(const SliceTask& t, const AcLds<BR>& L, int c, int y0,
                                            int nz, int& left, int& prev) {
  const int cb = 1 << t.lcb;
  left = nz;
  prev = nz > cb * 4 ? 0 : 1;  // nz > size / 16
  if (t.sl > 0) {
    for (int j = 0; j < t.sl; j++) left -= L.snz[c][block_of_slice(t, j, y0)];
    if (t.sl * 64 - 1 >= cb) prev = L.last[c][block_of_slice(t, t.sl - 1, y0)];
  }
}

// workgroup (NT threads) exclusive scan; *total = sum of all values
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sWave,
                                                    uint32_t* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  if (lane == 63) sWave[wv] = incl;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) {
    const uint32_t x = sWave[i];
    before += i < wv ? x : 0u;
    all += x;
  }
  *total = all;
  return before + incl - v;
}

// JXG_FRONT_PROFILE (experiment builds only): ac_hist phase clock sums of
// thread 0 of every band workgroup, printed by dump_hist_profile()
#ifdef JXG_FRONT_PROFILE
__device__ unsigned long long g_hprof[8];
#define HPROF(k)                                                     \
  do {                                                               \
    if (threadIdx.x == 0) {                                          \
      const unsigned long long now_ = __builtin_readcyclecounter();  \
      if ((k) > 0) atomicAdd(&g_hprof[(k)], now_ - hprof_t0);       \
      else atomicAdd(&g_hprof[0], 1ull);                             \
      hprof_t0 = now_;                                               \
    }                                                                \
  } while (0)
void dump_hist_profile() {
  unsigned long long h[8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_hprof), sizeof(h)) != hipSuccess) return;
  static const char* kNames[6] = {"workgroups", "fill slices", "token counts", "scan", "walk", "flush"};
  std::fprintf(stderr, "ac_hist thread-0 shader cycles (Mcycles summed over workgroups):\n");
  for (int k = 0; k < 6; k++) std::fprintf(stderr, "  %-16s %12.3f\n", kNames[k], k ? h[k] / 1e6 : (double)h[0]);
}
#else
#define HPROF(k) \
  do {           \
  } while (0)
void dump_hist_profile() {}
#endif
// The band's clustered histogram in LDS.  An 8-row band (BR = 8) has at most
// 256 x 3 x 64 + 768 = 49920 tokens, so its counts are u16, two bins per word,
// and a half never carries.  The whole-group form (BR = 32, effort >= 8) walks
// up to 1024 x 3 x 64 + 3072 tokens, and one bin can pass 65535 (a DCT256X256
// whose X and B hold only their last coefficient puts ~129 K zero tokens into
// one cluster; tests/test_gpu_bigvb.py::test_whole_group_histogram_bin_above_u16):
// u32 bins there (67.6 KB of LDS for the histogram).
template <int BR>
__global__ __launch_bounds__(BR * 32) void ac_hist_kernel(Batch<AcArgs> bt_) {
  constexpr int kBandBlocks = BR * 32, kHistThreads = kBandBlocks, kWgBands = 32 / BR;
  const AcArgs& a = bt_.a[blockIdx.z];  // the batch's frame
  constexpr bool kWide = BR == 32;  // u32 bins
  constexpr int kHistWords = kWide ? kMaxClusters * kAcTok : kMaxClusters * kAcTok / 2;
  __shared__ uint32_t sHist[kHistWords];
  __shared__ AcLds<BR> L;
  __shared__ __attribute__((aligned(16))) uint8_t sClu[kAcCtxPad];
  __shared__ uint32_t sTask[3][kBandBlocks];  // tokens per (channel, slice task)
  __shared__ uint32_t sBase[kBandBlocks];     // first token of each varblock (first block)
  __shared__ uint32_t sWave[kHistThreads / 64];
  __shared__ uint32_t sBound, sNtok[3];
  __shared__ uint16_t sNnzCtx[64];
  __shared__ uint8_t sFreqCtx[64];
  const uint32_t slot = blockIdx.x / kWgBands, band = blockIdx.x % kWgBands;
  const int g = (int)slot_group(a.glist, a.g0, slot);
  const GroupGeom G = group_geom(a, g);
  const int y0 = (int)band * BR;
  if (BR == 32 && threadIdx.x > 0 && threadIdx.x < kBands)
    a.bandtok[g * kBands + threadIdx.x] = 0;  // one band holds the whole group's stream
  if (y0 >= G.gh) {  // below a partial bottom group: an empty band
    if (threadIdx.x == 0) a.bandtok[g * kBands + band] = 0;
    return;
  }
#ifdef JXG_FRONT_PROFILE
  unsigned long long hprof_t0 = 0;
#endif
  HPROF(0);
  for (int i = threadIdx.x; i < kHistWords; i += blockDim.x) sHist[i] = 0;
  if (threadIdx.x < 64) {
    sNnzCtx[threadIdx.x] = (uint16_t)nnz_ctx(threadIdx.x);
    sFreqCtx[threadIdx.x] = (uint8_t)freq_ctx(threadIdx.x);
  }
  {  // the cluster map: 16-byte loads, all issued before the stores
    constexpr int kQ = kAcCtxPad / 16, kQIt = (kQ + kHistThreads - 1) / kHistThreads;
    uint4 q[kQIt];
#pragma unroll
    for (int it = 0; it < kQIt; it++) {
      const int i = threadIdx.x + it * kHistThreads;
      q[it] = i < kQ ? reinterpret_cast<const uint4*>(c_cluster)[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int it = 0; it < kQIt; it++) {
      const int i = threadIdx.x + it * kHistThreads;
      if (i < kQ) reinterpret_cast<uint4*>(sClu)[i] = q[it];
    }
  }
  if (threadIdx.x < 3) sNtok[threadIdx.x] = 0;
  if (threadIdx.x == 0) sBound = 0;
  const SliceTask t = slice_task(a, G, y0);
  uint32_t nzo[3];  // the varblock's non-zero counts (the walk's start state)
#pragma unroll
  for (int c = 0; c < 3; c++) nzo[c] = t.valid ? a.nz[c * (size_t)a.bxs * a.bys + t.ogb] : 0u;
  fill_slices(a, G, t, L, y0);
  __syncthreads();
  HPROF(1);
  const int me = threadIdx.x;
  // token counts per task without a walk -> stream positions (varblocks by
  // first block raster, channels Y, X, B, slices): one scan over varblocks
  if (t.valid) {
#pragma unroll 1
    for (int ci = 0; ci < 3; ci++) sTask[ci][me] = task_token_count(a, t, L, channel_of(ci), y0);
  }
  __syncthreads();
  HPROF(2);
  uint32_t vtot = 0;
  const int cb = 1 << t.lcb;
  if (t.valid && t.sl == 0) {
    for (int ci = 0; ci < 3; ci++)
      for (int j = 0; j < cb; j++) vtot += sTask[ci][block_of_slice(t, j, y0)];
  }
  uint32_t total;
  const uint32_t off = block_excl_scan<kHistThreads>(vtot, sWave, &total);
  if (t.valid && t.sl == 0) sBase[me] = off;
  __syncthreads();
  HPROF(3);
  // one walk: clustered histogram, bit bound, and every token's 32-bit record
  // at its stream position.  Wave-parallel: each thread derives the walk state
  // of its own task (slice, channel); the wave then takes its 64 tasks one at
  // a time with lane = coefficient, so a task costs one pass whatever its token
  // count (no walk divergence) and its records are stored contiguously.
  // Per coefficient k >= lo: left_k = left - (non-zeros in [lo, k)) (ballot +
  // popcount), prev_k = the walk's start flag at lo, else (coef k-1 != 0);
  // token iff left_k > 0 -- the serial walk of block_tokens /
  // varblock_slice_tokens, restated.
  uint32_t bound = 0, nt[3] = {0, 0, 0};
  uint32_t* rec = a.tokens + (uint64_t)slot * kGroupTokStride + (uint64_t)band * kBandTokStride;
  uint32_t pos = t.valid ? sBase[(t.oby - y0) * 32 + t.obx] : 0u;
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  auto hist_add = [&](uint32_t clu, uint32_t tok) {
    const uint32_t bin = clu * kAcTok + tok;
    if (kWide)
      atomicAdd(&sHist[bin], 1u);
    else
      atomicAdd(&sHist[bin >> 1], 1u << ((bin & 1u) * 16u));
  };
#pragma unroll 1
  for (int ci = 0; ci < 3; ci++) {
    const int c = channel_of(ci);
    uint32_t idx = 0, cnt = 0, info = 0, info2 = 0, tok0 = 0;
    if (t.valid) {
      uint32_t before = 0, chan_total = 0;
      for (int j = 0; j < cb; j++) {
        const uint32_t b = sTask[ci][block_of_slice(t, j, y0)];
        before += j < t.sl ? b : 0u;
        chan_total += b;
      }
      idx = pos + before;
      cnt = sTask[ci][me];
      pos += chan_total;
      const int nz = (int)nzo[c];
      int left, prev;
      slice_state(t, L, c, y0, nz, left, prev);
      const int bctx = block_ctx_of(c, t.type);
      // info: left (16 bits) | prev << 16 | lcb << 17 (4 bits) | bctx << 21;
      // info2: the slice index (varblocks of up to 1024 blocks)
      info = (uint32_t)left | ((uint32_t)prev << 16) | ((uint32_t)t.lcb << 17) |
             ((uint32_t)bctx << 21);
      info2 = (uint32_t)t.sl;
      if (t.sl == 0) {  // the non-zero count token, written by the task's own thread
        const int pred = predict_nz(L.nz[c], t.bx, t.by, y0);
        uint32_t tok, nb, bits;
        hybrid420((uint32_t)nz, tok, nb, bits);
        const uint32_t clu = sClu[nz_bucket(pred) * kBlockCtx + bctx];
        hist_add(clu, tok);
        bound += 15u + nb;
        tok0 = clu | (tok << 8) | (nb << 14) | (bits << 18);
        rec[idx] = tok0;
      }
      nt[0] += c == 0 ? cnt : 0u;
      nt[1] += c == 1 ? cnt : 0u;
      nt[2] += c == 2 ? cnt : 0u;
    }
    // tasks with coefficient tokens, taken kBatch at a time: their coefficient
    // loads are issued together (one memory latency per batch)
    const bool need = t.valid && cnt > (t.sl == 0 ? 1u : 0u);
    const uint32_t qoff = (uint32_t)((t.gb * 3 + c) * 64);
    uint64_t M = __ballot(need);
#ifndef JXG_AC_BATCH
#define JXG_AC_BATCH 8
#endif
    constexpr int kBatch = JXG_AC_BATCH;
    while (M) {
      int js[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; u++) {
        js[u] = M ? (int)__builtin_ctzll(M) : -1;
        M = M ? M & (M - 1) : 0ull;
      }
      int32_t v8[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; u++)
        v8[u] = js[u] >= 0 ? a.ac[(uint32_t)__builtin_amdgcn_readlane((int)qoff, js[u]) + lane] : 0;
#pragma unroll
      for (int u = 0; u < kBatch; u++) {
        if (js[u] < 0) break;
        const int j = js[u];
        const uint32_t ij = (uint32_t)__builtin_amdgcn_readlane((int)info, j);
        const uint32_t idxj = (uint32_t)__builtin_amdgcn_readlane((int)idx, j);
        const int slj = __builtin_amdgcn_readlane((int)info2, j), lcbj = (ij >> 17) & 15;
        const int leftj = ij & 0xFFFF, prevj = (ij >> 16) & 1, bctxj = ij >> 21;
        const int cbj = 1 << lcbj;
        const int k = slj * 64 + lane;
        const int lo = max(slj * 64, cbj);
        const int32_t v = v8[u];
        const bool on = k >= cbj;
        const uint64_t m = __ballot(on && v != 0);
        const int left_k = leftj - __popcll(m & below);
        if (on && left_k > 0) {
          const int prev_k = k == lo ? prevj : (int)((m >> (lane - 1)) & 1);
          const int ctx = kBlockCtx * kNzBuckets + kZdCtx * bctxj +
                          (sNnzCtx[(left_k + cbj - 1) >> lcbj] + sFreqCtx[k >> lcbj]) * 2 + prev_k;
          uint32_t tok, nb, bits;
          hybrid420(pack_signed(v), tok, nb, bits);
          const uint32_t clu = sClu[ctx];
          hist_add(clu, tok);
          bound += 15u + nb;
          rec[idxj + (slj == 0 ? 1u : 0u) + (uint32_t)(k - lo)] =
              clu | (tok << 8) | (nb << 14) | (bits << 18);
        }
      }
    }
  }
  atomicAdd(&sBound, bound);
  atomicAdd(&sNtok[0], nt[0]);
  atomicAdd(&sNtok[1], nt[1]);
  atomicAdd(&sNtok[2], nt[2]);
  __syncthreads();
  HPROF(4);
  for (int i = threadIdx.x; i < kHistWords; i += blockDim.x) {
    const uint32_t w = sHist[i];
    if (!w) continue;
    if (kWide) {
      atomicAdd(&a.hist[(i / kAcTok) * kAlpha + (i % kAcTok)], w);
      continue;
    }
    const int bin = 2 * i;
    if (w & 0xFFFFu) atomicAdd(&a.hist[(bin / kAcTok) * kAlpha + (bin % kAcTok)], w & 0xFFFFu);
    if (w >> 16) atomicAdd(&a.hist[((bin + 1) / kAcTok) * kAlpha + ((bin + 1) % kAcTok)], w >> 16);
  }
  // (bound and ntok: zeroed with the statistics arena; bandtok written here)
  if (threadIdx.x == 0) {
    atomicAdd(&a.bound[g], sBound);
    atomicAdd(&a.ntok[g * 3 + 0], sNtok[0]);
    atomicAdd(&a.ntok[g * 3 + 1], sNtok[1]);
    atomicAdd(&a.ntok[g * 3 + 2], sNtok[2]);
    a.bandtok[g * kBands + band] = total;
  }
  HPROF(5);
}

// prefix-code emission from the group's token records (no coefficient walk):
// wave w owns a contiguous record range; lanes read consecutive records
// (coalesced), the wave's bit total -> workgroup offsets; then per 64
// records a wave inclusive scan of the lengths gives every record its bit
// position, and each lane ORs its <= 28 bits into the LDS bit buffer (global
// atomics for groups larger than the buffer)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d);
    if (lane >= d) v += t;
  }
  return v;
}
__global__ __launch_bounds__(kAcThreads) void ac_emit_kernel(AcArgs a) {
  __shared__ uint32_t sCode[kMaxClusters * kAcTok];
  __shared__ __attribute__((aligned(16))) uint32_t sBits[kEmitLdsWords];
  __shared__ uint32_t sWave[kAcThreads / 64];
  const int g = (int)slot_group(a.glist, a.g0, blockIdx.x);
  for (int i = threadIdx.x; i < kMaxClusters * kAcTok; i += blockDim.x)
    sCode[i] = a.codes[(i / kAcTok) * kAlpha + (i % kAcTok)];
  for (int i = threadIdx.x; i < kEmitLdsWords / 4; i += blockDim.x)
    reinterpret_cast<uint4*>(sBits)[i] = make_uint4(0, 0, 0, 0);
  const uint32_t n = a.ntok[g * 3] + a.ntok[g * 3 + 1] + a.ntok[g * 3 + 2];
  const uint32_t* rec = a.tokens + (uint64_t)blockIdx.x * kGroupTokStride;
  uint32_t bt[kBands];
#pragma unroll
  for (int i = 0; i < kBands; i++) bt[i] = a.bandtok[g * kBands + i];
  constexpr int kWaves = kAcThreads / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t chunk = ((n + kWaves * 64 - 1) / (kWaves * 64)) * 64;
  const uint32_t lo = min(n, wv * chunk), hi = min(n, lo + chunk);
  __syncthreads();
  auto code_of = [&](uint32_t r) { return sCode[(r & 0xFF) * kAcTok + ((r >> 8) & 63)]; };
  uint32_t tot = 0;
  for (uint32_t k = lo + lane; k < hi; k += 64) {
    const uint32_t r = rec[rec_index(bt, k)];
    tot += (code_of(r) >> 16) + ((r >> 14) & 15);
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) tot += __shfl_xor(tot, d, 64);
  if (lane == 0) sWave[wv] = tot;
  __syncthreads();
  uint32_t run = 0, total = 0;
#pragma unroll
  for (int i = 0; i < kWaves; i++) {
    const uint32_t x = sWave[i];
    run += i < wv ? x : 0u;
    total += x;
  }
  const uint64_t base = a.base[g];  // word aligned
  const bool lds = total <= (uint32_t)kEmitLdsWords * 32u;
  if (!lds) {  // the section's scratch words zeroed before the global ORs (no arena memset)
    for (uint32_t i = threadIdx.x; i < (total + 31) / 32; i += blockDim.x) a.scratch[(base >> 5) + i] = 0;
    __threadfence();
    __syncthreads();
  }
  uint32_t* buf = lds ? sBits : a.scratch;
  const uint64_t bias = lds ? 0 : base;
  for (uint32_t k0 = lo; k0 < hi; k0 += 64) {
    const uint32_t k = k0 + lane;
    uint32_t len = 0, val = 0;
    if (k < hi) {
      const uint32_t r = rec[rec_index(bt, k)], cl = code_of(r);
      len = (cl >> 16) + ((r >> 14) & 15);
      // code (<= 15 bits) and raw bits (<= 13): one <= 28-bit value
      val = (cl & 0xFFFFu) | ((r >> 18) << (cl >> 16));
    }
    const uint32_t incl = wave_incl_scan(len);
    if (len) {
      const uint64_t pos = bias + run + incl - len;
      const uint64_t w = pos >> 5;
      const uint32_t sh = (uint32_t)(pos & 31);
      atomicOr(&buf[w], val << sh);
      if (sh + len > 32) atomicOr(&buf[w + 1], val >> (32 - sh));
    }
    run += __shfl(incl, 63, 64);
  }
  if (lds) {
    __syncthreads();
    const uint32_t nw = (total + 31) / 32;
    uint32_t* dst = a.scratch + (base >> 5);
    for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) dst[i] = sBits[i];
  }
  if (threadIdx.x == 0) a.bits[g] = total;
}

// ---------------------------------------------------------------------------
// ANS: the token records ac_hist wrote in stream order; one lane per group
// runs the rANS encoder backwards over its records (the stream's only
// sequential dependency), then the group's workgroup places the emitted bits
// in parallel.
// ---------------------------------------------------------------------------
// rANS backwards over each group's records, one wave per group, kAnsWaves
// groups per workgroup sharing the LDS tables (all alias inverses, 64 KB).
//
// The state recurrence is the stream's only sequential dependency, so its
// per-step latency sets the kernel time (a pass group holds up to ~100K
// tokens).  The chain runs "on the diagonal": lane L holds record L's
// constants in registers (no readlane per step) and step L is computed in
// lane L from lane L-1's result, which a DPP wave rotation (wave_ror:1, VALU
// to VALU) hands over; the other lanes run the same rANS steps on other
// (valid) states, so every lane's table address stays in range.  The state
// x = k << 12 | v is kept as (k = quotient of the previous step, v = its
// inverse-table entry).  One wave issues about one instruction per 4 cycles
// whatever its dependency depth, so the step is cut to its fewest
// instructions (15 issue slots; ns per token at 8K: 62.3 -> 56.5 -> 49.6 over
// the three forms tried, profiles/r03p):
//   * in the read's shadow: k from lane L-1 (DPP), emission k >= f << 8
//     (x >= f << 20), which makes the shift sh = 16 (x >> 16 = k >> 4: v
//     drops out) or 0; lane s-1 saves its pre-step state (constant-mask select);
//   * after the read: x = k << 12 + v, xs = x >> sh, the quotient
//     floor(xs / f) = trunc((xs + 0.5) * rcp(f)) in f64 (cvt, fma, cvt; exact:
//     one rounding, < 2^-19, while (xs + .5) / f stays >= .5 / f from an
//     integer), the table address base + 2 (xs - q f) (shift-add, 24-bit
//     multiply-add), the next read.
// Per 64 records the lanes decode record, f, rcp and table base in parallel
// (the next 64 records are fetched meanwhile) and store the emitted bits of
// their record with one coalesced store.
// (A uniform variant -- every lane runs the same step, the quotient on the
// scalar unit from readlane'd constants, two vector multiply-adds between the
// reads -- is exact but took 17.5 vs 6.35 ms: ~60 instructions per step.)
// Two chain waves per SIMD (8 per workgroup, 68 KB of LDS): the second wave
// delays every step by its own issue (one frame's chains 6.7 vs 6.0 ms at 8K
// with 4 per workgroup, profiles/r02g), but the chains of a frame occupy 64
// CUs instead of 128, so the transform kernels of the frames behind keep full
// occupancy on the rest (pipelined 8K +3.5 %).  The chain waves
// run at the highest wave priority so co-resident transform waves only fill
// their idle issue slots.
#ifndef JXG_ANS_WAVES  // (experiment builds override it: tools/build_variant.sh)
#define JXG_ANS_WAVES 8
#endif
constexpr int kAnsWaves = JXG_ANS_WAVES;
__device__ __forceinline__ uint32_t wave_ror1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x13C, 0xF, 0xF, false);
}
// blk: the chain workgroup's index within its frame
__device__ __forceinline__ void ans_chain(const AnsArgs& a, uint32_t blk) {
  __shared__ uint32_t sSym[kAnsHists * 128];
  __shared__ uint32_t sInv[kAnsHists * 4096 / 2];  // u16 pairs
  __shared__ uint8_t sMap[136];
  const uint32_t* src = reinterpret_cast<const uint32_t*>(a.tab);
  for (uint32_t i = threadIdx.x; i < a.nhist * 128; i += blockDim.x) sSym[i] = src[i];
  for (uint32_t i = threadIdx.x; i < a.nhist * 2048; i += blockDim.x)
    sInv[i] = src[kAnsInvOff / 4 + i];
  for (uint32_t i = threadIdx.x; i < 136; i += blockDim.x) sMap[i] = a.tab[kAnsMapOff + i];
  __syncthreads();
  const uint8_t* inv = reinterpret_cast<const uint8_t*>(sInv);
  const uint32_t lane = threadIdx.x & 63;
  // the chain's group: groups sorted longest first (host), kAnsWaves per
  // workgroup, so a workgroup's waves finish at about the same time and the
  // workgroups of short groups free their CUs early
  const uint32_t gi = __builtin_amdgcn_readfirstlane(blk * kAnsWaves + (threadIdx.x >> 6));
  if (gi >= a.n) return;
  const uint32_t slot = __builtin_amdgcn_readfirstlane(a.order[gi]);
  const uint32_t g = __builtin_amdgcn_readfirstlane(slot_group(a.glist, a.g0, slot));
  __builtin_amdgcn_s_setprio(3);
  const int n = (int)(a.ntok[g * 3] + a.ntok[g * 3 + 1] + a.ntok[g * 3 + 2]);
  const uint64_t b = (uint64_t)slot * kGroupTokStride;
  uint32_t bt[kBands];  // the group's stream = its bands' record spaces, in order
#pragma unroll
  for (int i = 0; i < kBands; i++) bt[i] = a.bandtok[g * kBands + i];
  // every lane starts from the initial state x = 0x130000
  uint32_t k = 0x130u, v = 0;
  uint32_t rec = (int)lane < min(64, n) ? a.tokens[b + rec_index(bt, n - 1 - lane)] : 0u;
  for (int hi = n; hi > 0; hi -= 64) {
    const int cnt = min(64, hi);
    // lane L: record hi - 1 - L.  Lanes past cnt get f = 4096 (a valid
    // never-emitting step on histogram 0).
    uint32_t f = 4096, base2 = 0;
    if ((int)lane < cnt) {
      const uint32_t h = sMap[rec & 0xFF], e = sSym[h * 128 + ((rec >> 8) & 63)];
      f = (e & 0xFFF) + 1;
      base2 = 2 * (h * 4096 + (e >> 12));  // byte offset of the symbol's inverse row
    }
    const uint32_t Fq = f << 8;  // emit iff k >= Fq
    const uint32_t nf2 = (uint32_t)(-(int)(2 * f));
    const double rcp = 1.0 / (double)f, hr = 0.5 * rcp;
    const int hn = hi - 64;
    const uint32_t nrec = (int)lane < min(64, hn) ? a.tokens[b + rec_index(bt, hn - 1 - lane)] : 0u;
    uint32_t X = 0;     // lane L: the state before record L's step
    uint32_t xin = 0;   // the state handed to the previous step
    auto step = [&](int s) {
      // shadow: emission (a shift of 16 drops v: (k << 12 | v) >> 16 = k >> 4),
      // and the previous step's input state into its lane
      const uint32_t kin = wave_ror1(k);
      const uint32_t sh = kin >= Fq ? 16u : 0u;
      if (s > 0)
        asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(X) : "v"(X), "v"(xin), "s"(1ull << (s - 1)));
      __builtin_amdgcn_sched_barrier(0);
      // critical path: v -> x -> xs -> quotient -> address -> next read
      const uint32_t vin = wave_ror1(v);
      const uint32_t x = (kin << 12) + vin;
      const uint32_t xs = x >> sh;
      const uint32_t kk = (uint32_t)__builtin_fma((double)xs, rcp, hr);
      const uint32_t x2 = (xs << 1) + base2;
      uint32_t addr;
      asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(addr) : "v"(kk), "v"(nf2), "v"(x2));
      v = *reinterpret_cast<const uint16_t*>(inv + addr);
      k = kk;
      xin = x;
      __builtin_amdgcn_sched_barrier(0);
    };
    if (cnt == 64) {
#pragma unroll
      for (int s = 0; s < 64; s++) step(s);
      asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(X) : "v"(X), "v"(xin), "s"(1ull << 63));
    } else {
      for (int s = 0; s < cnt; s++) {
        const uint32_t kin = wave_ror1(k);
        const bool emit = kin >= Fq;
        const uint32_t t = (kin << 12) >> (emit ? 16 : 0);
        const double P = __builtin_fma((double)t, rcp, hr);
        const uint32_t C = 2 * t + base2;
        const uint32_t vin = wave_ror1(v);
        X = (int)lane == s ? (kin << 12) + vin : X;
        const uint32_t vv = emit ? 0u : vin;
        const uint32_t kk = (uint32_t)__builtin_fma((double)vv, rcp, P);
        const uint32_t addr = (uint32_t)((int)(2 * vv + C) - (int)(2 * f) * (int)kk);
        v = *reinterpret_cast<const uint16_t*>(inv + addr);
        k = kk;
      }
    }
    if ((int)lane < cnt) {
      // emitted bits of the record: [16-bit chunk] then its raw bits (their
      // sums per chunk: ans_sums, off the chain)
      const bool em = (X >> 20) >= f;
      const uint32_t raw = rec >> 18, nb = (rec >> 14) & 15;
      a.val[b + hi - 1 - lane] = em ? (X & 0xFFFFu) | raw << 16 : raw;
      a.len[b + hi - 1 - lane] = (uint8_t)(em ? nb + 16 : nb);
    }
    rec = nrec;
    if (hi <= 64) {  // the final state: lane cnt - 1's result
      const uint32_t kf = __builtin_amdgcn_readlane(k, cnt - 1);
      const uint32_t vf = __builtin_amdgcn_readlane(v, cnt - 1);
      if (lane == 0) a.state[g] = (kf << 12) + vf;
    }
  }
  if (n == 0 && lane == 0) a.state[g] = 0x130000u;
}
__global__ __launch_bounds__(kAnsWaves * 64) void ans_encode_kernel(Batch<AnsArgs> bt_) {
  ans_chain(bt_.a[blockIdx.z], blockIdx.x);
}
// After the chains, one 256-thread workgroup per group: the emitted bits of
// every 64-record chunk q (stream order; records [n - 64 (K - q), n - 64 (K -
// q - 1)) clipped at 0) into csum[q], from which ans_emit places its
// segments; the section's bit count (the 32-bit state, then every record's
// bits); and the section's scratch words zeroed (ans_emit ORs the two words a
// segment shares with its neighbours; no arena memset).  Round 4 did this
// bookkeeping inside the chain, on its serial path.
constexpr int kSumThreads = 1024;
__global__ __launch_bounds__(kSumThreads) void ans_sums_kernel(Batch<AnsArgs> bt_) {
  __shared__ uint32_t sC[kAnsMaxChunks];
  __shared__ uint32_t sTot[kSumThreads / 64];
  const AnsArgs& a = bt_.a[blockIdx.z];
  const uint32_t slot = blockIdx.x;
  if (slot >= a.n) return;
  const uint32_t g = slot_group(a.glist, a.g0, slot);
  const uint32_t n = a.ntok[g * 3] + a.ntok[g * 3 + 1] + a.ntok[g * 3 + 2];
  const uint32_t K = (n + 63) / 64;
  const uint64_t b = (uint64_t)slot * kGroupTokStride;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t q = threadIdx.x; q < K; q += kSumThreads) sC[q] = 0;
  __syncthreads();
  // chunk q = records [64 q - off, 64 q + 64 - off) clipped at 0 (chunks end
  // at n); 16-byte words of the lengths: a chunk boundary can only fall at
  // byte r = n % 16 of a word (n - 64 (K - q) = r mod 16), so a word's bytes
  // below r go to one chunk and the rest to one chunk (LDS adds)
  const uint32_t off = (64u - (n & 63u)) & 63u, r = n & 15u;
  const uint4* L = reinterpret_cast<const uint4*>(a.len + b);
  for (uint32_t w = threadIdx.x; w < (n + 15) / 16; w += kSumThreads) {
    const uint4 v = L[w];
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
    const uint32_t valid = min(16u, n - 16u * w);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) {
      const uint32_t x = j < valid ? (d[j >> 2] >> (8 * (j & 3))) & 0xFFu : 0u;
      if (j < r) lo += x;
      else hi += x;
    }
    if (lo) atomicAdd(&sC[(16u * w + off) >> 6], lo);
    if (hi) atomicAdd(&sC[(16u * w + r + off) >> 6], hi);
  }
  __syncthreads();
  uint32_t* csum = a.csum + (uint64_t)slot * kAnsMaxChunks;
  uint32_t tot = 0;
  for (uint32_t q = threadIdx.x; q < K; q += kSumThreads) {
    const uint32_t c = sC[q];
    csum[q] = c;
    tot += c;
  }
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) tot += __shfl_xor(tot, m, 64);
  if (lane == 0) sTot[wv] = tot;
  __syncthreads();
  uint32_t total = 32;
#pragma unroll
  for (int i = 0; i < kSumThreads / 64; i++) total += sTot[i];
  if (threadIdx.x == 0) a.bits[g] = total;
  uint32_t* dst = a.scratch + (a.base[g] >> 5);
  for (uint32_t i = threadIdx.x; i < (total + 31) / 32; i += kSumThreads) dst[i] = 0;
}
// bit placement: the 32-bit state, then every record's bits, in order.  One
// 256-thread workgroup per (group, segment of kSegChunks chunks of 64
// records): the segment's first bit is 32 + the chain's chunk sums before it
// (no pass over the lengths); each wave places whole chunks (their offsets
// from the same sums) with a wave scan of the lengths into an LDS image of
// the segment aligned to the scratch words, then the workgroup stores it --
// plain stores inside the segment, atomic ORs on the two words it may share
// with its neighbours (zeroed by the chain).
constexpr int kSegChunks = 64, kEmitThreads = 256;
constexpr int kSegWords = (kSegChunks * 64 * 29 + 31) / 32 + 2;  // <= 29 bits per record
__global__ __launch_bounds__(kEmitThreads) void ans_emit_kernel(Batch<AnsArgs> bt_) {
  __shared__ __attribute__((aligned(16))) uint32_t sBits[kSegWords];
  __shared__ uint32_t sCs[kSegChunks + 1];
  __shared__ uint32_t sPre[kEmitThreads / 64];
  const AnsArgs& a = bt_.a[blockIdx.z];
  const uint32_t slot = blockIdx.x, seg = blockIdx.y;
  if (slot >= a.n) return;
  const uint32_t g = slot_group(a.glist, a.g0, slot);
  const uint32_t n = a.ntok[g * 3] + a.ntok[g * 3 + 1] + a.ntok[g * 3 + 2];
  const uint32_t K = (n + 63) / 64, q0 = seg * kSegChunks;
  const uint64_t base = a.base[g];  // word aligned
  if (seg == 0 && threadIdx.x == 0) a.scratch[base >> 5] = a.state[g];
  if (q0 >= K) return;
  const uint32_t q1 = min(K, q0 + kSegChunks);
  const uint32_t* csum = a.csum + (uint64_t)slot * kAnsMaxChunks;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // bits before the segment: 32 + sum of the chunks before q0
  uint32_t pre = 0;
  for (uint32_t q = threadIdx.x; q < q0; q += kEmitThreads) pre += csum[q];
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) pre += __shfl_xor(pre, d, 64);
  if (lane == 0) sPre[wv] = pre;
  if (threadIdx.x <= kSegChunks) sCs[threadIdx.x] = q0 + threadIdx.x < q1 ? csum[q0 + threadIdx.x] : 0u;
  for (int i = threadIdx.x; i < kSegWords; i += kEmitThreads) sBits[i] = 0;
  __syncthreads();
  const uint64_t start = base + 32 + sPre[0] + sPre[1] + sPre[2] + sPre[3];  // the segment's first bit
  const uint32_t sh0 = (uint32_t)(start & 31);
  uint32_t segbits = 0;
  for (uint32_t q = 0; q < q1 - q0; q++) segbits += sCs[q];
  // chunk q's records: [chunk_lo(q), chunk_lo(q + 1)), chunk_lo(K) = n
  auto chunk_lo = [&](uint32_t q) { return q == 0 ? 0u : n - 64u * (K - q); };
  const uint64_t b = (uint64_t)slot * kGroupTokStride;
  constexpr int kPerWave = kSegChunks / (kEmitThreads / 64);
  uint32_t run = sh0;  // bit offset inside the LDS image
  for (int i = 0; i < wv * kPerWave; i++) run += sCs[i];
  for (int i = 0; i < kPerWave; i++) {
    const uint32_t q = q0 + (uint32_t)(wv * kPerWave + i);
    if (q >= q1) break;
    const uint32_t lo = chunk_lo(q), hi = chunk_lo(q + 1);
    const uint32_t k = lo + (uint32_t)lane;
    const uint32_t len = k < hi ? a.len[b + k] : 0u;
    const uint32_t val = k < hi ? a.val[b + k] : 0u;
    const uint32_t incl = wave_incl_scan(len);
    if (len) {
      const uint32_t pos = run + incl - len;
      const uint32_t w = pos >> 5, sh = pos & 31;
      atomicOr(&sBits[w], val << sh);
      if (sh + len > 32) atomicOr(&sBits[w + 1], val >> (32 - sh));
    }
    run += sCs[wv * kPerWave + i];
  }
  __syncthreads();
  const uint32_t nw = (sh0 + segbits + 31) / 32;
  uint32_t* dst = a.scratch + (start >> 5);
  for (uint32_t i = threadIdx.x; i < nw; i += kEmitThreads) {
    const uint32_t v = sBits[i];
    if (i == 0 || i == nw - 1) {
      if (v) atomicOr(&dst[i], v);
    } else {
      dst[i] = v;
    }
  }
}

// the chains, then the bit placement, of k frames (same plan: same group
// count; the segment grid covers the longest group of any of them)
void launch_ans(const AnsArgs* a, uint32_t k, hipStream_t s) {
  if (!k || !a[0].n) return;
  const Batch<AnsArgs> b = make_batch(a, k);
  uint32_t n = 0, maxtok = 0;
  for (uint32_t i = 0; i < k; i++) {
    n = max(n, a[i].n);
    maxtok = max(maxtok, a[i].max_tokens);
  }
  hipLaunchKernelGGL(ans_encode_kernel, dim3((n + kAnsWaves - 1) / kAnsWaves, 1, k),
                     dim3(kAnsWaves * 64), 0, s, b);
  hipLaunchKernelGGL(ans_sums_kernel, dim3(n, 1, k), dim3(kSumThreads), 0, s, b);
  const uint32_t nseg = (maxtok + kSegChunks * 64 - 1) / (kSegChunks * 64);
  if (nseg) hipLaunchKernelGGL(ans_emit_kernel, dim3(n, nseg, k), dim3(kEmitThreads), 0, s, b);
}

void launch_ac_hist(const AcArgs* a, uint32_t k, uint32_t ngroups, hipStream_t s, bool whole_group) {
  if (!ngroups || !k) return;
  if (whole_group)  // varblocks of 128 / 256 px (effort >= 8) span bands
    hipLaunchKernelGGL(ac_hist_kernel<32>, dim3(ngroups, 1, k), dim3(1024), 0, s, make_batch(a, k));
  else
    hipLaunchKernelGGL(ac_hist_kernel<8>, dim3(ngroups * kBands, 1, k), dim3(256), 0, s, make_batch(a, k));
}
void launch_ac_emit(const AcArgs& a, uint32_t ngroups, hipStream_t s) {
  if (ngroups) hipLaunchKernelGGL(ac_emit_kernel, dim3(ngroups), dim3(kAcThreads), 0, s, a);
}
hipError_t set_cluster_table(const uint8_t* tab, hipStream_t s) {
  return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_cluster), tab, kAcCtx, 0, hipMemcpyHostToDevice, s);
}

}  // namespace jxg
