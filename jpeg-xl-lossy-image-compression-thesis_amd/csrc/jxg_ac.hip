// jxg_ac.hip -- pass-group AC token statistics and bit emission on gfx950.
//
// One 1024-thread workgroup per 256x256-pixel pass group: thread = 8x8 block,
// its (block, channel) tasks Y, X, B in stream order.  A task's 64 int16 coefficients
// (128 B) are loaded with 8 x 16-byte loads into 32 VGPRs and the token walk
// runs on registers (fully unrolled, wave-uniform early exit every 8
// coefficients), so there are no dependent global loads in the walk.
//   ac_hist : non-zero counts -> predicted-nz + zero-density contexts ->
//             clustered histograms (LDS, one global atomic per non-empty bin),
//             exact per-group token counts, per-group bit upper bound.
//   ac_emit : same walk with the prefix codes (LDS table): per-block bit
//             lengths -> workgroup exclusive scan (stream order: blocks
//             raster, channels Y, X, B) -> every block writes its bits into an
//             LDS bit buffer (ds_or), copied out with plain 4-byte stores
//             (global atomics only for groups larger than the buffer).
// Token order / contexts are those of oracle/encode.c group_tokens, [ext]
// libjxl dec_group DecodeACVarBlock.
#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

__constant__ uint8_t c_cluster[kAcCtx];  // context -> static cluster id

constexpr int kAcThreads = 1024;

struct GroupGeom {
  int bx0, by0, gw, gh;
};
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

// Tokens of one (block, channel): f(ctx, value) in bitstream order.
template <class F>
__device__ __forceinline__ void block_tokens(const uint32_t* w, int nz, int pred, int bctx,
                                             F&& f) {
  f(nz_bucket(pred) * kBlockCtx + bctx, (uint32_t)nz);
  const int zoff = kBlockCtx * kNzBuckets + kZdCtx * bctx;
  int prev = nz > 4 ? 0 : 1;
  int left = nz;
  // 8 chunks of 8 coefficients; a chunk is skipped (wave-uniform branch) once
  // no lane of the wave has non-zeros left.  No loop exit, so every k stays a
  // compile-time register index.
#pragma unroll
  for (int ch = 0; ch < 8; ch++) {
    if (__any(left > 0)) {
#pragma unroll
      for (int kk = 0; kk < 8; kk++) {
        const int k = ch * 8 + kk;
        if (k == 0) continue;
        if (left > 0) {
          const int32_t v = coef(w, k);
          f(zoff + (kNnzCtx[left] + kFreqCtx[k]) * 2 + prev, pack_signed(v));
          prev = v != 0;
          left -= prev;
        }
      }
    }
  }
}

__device__ __forceinline__ int predict_nz(const uint8_t* nzc, int bx, int by) {
  if (bx == 0) return by == 0 ? 32 : nzc[(by - 1) * 32 + bx];
  if (by == 0) return nzc[by * 32 + bx - 1];
  return (nzc[(by - 1) * 32 + bx] + nzc[by * 32 + bx - 1] + 1) / 2;
}

__device__ __forceinline__ int block_ctx_of(int c, int acs) {
  return kDefaultCtxMap[(c < 2 ? c ^ 1 : 2) * 13 + kStrategyOrder[acs]];
}

// AC tokens are < 64: |q| <= 32767 -> packed value <= 65534 -> hybrid token
// <= 63; the non-zero count (<= 4032) token is <= 47.  Device tables use 64 columns.
constexpr int kAcTok = 64;
// LDS bit buffer of ac_emit (groups whose exact size exceeds it fall back to
// global atomics)
constexpr int kEmitLdsWords = 8192;  // 32 KiB = 262144 bits

__device__ __forceinline__ int channel_of(int ci) { return ci == 0 ? 1 : (ci == 1 ? 0 : 2); }

// covered blocks (log2) of a raw strategy id: 0 for the 8x8 class
__device__ __forceinline__ int log2_covered(int type) {
  switch (type) {
    case 6: case 7: return 1;                 // 16x8, 8x16
    case 4: case 10: case 11: return type == 4 ? 2 : 3;  // 16x16; 32x16, 16x32
    case 5: case 19: case 20: return type == 5 ? 4 : 5;  // 32x32; 64x32, 32x64
    case 18: return 6;                        // 64x64
    default: return 0;
  }
}
__device__ __forceinline__ int covered_x(int type) {  // blocks across
  switch (type) {
    case 7: case 4: return 2;
    case 10: return 2;
    case 11: case 5: case 19: return 4;
    case 20: case 18: return 8;
    default: return 1;
  }
}

// predicted-nz image of the group: per block, the varblock's non-zero count
// scaled down by its covered blocks (the merge kernel already stores the
// scaled value at covered non-first blocks)
__device__ __forceinline__ void fill_nz(const AcArgs& a, const GroupGeom& G,
                                        uint8_t (*sNz)[1024]) {
  const size_t nb = (size_t)a.bxs * a.bys;
  for (int i = threadIdx.x; i < 3 * 1024; i += blockDim.x) {
    const int c = i >> 10, by = (i >> 5) & 31, bx = i & 31;
    if (bx < G.gw && by < G.gh) {
      const size_t gb = (size_t)(G.by0 + by) * a.bxs + G.bx0 + bx;
      const int t = a.acs[gb];
      const int l = (t & 0x80) ? 0 : log2_covered(t);
      sNz[c][by * 32 + bx] = (uint8_t)((a.nz[c * nb + gb] + (1 << l) - 1) >> l);
    }
  }
}

// workgroup (1024 threads) exclusive scan; *total = sum of all values
__device__ __forceinline__ uint32_t block_excl_scan1024(uint32_t v, uint32_t* sWave,
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
  for (int i = 0; i < kAcThreads / 64; i++) {
    const uint32_t x = sWave[i];
    before += i < wv ? x : 0u;
    all += x;
  }
  *total = all;
  return before + incl - v;
}

// One thread per block of the group (<= 32 x 32 = 1024 blocks); the thread
// of a varblock's first block codes the whole varblock, its three
// (varblock, channel) tasks Y, X, B consecutive in the group's stream order;
// threads of covered blocks code nothing.
struct BlockTask {
  bool valid;
  int bx, by;
  size_t gb;
  int acs;
  int lcb, cx;  // log2 covered blocks, blocks across
};
__device__ __forceinline__ BlockTask block_task(const AcArgs& a, const GroupGeom& G) {
  BlockTask t;
  const int b = threadIdx.x;
  t.valid = b < G.gw * G.gh;
  t.bx = t.valid ? b % G.gw : 0;
  t.by = t.valid ? b / G.gw : 0;
  t.gb = (size_t)(G.by0 + t.by) * a.bxs + G.bx0 + t.bx;
  t.acs = t.valid ? a.acs[t.gb] : 0;
  if (t.acs & 0x80) t.valid = false;
  t.lcb = log2_covered(t.acs);
  t.cx = covered_x(t.acs);
  return t;
}

// Tokens of one merged varblock and channel: the non-zero count, then the
// coefficients k = cb .. (natural order, LLF skipped) while non-zeros are
// left; slices of 64 coefficients live in the covered blocks in raster order.
template <class F>
__device__ __forceinline__ void varblock_tokens(const AcArgs& a, const BlockTask& t, int nz,
                                                int pred, int bctx, int c, F&& f) {
  f(nz_bucket(pred) * kBlockCtx + bctx, (uint32_t)nz);
  const int cb = 1 << t.lcb, size = cb * 64;
  const int zoff = kBlockCtx * kNzBuckets + kZdCtx * bctx;
  int prev = nz > size / 16 ? 0 : 1;
  int left = nz;
#pragma unroll 1
  for (int sl = 0; sl < cb && left > 0; sl++) {
    const size_t gbs = t.gb + (size_t)(sl / t.cx) * a.bxs + sl % t.cx;
    uint32_t w[32];
    load_coefs(a.ac + (gbs * 3 + c) * 64, w);
#pragma unroll
    for (int kk = 0; kk < 64; kk++) {
      const int k = sl * 64 + kk;
      if (left > 0 && k >= cb) {
        const int32_t v = coef(w, kk);
        f(zoff + (kNnzCtx[(left + cb - 1) >> t.lcb] + kFreqCtx[k >> t.lcb]) * 2 + prev,
          pack_signed(v));
        prev = v != 0;
        left -= prev;
      }
    }
  }
}

template <class F>
__device__ __forceinline__ void block_channel_tokens(const AcArgs& a, const BlockTask& t,
                                                     uint8_t (*sNz)[1024], int c, F&& f) {
  const int pred = predict_nz(sNz[c], t.bx, t.by);
  const int bctx = block_ctx_of(c, t.acs);
  const int nz = a.nz[c * (size_t)a.bxs * a.bys + t.gb];
  if (t.lcb == 0) {
    uint32_t w[32];
    load_coefs(a.ac + (t.gb * 3 + c) * 64, w);
    block_tokens(w, nz, pred, bctx, f);
  } else {
    varblock_tokens(a, t, nz, pred, bctx, c, f);
  }
}

__global__ __launch_bounds__(kAcThreads) void ac_hist_kernel(AcArgs a) {
  __shared__ uint32_t sHist[kMaxClusters * kAcTok];
  __shared__ uint8_t sNz[3][1024];
  __shared__ uint8_t sClu[kAcCtx];
  __shared__ uint32_t sBound, sNtok[3];
  const int g = blockIdx.x;
  const GroupGeom G = group_geom(a, g);
  for (int i = threadIdx.x; i < kMaxClusters * kAcTok; i += blockDim.x) sHist[i] = 0;
  for (int i = threadIdx.x; i < kAcCtx; i += blockDim.x) sClu[i] = c_cluster[i];
  if (threadIdx.x < 3) sNtok[threadIdx.x] = 0;
  if (threadIdx.x == 0) sBound = 0;
  fill_nz(a, G, sNz);
  __syncthreads();
  const BlockTask t = block_task(a, G);
  uint32_t bound = 0, nt[3] = {0, 0, 0};
  if (t.valid) {
#pragma unroll 1
    for (int ci = 0; ci < 3; ci++) {
      const int c = channel_of(ci);
      uint32_t cnt = 0;
      block_channel_tokens(a, t, sNz, c, [&](int ctx, uint32_t v) {
        uint32_t tok, nb, bits;
        hybrid420(v, tok, nb, bits);
        atomicAdd(&sHist[sClu[ctx] * kAcTok + tok], 1u);
        bound += 15u + nb;
        cnt++;
      });
      nt[0] += c == 0 ? cnt : 0u;
      nt[1] += c == 1 ? cnt : 0u;
      nt[2] += c == 2 ? cnt : 0u;
    }
  }
  atomicAdd(&sBound, bound);
  atomicAdd(&sNtok[0], nt[0]);
  atomicAdd(&sNtok[1], nt[1]);
  atomicAdd(&sNtok[2], nt[2]);
  __syncthreads();
  for (int i = threadIdx.x; i < kMaxClusters * kAcTok; i += blockDim.x)
    if (sHist[i]) atomicAdd(&a.hist[(i / kAcTok) * kAlpha + (i % kAcTok)], sHist[i]);
  if (threadIdx.x == 0) {
    a.bound[g] = sBound;
    a.ntok[g * 3 + 0] = sNtok[0];
    a.ntok[g * 3 + 1] = sNtok[1];
    a.ntok[g * 3 + 2] = sNtok[2];
  }
}

template <class Sink>
__device__ __forceinline__ void emit_block(const AcArgs& a, const BlockTask& t,
                                           uint8_t (*sNz)[1024], const uint8_t* sClu,
                                           const uint32_t* sCode, Sink& s) {
#pragma unroll 1
  for (int ci = 0; ci < 3; ci++) {
    block_channel_tokens(a, t, sNz, channel_of(ci), [&](int ctx, uint32_t v) {
      uint32_t tok, nb, bits;
      hybrid420(v, tok, nb, bits);
      const uint32_t cl = sCode[sClu[ctx] * kAcTok + tok];
      // code (<= 15 bits) and raw bits (<= 13) in one put
      s.put((cl >> 16) + nb, (cl & 0xFFFFu) | (bits << (cl >> 16)));
    });
  }
  s.finish();
}

__global__ __launch_bounds__(kAcThreads) void ac_emit_kernel(AcArgs a) {
  __shared__ uint32_t sCode[kMaxClusters * kAcTok];
  __shared__ uint32_t sBits[kEmitLdsWords];
  __shared__ uint8_t sNz[3][1024];
  __shared__ uint8_t sClu[kAcCtx];
  __shared__ uint32_t sWave[kAcThreads / 64];
  const int g = blockIdx.x;
  const GroupGeom G = group_geom(a, g);
  for (int i = threadIdx.x; i < kAcCtx; i += blockDim.x) sClu[i] = c_cluster[i];
  for (int i = threadIdx.x; i < kMaxClusters * kAcTok; i += blockDim.x)
    sCode[i] = a.codes[(i / kAcTok) * kAlpha + (i % kAcTok)];
  for (int i = threadIdx.x; i < kEmitLdsWords; i += blockDim.x) sBits[i] = 0;
  fill_nz(a, G, sNz);
  __syncthreads();
  const BlockTask t = block_task(a, G);
  // pass 1: exact bits of this block's three tasks
  uint32_t tot = 0;
  if (t.valid) {
#pragma unroll 1
    for (int ci = 0; ci < 3; ci++) {
      block_channel_tokens(a, t, sNz, channel_of(ci), [&](int ctx, uint32_t v) {
        uint32_t tok, nb, bits;
        hybrid420(v, tok, nb, bits);
        tot += (sCode[sClu[ctx] * kAcTok + tok] >> 16) + nb;
      });
    }
  }
  uint32_t total;
  const uint32_t off = block_excl_scan1024(tot, sWave, &total);
  // pass 2: emission (LDS bit buffer when the group fits, else global atomics)
  const uint64_t base = a.base[g];  // word aligned
  if (total <= (uint32_t)kEmitLdsWords * 32u) {
    if (t.valid) {
      BitSink s{sBits, off, 0, 0};
      emit_block(a, t, sNz, sClu, sCode, s);
    }
    __syncthreads();
    const uint32_t nw = (total + 31) / 32;
    uint32_t* dst = a.scratch + (base >> 5);
    for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) dst[i] = sBits[i];
  } else if (t.valid) {
    BitSink s{a.scratch, base + off, 0, 0};
    emit_block(a, t, sNz, sClu, sCode, s);
  }
  if (threadIdx.x == 0) a.bits[g] = total;
}

void launch_ac_hist(const AcArgs& a, uint32_t ngroups, hipStream_t s) {
  hipLaunchKernelGGL(ac_hist_kernel, dim3(ngroups), dim3(kAcThreads), 0, s, a);
}
void launch_ac_emit(const AcArgs& a, uint32_t ngroups, hipStream_t s) {
  hipLaunchKernelGGL(ac_emit_kernel, dim3(ngroups), dim3(kAcThreads), 0, s, a);
}
void set_cluster_table(const uint8_t* tab, hipStream_t s) {
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(c_cluster), tab, kAcCtx, 0, hipMemcpyHostToDevice, s);
}

}  // namespace jxg
