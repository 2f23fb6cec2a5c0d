// jxg_ac.hip -- pass-group AC token statistics and bit emission on gfx950.
//
// One 1024-thread workgroup per 256x256-pixel pass group (32x32 blocks, 3072
// (block, channel) tasks, 3 per thread).  A task's 64 int16 coefficients
// (128 B) are loaded with 8 x 16-byte loads into 32 VGPRs and the token walk
// runs on registers (fully unrolled, wave-uniform early exit every 8
// coefficients), so there are no dependent global loads in the walk.
//   ac_hist : non-zero counts -> predicted-nz + zero-density contexts ->
//             clustered histograms (LDS, one global atomic per non-empty bin),
//             exact per-group token counts, per-group bit upper bound.
//   ac_emit : same walk with the prefix codes: per-task bit lengths ->
//             workgroup exclusive scan (stream order: blocks raster, channels
//             Y, X, B) -> every task writes its bits with atomicOr.
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

// task t (stream order) -> (block x, block y, channel)
struct Task {
  int bx, by, c;
  size_t gb;
};
__device__ __forceinline__ Task task_of(const AcArgs& a, const GroupGeom& G, int t) {
  Task k;
  const int b = t / 3, ci = t - b * 3;
  k.c = ci == 0 ? 1 : (ci == 1 ? 0 : 2);
  k.bx = b % G.gw;
  k.by = b / G.gw;
  k.gb = (size_t)(G.by0 + k.by) * a.bxs + G.bx0 + k.bx;
  return k;
}

// non-zero counts of the group's blocks (written by the front kernel)
__device__ void fill_nz(const AcArgs& a, const GroupGeom& G, uint8_t (*sNz)[1024]) {
  const size_t nb = (size_t)a.bxs * a.bys;
  for (int i = threadIdx.x; i < 3 * 1024; i += blockDim.x) {
    const int c = i >> 10, by = (i >> 5) & 31, bx = i & 31;
    if (bx < G.gw && by < G.gh)
      sNz[c][by * 32 + bx] = a.nz[c * nb + (size_t)(G.by0 + by) * a.bxs + G.bx0 + bx];
  }
}

__global__ __launch_bounds__(kAcThreads) void ac_hist_kernel(AcArgs a) {
  __shared__ uint32_t sHist[kMaxClusters * kAlpha];
  __shared__ uint8_t sNz[3][1024];
  __shared__ uint8_t sClu[kAcCtx];
  __shared__ uint32_t sBound, sNtok[3];
  const int g = blockIdx.x;
  const GroupGeom G = group_geom(a, g);
  for (int i = threadIdx.x; i < kMaxClusters * kAlpha; i += blockDim.x) sHist[i] = 0;
  for (int i = threadIdx.x; i < kAcCtx; i += blockDim.x) sClu[i] = c_cluster[i];
  if (threadIdx.x < 3) sNtok[threadIdx.x] = 0;
  if (threadIdx.x == 0) sBound = 0;
  fill_nz(a, G, sNz);
  __syncthreads();
  const int ntask = G.gw * G.gh * 3;
  uint32_t bound = 0, nt[3] = {0, 0, 0};
  for (int t = threadIdx.x; t < ntask; t += blockDim.x) {
    const Task k = task_of(a, G, t);
    uint32_t w[32];
    load_coefs(a.ac + (k.gb * 3 + k.c) * 64, w);
    const int nz = sNz[k.c][k.by * 32 + k.bx];
    uint32_t cnt = 0;
    block_tokens(w, nz, predict_nz(sNz[k.c], k.bx, k.by), block_ctx_of(k.c, a.acs[k.gb]),
                 [&](int ctx, uint32_t v) {
                   uint32_t tok, nb, bits;
                   hybrid420(v, tok, nb, bits);
                   atomicAdd(&sHist[sClu[ctx] * kAlpha + tok], 1u);
                   bound += 15u + nb;
                   cnt++;
                 });
    nt[k.c] += cnt;
  }
  atomicAdd(&sBound, bound);
  atomicAdd(&sNtok[0], nt[0]);
  atomicAdd(&sNtok[1], nt[1]);
  atomicAdd(&sNtok[2], nt[2]);
  __syncthreads();
  for (int i = threadIdx.x; i < kMaxClusters * kAlpha; i += blockDim.x)
    if (sHist[i]) atomicAdd(&a.hist[i], sHist[i]);
  if (threadIdx.x == 0) {
    a.bound[g] = sBound;
    a.ntok[g * 3 + 0] = sNtok[0];
    a.ntok[g * 3 + 1] = sNtok[1];
    a.ntok[g * 3 + 2] = sNtok[2];
  }
}

__global__ __launch_bounds__(kAcThreads) void ac_emit_kernel(AcArgs a) {
  __shared__ uint8_t sNz[3][1024];
  __shared__ uint8_t sClu[kAcCtx];
  __shared__ uint32_t sOff[3 * 1024];
  __shared__ uint32_t sScan[kAcThreads];
  const int g = blockIdx.x;
  const GroupGeom G = group_geom(a, g);
  for (int i = threadIdx.x; i < kAcCtx; i += blockDim.x) sClu[i] = c_cluster[i];
  fill_nz(a, G, sNz);
  __syncthreads();
  const int ntask = G.gw * G.gh * 3;
  // pass 1: bits per task
  for (int t = threadIdx.x; t < ntask; t += blockDim.x) {
    const Task k = task_of(a, G, t);
    uint32_t w[32];
    load_coefs(a.ac + (k.gb * 3 + k.c) * 64, w);
    uint32_t bits_t = 0;
    block_tokens(w, sNz[k.c][k.by * 32 + k.bx], predict_nz(sNz[k.c], k.bx, k.by),
                 block_ctx_of(k.c, a.acs[k.gb]), [&](int ctx, uint32_t v) {
                   uint32_t tok, nb, bits;
                   hybrid420(v, tok, nb, bits);
                   bits_t += (a.codes[sClu[ctx] * kAlpha + tok] >> 16) + nb;
                 });
    sOff[t] = bits_t;
  }
  __syncthreads();
  // exclusive scan over tasks in stream order: thread i owns [i*per, (i+1)*per)
  const int per = (ntask + kAcThreads - 1) / kAcThreads;
  const int t0 = threadIdx.x * per;
  uint32_t local = 0;
  for (int t = t0; t < t0 + per && t < ntask; t++) local += sOff[t];
  sScan[threadIdx.x] = local;
  __syncthreads();
  for (int d = 1; d < kAcThreads; d <<= 1) {
    uint32_t v = threadIdx.x >= (unsigned)d ? sScan[threadIdx.x - d] : 0;
    __syncthreads();
    sScan[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = sScan[threadIdx.x] - local;
  for (int t = t0; t < t0 + per && t < ntask; t++) {
    const uint32_t v = sOff[t];
    sOff[t] = run;
    run += v;
  }
  __syncthreads();
  const uint64_t base = a.base[g];
  for (int t = threadIdx.x; t < ntask; t += blockDim.x) {
    const Task k = task_of(a, G, t);
    uint32_t w[32];
    load_coefs(a.ac + (k.gb * 3 + k.c) * 64, w);
    BitSink s{a.scratch, base + sOff[t], 0, 0};
    block_tokens(w, sNz[k.c][k.by * 32 + k.bx], predict_nz(sNz[k.c], k.bx, k.by),
                 block_ctx_of(k.c, a.acs[k.gb]), [&](int ctx, uint32_t v) {
                   uint32_t tok, nb, bits;
                   hybrid420(v, tok, nb, bits);
                   const uint32_t cl = a.codes[sClu[ctx] * kAlpha + tok];
                   // code (<= 15 bits) and raw bits (<= 15) in one put
                   s.put((cl >> 16) + nb, (cl & 0xFFFFu) | (bits << (cl >> 16)));
                 });
    s.finish();
  }
  if (threadIdx.x == kAcThreads - 1) a.bits[g] = sScan[kAcThreads - 1];
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
