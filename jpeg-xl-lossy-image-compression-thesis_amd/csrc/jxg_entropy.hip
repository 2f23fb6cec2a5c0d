// jxg_entropy.hip -- token statistics and bit emission on gfx950.
//
// (pass-group AC kernels: jxg_ac.hip)
// LF groups (modular streams of quantized DC and AC metadata) are processed
// one row per workgroup: lf_hist -> lf_rowbits -> lf_scan -> lf_emit.
// concat  : bit-exact assembly of all sections (device scratch + host chunks)
//           into the final codestream, one word per lane.
// Token order, contexts and hybrid-uint split are those of oracle/encode.c
// (group_tokens, put_modular) -- [ext] JPEG XL AC/modular coding.
#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

// ----------------------------- LF groups -----------------------------------
struct LfGeom {
  uint32_t bx0, by0, bw, bh;
};
__device__ __forceinline__ LfGeom lf_geom(const LfArgs& a, uint32_t lg) {
  LfGeom r;
  r.bx0 = (lg % a.lfxs) * 256;
  r.by0 = (lg / a.lfxs) * 256;
  r.bw = min(256u, a.bxs - r.bx0);
  r.bh = min(256u, a.bys - r.by0);
  return r;
}

__device__ __forceinline__ int32_t lf_value(const LfArgs& a, const LfRow& r, const LfGeom& L,
                                            int x, int y) {
  const size_t nb = (size_t)a.bxs * a.bys;
  if (r.stream == 0) {
    const int c = r.chan == 0 ? 1 : (r.chan == 1 ? 0 : 2);
    return a.dc[c * nb + (size_t)(L.by0 + y) * a.bxs + L.bx0 + x];
  }
  if (r.chan != 2) return 0;
  const uint32_t bx = (uint32_t)x % L.bw, by = (uint32_t)x / L.bw;
  const size_t b = (size_t)(L.by0 + by) * a.bxs + L.bx0 + bx;
  return y == 0 ? (int32_t)a.acs[b] : (int32_t)a.qf[b];
}

// residual and leaf of sample (x, row.y)
__device__ __forceinline__ void lf_residual(const LfArgs& a, const LfRow& r, const LfGeom& L,
                                            int x, uint32_t& u, int& leaf) {
  const int y = (int)r.y;
  const int32_t v = lf_value(a, r, L, x, y);
  int32_t pred = 0;
  if (r.stream == 0) {
    leaf = r.chan == 0 ? 0 : (r.chan == 2 ? 1 : 2);
    const int32_t W = x > 0 ? lf_value(a, r, L, x - 1, y) : (y > 0 ? lf_value(a, r, L, x, y - 1) : 0);
    const int32_t N = y > 0 ? lf_value(a, r, L, x, y - 1) : W;
    const int32_t NW = (x > 0 && y > 0) ? lf_value(a, r, L, x - 1, y - 1) : W;
    const int32_t gr = W + N - NW;
    const int32_t lo = W < N ? W : N, hi = W < N ? N : W;
    pred = gr < lo ? lo : (gr > hi ? hi : gr);
  } else {
    if (r.chan <= 1) {
      leaf = 0;
    } else if (r.chan == 3) {
      leaf = 1;
    } else if (y > 0) {
      leaf = 2;
      pred = x > 0 ? lf_value(a, r, L, x - 1, y) : lf_value(a, r, L, x, y - 1);
    } else {
      leaf = 3;
    }
  }
  u = pack_signed(v - pred);
}

__global__ __launch_bounds__(256) void lf_hist_kernel(LfArgs a) {
  __shared__ uint32_t sHist[4 * kAlpha];
  __shared__ uint32_t sBound;
  const LfRow r = a.rows[blockIdx.x];
  const LfGeom L = lf_geom(a, r.lg);
  for (int i = threadIdx.x; i < 4 * kAlpha; i += blockDim.x) sHist[i] = 0;
  if (threadIdx.x == 0) sBound = 0;
  __syncthreads();
  uint32_t bound = 0;
  for (uint32_t i = threadIdx.x; i < r.width; i += blockDim.x) {
    uint32_t u, tok, nb, bits;
    int leaf;
    lf_residual(a, r, L, (int)(r.x0 + i), u, leaf);
    hybrid420(u, tok, nb, bits);
    atomicAdd(&sHist[leaf * kAlpha + tok], 1u);
    bound += 15u + nb;
  }
  atomicAdd(&sBound, bound);
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * kAlpha; i += blockDim.x)
    if (sHist[i]) atomicAdd(&a.hist[(size_t)r.sid * 4 * kAlpha + i], sHist[i]);
  if (threadIdx.x == 0) atomicAdd(&a.sbound[r.sid], sBound);
}

__device__ __forceinline__ uint32_t lf_sample_bits(const LfArgs& a, const LfRow& r,
                                                   const LfGeom& L, int x, uint32_t& code,
                                                   uint32_t& clen, uint32_t& nb,
                                                   uint32_t& bits) {
  uint32_t u, tok;
  int leaf;
  lf_residual(a, r, L, x, u, leaf);
  hybrid420(u, tok, nb, bits);
  const uint32_t cl = a.codes[((size_t)r.sid * 4 + leaf) * kAlpha + tok];
  code = cl & 0xFFFFu;
  clen = cl >> 16;
  return clen + nb;
}

__global__ __launch_bounds__(256) void lf_rowbits_kernel(LfArgs a) {
  __shared__ uint32_t sSum;
  const LfRow r = a.rows[blockIdx.x];
  const LfGeom L = lf_geom(a, r.lg);
  if (threadIdx.x == 0) sSum = 0;
  __syncthreads();
  uint32_t s = 0;
  for (uint32_t i = threadIdx.x; i < r.width; i += blockDim.x) {
    uint32_t code, clen, nb, bits;
    s += lf_sample_bits(a, r, L, (int)(r.x0 + i), code, clen, nb, bits);
  }
  atomicAdd(&sSum, s);
  __syncthreads();
  if (threadIdx.x == 0) a.row_bits[blockIdx.x] = sSum;
}

// per-stream exclusive scan of row bits -> absolute row offsets
__global__ __launch_bounds__(256) void lf_scan_kernel(LfArgs a) {
  __shared__ uint32_t sScan[256];
  const uint32_t sid = blockIdx.x;
  const uint32_t r0 = a.stream_rows[sid], r1 = a.stream_rows[sid + 1];
  uint64_t run = a.stream_base[sid];
  const uint64_t start = run;
  for (uint32_t c0 = r0; c0 < r1; c0 += blockDim.x) {
    const uint32_t r = c0 + threadIdx.x;
    const uint32_t v = r < r1 ? a.row_bits[r] : 0;
    sScan[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
      uint32_t t = threadIdx.x >= (uint32_t)d ? sScan[threadIdx.x - d] : 0;
      __syncthreads();
      sScan[threadIdx.x] += t;
      __syncthreads();
    }
    if (r < r1) a.row_off[r] = run + sScan[threadIdx.x] - v;
    run += sScan[255];
    __syncthreads();
  }
  if (threadIdx.x == 0) a.stream_bits[sid] = (uint32_t)(run - start);
}

__global__ __launch_bounds__(256) void lf_emit_kernel(LfArgs a) {
  __shared__ uint32_t sScan[256];
  const LfRow r = a.rows[blockIdx.x];
  const LfGeom L = lf_geom(a, r.lg);
  uint64_t run = a.row_off[blockIdx.x];
  for (uint32_t x0 = 0; x0 < r.width; x0 += blockDim.x) {
    const uint32_t x = x0 + threadIdx.x;
    uint32_t code = 0, clen = 0, nb = 0, bits = 0, tot = 0;
    if (x < r.width) tot = lf_sample_bits(a, r, L, (int)(r.x0 + x), code, clen, nb, bits);
    sScan[threadIdx.x] = tot;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
      uint32_t v = threadIdx.x >= (uint32_t)d ? sScan[threadIdx.x - d] : 0;
      __syncthreads();
      sScan[threadIdx.x] += v;
      __syncthreads();
    }
    if (x < r.width) {
      BitSink s{a.scratch, run + sScan[threadIdx.x] - tot, 0, 0};
      s.put(clen, code);
      s.put(nb, bits);
      s.finish();
    }
    run += sScan[255];
    __syncthreads();
  }
}

// ------------------------------- concat ------------------------------------
__device__ __forceinline__ uint32_t read_bits32(const uint32_t* src, uint64_t bit) {
  const uint64_t w = bit >> 5;
  const int sh = (int)(bit & 31);
  uint32_t lo = src[w] >> sh;
  if (sh) lo |= src[w + 1] << (32 - sh);
  return lo;
}

__global__ __launch_bounds__(256) void concat_kernel(const ConcatPiece* pieces,
                                                     const uint32_t* scratch,
                                                     const uint32_t* chunks, uint32_t* out) {
  const ConcatPiece p = pieces[blockIdx.y];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i * 32 >= p.nbits) return;
  const uint32_t* src = p.arena ? chunks : scratch;
  const uint64_t nb = p.nbits - i * 32 < 32 ? p.nbits - i * 32 : 32;
  uint32_t v = read_bits32(src, p.src_bit + i * 32);
  if (nb < 32) v &= (1u << nb) - 1u;
  const uint64_t d = p.dst_bit + i * 32;
  const uint64_t w = d >> 5;
  const int sh = (int)(d & 31);
  if (v == 0) return;
  atomicOr(&out[w], v << sh);
  if (sh && (uint64_t)sh + nb > 32) atomicOr(&out[w + 1], v >> (32 - sh));
}

// ------------------------------- launchers ---------------------------------
void launch_lf_hist(const LfArgs& a, uint32_t nrows, hipStream_t s) {
  hipLaunchKernelGGL(lf_hist_kernel, dim3(nrows), dim3(256), 0, s, a);
}
void launch_lf_rowbits(const LfArgs& a, uint32_t nrows, hipStream_t s) {
  hipLaunchKernelGGL(lf_rowbits_kernel, dim3(nrows), dim3(256), 0, s, a);
}
void launch_lf_scan(const LfArgs& a, uint32_t nstreams, hipStream_t s) {
  hipLaunchKernelGGL(lf_scan_kernel, dim3(nstreams), dim3(256), 0, s, a);
}
void launch_lf_emit(const LfArgs& a, uint32_t nrows, hipStream_t s) {
  hipLaunchKernelGGL(lf_emit_kernel, dim3(nrows), dim3(256), 0, s, a);
}
void launch_concat(const ConcatPiece* pieces, uint32_t npieces, uint64_t max_words,
                   const uint32_t* scratch, const uint32_t* chunks, uint32_t* out,
                   hipStream_t s) {
  if (npieces == 0 || max_words == 0) return;
  const uint32_t gx = (uint32_t)((max_words + 255) / 256);
  hipLaunchKernelGGL(concat_kernel, dim3(gx, npieces), dim3(256), 0, s, pieces, scratch,
                     chunks, out);
}


}  // namespace jxg
