// jxg_bigvb.hip -- merge levels 128 and 256 px of the AC-strategy search
// (effort >= 8): DCT128X64 / 64X128 / 128X128 / 256X128 / 128X256 / 256X256
// (raw ids 22 / 23 / 21 / 25 / 26 / 24; north_star's "2x2 ... 256x256").
//
// libjxl's e7 search stops at 64x64 squares (ProcessRectACS ->
// FindBestFirstLevelDivisionForSquare(8, ...), proposals/combined.diff:346-353);
// the larger transforms exist in the format and the harness sweeps efforts
// 5..9 (benchmark-jpegxl/src/benchmark.rs:637-642).  This stage runs after
// the 64x64 tile stage (jxg_merge.hip) with the same TryMergeAcs comparison
// (a candidate replaces the current decisions unless `candidate >= current`,
// so NaN estimates are accepted, combined.diff:294 context) and hook F on
// every candidate (combined.diff:247-253).  Float op order == oracle/merge.c
// (jxo_varblock, jxo_llf_dc, jxo_merge_big).
//
// A varblock of up to 256 x 256 coefficients per channel does not fit the
// LDS image the tile kernels use, so the planes live in a per-workgroup
// global scratch slot (persistent workgroups, L2-resident for the 128 level):
//   transform  rows, then columns, in batches through LDS: Lee's recursive
//              DCT evaluated breadth-first (every split stage over all rows
//              of the batch, then every recombination stage) -- the same
//              float ops as the recursion, in another order, so bit-identical;
//   quantize   Y first (its dequantized values replace its coefficients for
//              the X / B residuals), then X, then B transformed into X's
//              plane; item = (16-row chunk, column): fmaf(e, e) over the
//              chunk's rows ascending, the chunk's column partials tree-summed
//              pairwise, chunks in order, dist = (Y + X) + B.
// Kernels: big_eval (one candidate varblock per task), big_resolve (one
// thread per region), big_list (the chosen big varblocks), big_write
// (transform + quantization + coefficients / non-zero counts / quant field /
// LLF-derived DC of every covered block).
#include <float.h>

#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

constexpr int kBT = 1024;      // threads per workgroup
constexpr int kLeeBuf = 2048;  // floats per Lee ping-pong buffer (a batch of rows / columns)

// shape index = level * 3 + {0 tall, 1 wide, 2 full}; level 0 = 128 px, 1 = 256 px
struct BigShape {
  int type, lcy, lcx, kind;
  float tmul;
};
constexpr BigShape kBig[6] = {{22, 4, 3, 0, 1.07f}, {23, 3, 4, 0, 1.07f}, {21, 4, 4, 1, 1.07f},
                              {25, 5, 4, 2, 1.09f}, {26, 4, 5, 2, 1.09f}, {24, 5, 5, 3, 1.09f}};

struct BigLds {
  float buf[2][kLeeBuf];  // Lee ping-pong
  float part[4096];       // quantization: [chunk][column] partials
  float llf[3][32 * 32];  // write: the LLF (cy x cx) of each channel
  float pc[3];
  int bits, nz[3], raw;
};

__device__ __forceinline__ int ilog2i(int n) { return 31 - __clz(n); }

// Lee's DCT-II of `nrows` vectors of N (2..256) held in S.buf[0], breadth-
// first; returns the buffer holding the unnormalized result
__device__ __forceinline__ float* lee_batch(BigLds& S, int nrows, int N, const float* lee_c) {
  const int L = ilog2i(N);
  float* src = S.buf[0];
  float* dst = S.buf[1];
  for (int d = 0; d < L; d++) {  // split: segment n -> (sums | scaled differences)
    const int n = N >> d, h = n >> 1, l = L - d;
    const int half = N >> 1;
    for (int t = threadIdx.x; t < nrows * half; t += kBT) {
      const int row = t / half, i = t - row * half;
      const int seg = i / h, j = i - seg * h;
      const int s0 = row * N + seg * n;
      const float x = src[s0 + j], y = src[s0 + n - 1 - j];
      dst[s0 + j] = x + y;
      dst[s0 + h + j] = (x - y) * lee_c[l * 128 + j];
    }
    __syncthreads();
    float* tt = src;
    src = dst;
    dst = tt;
  }
  for (int d = L - 2; d >= 0; d--) {  // recombine (segments of 2 are already in place)
    const int n = N >> d, h = n >> 1;
    for (int t = threadIdx.x; t < nrows * N; t += kBT) {
      const int row = t / N, o = t - row * N;
      const int seg = o / n, k = o - seg * n;
      const int s0 = row * N + seg * n;
      float out;
      if (!(k & 1)) out = src[s0 + (k >> 1)];
      else if (k < n - 1) out = src[s0 + h + (k >> 1)] + src[s0 + h + (k >> 1) + 1];
      else out = src[s0 + n - 1];
      dst[s0 + k] = out;
    }
    __syncthreads();
    float* tt = src;
    src = dst;
    dst = tt;
  }
  return src;
}

// the candidate's channel ch (0 X, 1 Y, 2 B) from the tile-major XYB copy
// into plane P (R x C, row-major): rows, then columns
__device__ __forceinline__ void vb_transform(const MergeArgs& a, const float* tab, const BigShape& sh, int bx,
                             int by, int ch, float* P, BigLds& S) {
  const int R = 8 << sh.lcy, C = 8 << sh.lcx;
  const float* lee_c = tab + kBigTabLeeC;
  const float* lee_s = tab + kBigTabLeeS;
  const int lR = ilog2i(R), lC = ilog2i(C);
  const int RB = kLeeBuf / C;
  for (int y0 = 0; y0 < R; y0 += RB) {
    for (int e = threadIdx.x; e < RB * C; e += kBT) {
      const int r = e >> lC, x = e & (C - 1);
      const int X = bx * 8 + x, Y = by * 8 + y0 + r;
      const size_t tile = (size_t)(Y >> 6) * a.tiles_x + (X >> 6);
      S.buf[0][e] = a.xyb[tile * (3 * 4096) + ch * 4096 + (Y & 63) * 64 + (X & 63)];
    }
    __syncthreads();
    const float* o = lee_batch(S, RB, C, lee_c);
    for (int e = threadIdx.x; e < RB * C; e += kBT) {
      const int x = e & (C - 1);
      P[(size_t)(y0 + (e >> lC)) * C + x] = o[e] * lee_s[lC * 256 + x];
    }
    __syncthreads();
  }
  const int CB = kLeeBuf / R;
  for (int x0 = 0; x0 < C; x0 += CB) {
    for (int e = threadIdx.x; e < R * CB; e += kBT) {
      const int y = e / CB, j = e - y * CB;
      S.buf[0][j * R + y] = P[(size_t)y * C + x0 + j];
    }
    __syncthreads();
    const float* o = lee_batch(S, CB, R, lee_c);
    for (int e = threadIdx.x; e < R * CB; e += kBT) {
      const int y = e / CB, j = e - y * CB;
      P[(size_t)y * C + x0 + j] = o[j * R + y] * lee_s[lR * 256 + y];
    }
    __syncthreads();
  }
}

// quantization of channel ch of the candidate (jxo_varblock's loop): S.bits,
// S.nz[ch] and S.pc[ch] accumulate; Y's dequantized values replace its
// coefficients in Yp (LLF positions untouched); WRITE: the quantized
// coefficients go to the covered blocks' natural-order slices and the LLF to
// S.llf
template <bool WRITE>
__device__ __forceinline__ void vb_quant(const MergeArgs& a, const float* tab, const uint16_t* natt,
                         const BigShape& sh, int bx, int by, int ch, float* P, const float* Yp,
                         float scale, float kc, BigLds& S) {
  constexpr float kBias1 = 1.0f - 0.07005449891748593f;
  const int R = 8 << sh.lcy, C = 8 << sh.lcx, cy = 1 << sh.lcy, cx = 1 << sh.lcx;
  const int lC = ilog2i(C);
  const int koff = kBigKindOff[sh.kind];
  const float* W = tab + kBigTabW + (size_t)ch * kBigKindOff[4] + koff;
  const float* SD = tab + kBigTabSd + (size_t)ch * kBigKindOff[4] + koff;
  const float* IW = tab + kBigTabIw + koff;
  const uint16_t* NAT = natt + koff;
  const float inv_scale = 1.0f / scale;
  const int nch = R >> 4;
  int bits = 0, nzc = 0;
  const size_t nb = (size_t)a.bxs * a.bys;
  for (int t = threadIdx.x; t < nch * C; t += kBT) {
    const int chunk = t >> lC, x = t & (C - 1);
    float cp = 0.0f;
    for (int ky = chunk * 16; ky < chunk * 16 + 16; ky++) {
      const int si = C >= R ? ky * C + x : x * R + ky;
      float qq_f = 0.0f;
      bool neg = false;
      if (ky < cy && x < cx) {  // LLF: carried by the DC image
        if (WRITE) S.llf[ch][ky * 32 + x] = P[(size_t)ky * C + x];
      } else {
        const float w = W[si];
        float rv = P[(size_t)ky * C + x];
        if (ch != 1) rv = rv - kc * Yp[(size_t)ky * C + x];
        const float v = rv * (w * scale);
        const float av = fabsf(v);
        const float qf = av < 0.58f ? 0.0f : floorf(fminf(av, 32767.0f) + 0.5f);
        const int qa = (int)qf;
        if (ch == 1) {
          float adj = qa == 0 ? 0.0f : (qa == 1 ? kBias1 : qf - 0.145f / qf);
          if (v < 0.0f) adj = -adj;
          P[(size_t)ky * C + x] = adj * (IW[si] * inv_scale);
        }
        const float e = (av - qf) * SD[si];
        cp = fmaf(e, e, cp);
        if (qa) {
          bits += 2 + 2 * (32 - __clz((uint32_t)qa));
          nzc++;
        }
        qq_f = qf;
        neg = v < 0.0f;
      }
      if (WRITE) {
        const int q = neg ? -(int)qq_f : (int)qq_f;
        const int p = NAT[si];
        const int sl = p >> 6;
        const size_t gb = (size_t)(by + (sl >> sh.lcx)) * a.bxs + bx + (sl & (cx - 1));
        a.ac[(gb * 3 + ch) * 64 + (p & 63)] = (int16_t)q;
      }
    }
    S.part[t] = cp;
  }
  (void)nb;
  if (bits) atomicAdd(&S.bits, bits);
  if (nzc) atomicAdd(&S.nz[ch], nzc);
  __syncthreads();
  // a chunk's column partials: pairwise tree over its C columns (tree_sum)
  for (int st = 1; st < C; st <<= 1) {
    const int per = C / (2 * st);
    for (int t = threadIdx.x; t < nch * per; t += kBT) {
      const int chunk = t / per, i = chunk * C + (t - chunk * per) * 2 * st;
      S.part[i] = S.part[i] + S.part[i + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float pc = S.part[0];
    for (int k = 1; k < nch; k++) pc = pc + S.part[k * C];
    S.pc[ch] = pc;
  }
  __syncthreads();
}

// transform + quantization of one candidate (scratch slot: planes Yp, Xp);
// returns the estimate (thread 0's value is the one used)
template <bool WRITE>
__device__ __forceinline__ float vb_eval(const BigArgs& b, const BigShape& sh, int bx, int by, BigLds& S,
                         float* Yp, float* Xp) {
  const MergeArgs& a = b.m;
  const int cy = 1 << sh.lcy, cx = 1 << sh.lcx;
  if (threadIdx.x == 0) {
    S.bits = 0;
    S.nz[0] = S.nz[1] = S.nz[2] = 0;
    S.raw = 0;
  }
  __syncthreads();
  // quant field of the varblock: the max raw of its covered blocks
  int r = 0;
  for (int i = threadIdx.x; i < cy * cx; i += kBT)
    r = max(r, (int)a.qf[(size_t)(by + (i >> sh.lcx)) * a.bxs + bx + (i & (cx - 1))] + 1);
  if (r) atomicMax(&S.raw, r);
  __syncthreads();
  const float scale = (float)a.G * (float)S.raw / 65536.0f;
  // chroma from luma of the top-left block's tile (as the decoder applies it)
  const size_t tile = (size_t)(by >> 3) * a.tiles_x + (bx >> 3);
  const float kx = (float)a.cmap[tile] * (1.0f / 84.0f);
  const float kb = 1.0f + (float)a.cmap[a.ntiles_all + tile] * (1.0f / 84.0f);
  vb_transform(a, b.tab, sh, bx, by, 1, Yp, S);
  vb_quant<WRITE>(a, b.tab, b.nat, sh, bx, by, 1, Yp, Yp, scale, 0.0f, S);
  vb_transform(a, b.tab, sh, bx, by, 0, Xp, S);
  vb_quant<WRITE>(a, b.tab, b.nat, sh, bx, by, 0, Xp, Yp, scale, kx, S);
  vb_transform(a, b.tab, sh, bx, by, 2, Xp, S);
  vb_quant<WRITE>(a, b.tab, b.nat, sh, bx, by, 2, Xp, Yp, scale, kb, S);
  const float dist = (S.pc[1] + S.pc[0]) + S.pc[2];
  const int tb = S.bits + (32 - __clz((uint32_t)S.nz[0])) + (32 - __clz((uint32_t)S.nz[1])) +
                 (32 - __clz((uint32_t)S.nz[2]));
  float e = ((float)tb + 8.0f * dist) * sh.tmul;
  if (a.proposals & 2u) {
    const size_t gb = (size_t)by * a.bxs + bx;
    e = hook_f(e, a.homog[gb * 3], a.homog[gb * 3 + 1], a.homog[gb * 3 + 2]);
  }
  return e;
}

// region r of level L (0: 128 px, 1: 256 px) of group slot gi: origin (blocks)
__device__ __forceinline__ bool big_region(const BigArgs& b, int L, uint32_t gi, int r, int& bx0,
                                           int& by0) {
  const uint32_t g = b.glist ? b.glist[gi] : b.g0 + gi;
  const int gx = (int)(g % b.gxs), gy = (int)(g / b.gxs), s = 16 << L;
  bx0 = gx * 32 + (L == 0 ? (r & 1) * 16 : 0);
  by0 = gy * 32 + (L == 0 ? (r >> 1) * 16 : 0);
  return bx0 + s <= (int)b.m.bxs && by0 + s <= (int)b.m.bys;
}
// candidate j of a region: 0 full, 1 / 2 tall halves (left / right), 3 / 4
// wide halves (top / bottom)
__device__ __forceinline__ const BigShape& big_cand(int L, int j, int bx0, int by0, int& bx,
                                                    int& by) {
  const int s = 16 << L;
  bx = bx0 + (j == 2 ? s / 2 : 0);
  by = by0 + (j == 4 ? s / 2 : 0);
  return kBig[L * 3 + (j == 0 ? 2 : (j <= 2 ? 0 : 1))];
}
constexpr int kBigCost = 25;  // per group slot: level 128 (4 regions x 5), level 256 (5)

__global__ __launch_bounds__(kBT) void big_eval_kernel(Batch<BigArgs> bt_, int L) {
  const BigArgs& b = bt_.a[blockIdx.z];
  __shared__ BigLds S;
  if (L == 0 && blockIdx.x == 0 && threadIdx.x == 0) b.work[0] = 0;  // big_list's count
  const int nreg = L == 0 ? 4 : 1;
  const uint32_t total = b.ng * (uint32_t)nreg * 5u;
  float* Yp = b.scratch + (size_t)blockIdx.x * 2 * 65536;
  float* Xp = Yp + 65536;
  for (uint32_t w = blockIdx.x; w < total; w += gridDim.x) {
    const uint32_t gi = w / (nreg * 5), rem = w - gi * (nreg * 5);
    const int r = (int)rem / 5, j = (int)rem % 5;
    int bx0, by0;
    if (!big_region(b, L, gi, r, bx0, by0)) continue;  // (uniform)
    int bx, by;
    const BigShape& sh = big_cand(L, j, bx0, by0, bx, by);
    const float e = vb_eval<false>(b, sh, bx, by, S, Yp, Xp);
    if (threadIdx.x == 0) b.cost[(size_t)gi * kBigCost + (L == 0 ? r * 5 + j : 20 + j)] = e;
    __syncthreads();
  }
}

// one thread per region: the TryMergeAcs comparison against the decisions of
// the levels below (ent: each varblock's estimate at its first block, 0 at
// covered blocks; summed in raster order), then the chosen varblocks' blocks
__global__ __launch_bounds__(256) void big_resolve_kernel(Batch<BigArgs> bt_, int L) {
  const BigArgs& b = bt_.a[blockIdx.z];
  const MergeArgs& a = b.m;
  const int nreg = L == 0 ? 4 : 1, s = 16 << L;
  const uint32_t idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= b.ng * (uint32_t)nreg) return;
  const uint32_t gi = idx / nreg;
  const int r = (int)(idx - gi * nreg);
  int bx0, by0;
  if (!big_region(b, L, gi, r, bx0, by0)) return;
  float cur = 0.0f;
  for (int iy = 0; iy < s; iy++)
    for (int ix = 0; ix < s; ix++) cur += a.ent[(size_t)(by0 + iy) * a.bxs + bx0 + ix];
  const float* cost = b.cost + (size_t)gi * kBigCost + (L == 0 ? r * 5 : 20);
  const float e0 = cost[0], et = cost[1] + cost[2], ew = cost[3] + cost[4];
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
  if (!choice) return;
  const int first = choice == 1 ? 0 : (choice == 2 ? 1 : 3), nv = choice == 1 ? 1 : 2;
  for (int j = first; j < first + nv; j++) {
    int bx, by;
    const BigShape& sh = big_cand(L, j, bx0, by0, bx, by);
    for (int iy = 0; iy < (1 << sh.lcy); iy++)
      for (int ix = 0; ix < (1 << sh.lcx); ix++) {
        const size_t gb = (size_t)(by + iy) * a.bxs + bx + ix;
        a.acs[gb] = (uint8_t)(sh.type | ((iy | ix) ? 0x80 : 0));
        a.ent[gb] = (iy | ix) ? 0.0f : cost[j];
      }
  }
}

// the chosen big varblocks (first blocks on the 64-px grid of each group)
__global__ __launch_bounds__(64) void big_list_kernel(Batch<BigArgs> bt_) {
  const BigArgs& b = bt_.a[blockIdx.z];
  const MergeArgs& a = b.m;
  const uint32_t gi = blockIdx.x;
  if (gi >= b.ng || threadIdx.x >= 16) return;
  const uint32_t g = b.glist ? b.glist[gi] : b.g0 + gi;
  const uint32_t bx = (g % b.gxs) * 32 + (threadIdx.x & 3) * 8;
  const uint32_t by = (g / b.gxs) * 32 + (threadIdx.x >> 2) * 8;
  if (bx >= a.bxs || by >= a.bys) return;
  const uint32_t gb = by * a.bxs + bx;
  const uint8_t t = a.acs[gb];
  if (t >= 21 && t <= 26) b.work[1 + atomicAdd(b.work, 1u)] = gb;
}

__global__ __launch_bounds__(kBT) void big_write_kernel(Batch<BigArgs> bt_) {
  const BigArgs& b = bt_.a[blockIdx.z];
  const MergeArgs& a = b.m;
  __shared__ BigLds S;
  float* Yp = b.scratch + (size_t)blockIdx.x * 2 * 65536;
  float* Xp = Yp + 65536;
  const uint32_t n = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)b.work);
  const size_t nb = (size_t)a.bxs * a.bys;
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
    const uint32_t gb0 = b.work[1 + w];
    const int bx = (int)(gb0 % a.bxs), by = (int)(gb0 / a.bxs);
    const uint8_t t = a.acs[gb0];
    int si = 0;
    for (int i = 0; i < 6; i++) si = kBig[i].type == t ? i : si;
    const BigShape& sh = kBig[si];
    (void)vb_eval<true>(b, sh, bx, by, S, Yp, Xp);
    // per covered block: non-zero counts, quant field, DC from the LLF
    const int lcy = sh.lcy, lcx = sh.lcx, cy = 1 << lcy, cx = 1 << lcx, lcb = lcy + lcx;
    const float* llf_p = b.tab + kBigTabLlfP;
    const float* llf_ib = b.tab + kBigTabLlfIb;
    for (int k = threadIdx.x; k < cy * cx; k += kBT) {
      const int iy = k >> lcx, ix = k & (cx - 1);
      const size_t gb = (size_t)(by + iy) * a.bxs + bx + ix;
      for (int c = 0; c < 3; c++) {
        const int nzv = S.nz[c];
        a.nz[c * nb + gb] = (uint16_t)(k == 0 ? nzv : (nzv + (1 << lcb) - 1) >> lcb);
      }
      float dc[3];
      for (int c = 0; c < 3; c++) {
        float acc = 0.0f;
        for (int ky = 0; ky < cy; ky++) {
          float u = 0.0f;
          for (int kx = 0; kx < cx; kx++) {
            const float tt = (S.llf[c][ky * 32 + kx] * llf_p[lcy * 32 + ky]) * llf_p[lcx * 32 + kx];
            u = fmaf(tt, llf_ib[(lcx * 32 + ix) * 32 + kx], u);
          }
          acc = fmaf(u, llf_ib[(lcy * 32 + iy) * 32 + ky], acc);
        }
        dc[c] = acc;
      }
      int32_t q[3];
      quant_dc3(dc, a.dc_mul, a.dc_step, q);
      a.dc[gb] = q[0];
      a.dc[nb + gb] = q[1];
      a.dc[2 * nb + gb] = q[2];
      a.qf[gb] = (uint8_t)(S.raw - 1);
    }
    __syncthreads();
  }
}

// levels 128 and 256 of k frames (same plan): eval / resolve per level, then
// the chosen varblocks' write pass
hipError_t launch_big(const BigArgs* a, uint32_t k, hipStream_t s) {
  if (!k || !a[0].ng) return hipSuccess;
  const Batch<BigArgs> bt = make_batch(a, k);
  const uint32_t ng = a[0].ng;
  for (int L = 0; L < 2; L++) {
    const uint32_t tasks = ng * (L == 0 ? 20u : 5u);
    hipLaunchKernelGGL(big_eval_kernel, dim3(min(tasks, a[0].slots), 1, k), dim3(kBT), 0, s, bt, L);
    const uint32_t nreg = ng * (L == 0 ? 4u : 1u);
    hipLaunchKernelGGL(big_resolve_kernel, dim3((nreg + 255) / 256, 1, k), dim3(256), 0, s, bt, L);
  }
  hipLaunchKernelGGL(big_list_kernel, dim3(ng, 1, k), dim3(64), 0, s, bt);
  hipLaunchKernelGGL(big_write_kernel, dim3(min(ng * 16u, a[0].slots), 1, k), dim3(kBT), 0, s, bt);
  return hipGetLastError();
}

}  // namespace jxg
