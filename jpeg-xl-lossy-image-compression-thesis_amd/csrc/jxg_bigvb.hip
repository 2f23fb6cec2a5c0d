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
// global scratch slot (512 persistent workgroups, three column-major planes):
//   transform  Y first, then X and B: rows from the tile-major XYB copy, then
//              columns in place, one 32-point Lee DCT per lane in registers
//              (a vector of 64 / 128 / 256 points over 2 / 4 / 8 adjacent
//              lanes: the first splits evaluated from the elements, the upper
//              recombinations by lane shuffles) -- the recursion's float ops;
//   quantize   Y (its dequantized values replace its coefficients for the X
//              / B residuals), then X and B; item = (16-row chunk, column):
//              fmaf(e, e) over the chunk's rows ascending, the chunk's column
//              partials tree-summed pairwise, chunks in order,
//              dist = (Y + X) + B;
//   prune      a candidate whose estimate after Y alone reaches its region's
//              current sum cannot be chosen (exact: every later term only
//              adds), so its X / B half is skipped and it reads +inf.
// Kernels: big_cur (each region's current sum), big_eval (one candidate
// varblock per task), big_resolve (one thread per region), big_list (the
// chosen big varblocks), big_write (transform + quantization + coefficients /
// non-zero counts / quant field / LLF-derived DC of every covered block).
#include <float.h>

#include "jxg_device.h"
#include "jxg_kernels.h"
#include "jxg_lee_tables.h"

namespace jxg {

constexpr int kBT = 512;  // threads per workgroup (two per CU)

// shape index = level * 3 + {0 tall, 1 wide, 2 full}; level 0 = 128 px, 1 = 256 px
struct BigShape {
  int type, lcy, lcx, kind;
  float tmul;
};
constexpr BigShape kBig[6] = {{22, 4, 3, 0, 1.07f}, {23, 3, 4, 0, 1.07f}, {21, 4, 4, 1, 1.07f},
                              {25, 5, 4, 2, 1.09f}, {26, 4, 5, 2, 1.09f}, {24, 5, 5, 3, 1.09f}};

struct BigLds {
  float part[4096];       // quantization: [chunk][column] partials
  float llf[3][32 * 32];  // write: the LLF (cy x cx) of each channel
  float lee_c[9 * 128];   // the Lee tables (kBigTabLeeC / kBigTabLeeS), copied once per workgroup
  float lee_s[9 * 256];
  float pc[3];
  int bits, nz[3], raw;
};

__device__ __forceinline__ int ilog2i(int n) { return 31 - __clz(n); }

// unnormalized DCT-II in registers, Lee's recursive even/odd split (== the
// oracle's lee; constants of jxg_lee_tables.h)
template <int N>
__device__ __forceinline__ void lee_reg(float* x) {
  if constexpr (N > 1) {
    constexpr int h = N / 2, l = N == 2 ? 1 : (N == 4 ? 2 : (N == 8 ? 3 : (N == 16 ? 4 : (N == 32 ? 5 : 6))));
    float a[h], b[h];
#pragma unroll
    for (int i = 0; i < h; i++) {
      a[i] = x[i] + x[N - 1 - i];
      b[i] = (x[i] - x[N - 1 - i]) * kLeeC[l][i];
    }
    lee_reg<h>(a);
    lee_reg<h>(b);
#pragma unroll
    for (int k = 0; k < h; k++) x[2 * k] = a[k];
#pragma unroll
    for (int k = 0; k < h - 1; k++) x[2 * k + 1] = b[k] + b[k + 1];
    x[N - 1] = b[h - 1];
  }
}

// One N-point transform (N = 64, 128, 256) of a vector, element p = ld(p),
// spread over NP = N / 32 adjacent lanes (D = log2 NP split levels).  Lane
// r of the group (bit d - 1 of r: s_d, the branch taken at split level d,
// 0 the sums, 1 the scaled differences) evaluates its 32-point sub-vector
// v_D[j] straight from the elements (each node u0 + u1 or (u0 - u1) c, the
// recursion's float ops), runs Lee's 32-point DCT in registers, then the
// recombinations upward: at the 64-point level the lane alone (odd outputs
// b[k] + b[k + 1]); at the higher levels the b-child's values are spread
// over the lanes r + 2^d (same k) and, for the last of them, r - 2^d rho_max
// (k + 1): DPP-free shuffles (ds_bpermute).  Output k of lane r lands at
// position k NP + r.
template <int NN, int d, class Ld>
__device__ __forceinline__ float vb_node(Ld ld, int i, int r, const BigLds& S) {
  // v_d[i] of the sub-vector chosen by the low d bits of r (v_0 = x)
  if constexpr (d == 0) {
    return ld(i);
  } else {
    constexpr int n = NN >> (d - 1), l = n == 64 ? 6 : (n == 128 ? 7 : 8);
    const float u0 = vb_node<NN, d - 1>(ld, i, r, S), u1 = vb_node<NN, d - 1>(ld, n - 1 - i, r, S);
    const float c = l == 6 ? kLeeC[6][i] : S.lee_c[l * 128 + i];
    return ((r >> (d - 1)) & 1) ? (u0 - u1) * c : u0 + u1;
  }
}
template <int N, class Ld>
__device__ __forceinline__ void vb_vec(Ld ld, int r, float* o, const BigLds& S) {
  constexpr int NP = N / 32, D = NP == 2 ? 1 : (NP == 4 ? 2 : 3);
#pragma unroll
  for (int j = 0; j < 32; j++) {
    o[j] = vb_node<N, D>(ld, j, r, S);
    // (the scheduler keeps at most four vectors' leaves in flight: hoisting
    // all 32 x NP leaf loads would spill)
    if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  }
  lee_reg<32>(o);
  // level D (64 points of v_{D-1}): the b-lanes' odd outputs, in-lane
  const bool bD = (r >> (D - 1)) & 1;
#pragma unroll
  for (int k = 0; k < 31; k++) o[k] = bD ? o[k] + o[k + 1] : o[k];
  // levels D - 1 .. 1: the b-child spread over 2^(D - d) lanes
#pragma unroll
  for (int d = D - 1; d >= 1; d--) {
    const int lane = (int)(threadIdx.x & 63);
    const int rho = r >> d, rmax = (1 << (D - d)) - 1;
    const int src_same = lane + (1 << d);                 // rho + 1, same k
    const int src_next = lane - (rho << d);               // rho 0, k + 1
    const bool bl = (r >> (d - 1)) & 1;
#pragma unroll
    for (int k = 0; k < 32; k++) {
      const float qs = __shfl(o[k], rho < rmax ? src_same : lane, 64);
      const float qn = __shfl(o[k < 31 ? k + 1 : 31], src_next, 64);
      // (selects, no branches: the last value of the last lane stays alone)
      const float sum = o[k] + (rho < rmax ? qs : qn);
      o[k] = bl && (rho < rmax || k < 31) ? sum : o[k];
    }
  }
}

// item i of a pass over the three channels' nv vectors -> (channel c, vector
// v, lane r of its NP-lane group)
template <int NP>
__device__ __forceinline__ void pass_item(int i, int nv, int& c, int& v, int& r) {
  r = i & (NP - 1);
  const int u = i / NP;
  c = u / nv;
  v = u - c * nv;
}

// rows: the candidate's rows of the three channels from the tile-major XYB
// copy into their planes (R x C, row-major; pl[c]: X, Y, B)
template <int C>
__device__ __forceinline__ void rows_pass(const MergeArgs& a, int bx, int by, int R, float* pl,
                                          int nch, int c0, int cstep, const BigLds& S) {
  constexpr int NP = C / 32, L = C == 64 ? 6 : (C == 128 ? 7 : 8);
  const int n = nch * R * NP;
  for (int base = 0; base < n; base += kBT) {
    const int i = base + (int)threadIdx.x;
    const bool act = i < n;
    int c, y, r;
    pass_item<NP>(act ? i : (i & (NP - 1)), R, c, y, r);  // (idle lanes: a valid row, not stored)
    c = c0 + c * cstep;  // the pass's channel list
    // pixel x of the row: tile (Y >> 6, (bx >> 3) + (x >> 6)), column x & 63
    // (varblocks start on the 64-px grid); 32-bit offsets from the frame's XYB base
    const int Y = by * 8 + y;
    const uint32_t row0 = ((uint32_t)(Y >> 6) * a.tiles_x + (uint32_t)(bx >> 3)) * (3u * 4096u) +
                          (uint32_t)(c * 4096 + (Y & 63) * 64);
    const float* xyb = a.xyb;
    float o[32];
    vb_vec<C>([&](int x) { return xyb[row0 + (uint32_t)((x >> 6) * (3 * 4096) + (x & 63))]; }, r, o, S);
    if (act) {  // column-major planes: coefficient (row y, column pos) at pos R + y
      const uint32_t d0 = (uint32_t)c * 65536u + (uint32_t)y;
#pragma unroll
      for (int k = 0; k < 32; k++) {
        const int pos = k * NP + r;
        pl[d0 + (uint32_t)(pos * R)] = o[k] * S.lee_s[L * 256 + pos];
      }
    }
  }
}
// columns, in place: every lane of a round computes before any stores
template <int R>
__device__ __forceinline__ void cols_pass(int C, float* pl, int nch, int c0, int cstep, const BigLds& S) {
  constexpr int NP = R / 32, L = R == 64 ? 6 : (R == 128 ? 7 : 8);
  const int n = nch * C * NP;
  for (int base = 0; base < n; base += kBT) {
    const int i = base + (int)threadIdx.x;
    const bool act = i < n;
    int c, x, r;
    pass_item<NP>(act ? i : (i & (NP - 1)), C, c, x, r);
    c = c0 + c * cstep;
    const uint32_t c0 = (uint32_t)c * 65536u + (uint32_t)(x * R);  // column x: R contiguous floats
    float o[32];
    vb_vec<R>([&](int p) { return pl[c0 + (uint32_t)p]; }, r, o, S);
    __syncthreads();
    if (act) {
#pragma unroll
      for (int k = 0; k < 32; k++) {
        const int pos = k * NP + r;
        pl[c0 + (uint32_t)pos] = o[k] * S.lee_s[L * 256 + pos];
      }
    }
  }
}

// channels c0, c0 + cstep, ... (nch of them)
__device__ __forceinline__ void vb_transform(const MergeArgs& a, const BigShape& sh, int bx, int by,
                                             float* pl, int nch, int c0, int cstep, const BigLds& S) {
  const int R = 8 << sh.lcy, C = 8 << sh.lcx;
  switch (sh.lcx) {
    case 3: rows_pass<64>(a, bx, by, R, pl, nch, c0, cstep, S); break;
    case 4: rows_pass<128>(a, bx, by, R, pl, nch, c0, cstep, S); break;
    default: rows_pass<256>(a, bx, by, R, pl, nch, c0, cstep, S); break;
  }
  __syncthreads();
  switch (sh.lcy) {
    case 3: cols_pass<64>(C, pl, nch, c0, cstep, S); break;
    case 4: cols_pass<128>(C, pl, nch, c0, cstep, S); break;
    default: cols_pass<256>(C, pl, nch, c0, cstep, S); break;
  }
  __syncthreads();
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
  float* part = S.part;
  int bits = 0, nzc = 0;
  const size_t nb = (size_t)a.bxs * a.bys;
  for (int t = threadIdx.x; t < nch * C; t += kBT) {
    const int chunk = t >> lC, x = t & (C - 1);
    float cp = 0.0f;
    // the chunk's 16 coefficients, Y's dequantized values (X / B) or the
    // inverse weights (Y) and the tables, loaded before the first use
    for (int hh = 0; hh < 16; hh += 8) {
    float pv[8], yv[8], wv[8], sdv[8];
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const int ky = chunk * 16 + hh + r;
      const int si = C >= R ? ky * C + x : x * R + ky;
      pv[r] = P[(size_t)x * R + ky];  // column-major planes
      yv[r] = ch != 1 ? Yp[(size_t)x * R + ky] : IW[si];  // Y: the inverse weight
      wv[r] = W[si];
      sdv[r] = SD[si];
    }
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const int ky = chunk * 16 + hh + r;
      const int si = C >= R ? ky * C + x : x * R + ky;
      float qq_f = 0.0f;
      bool neg = false;
      if (ky < cy && x < cx) {  // LLF: carried by the DC image
        if (WRITE) S.llf[ch][ky * 32 + x] = pv[r];
      } else {
        const float w = wv[r];
        float rv = pv[r];
        if (ch != 1) rv = rv - kc * yv[r];
        const float v = rv * (w * scale);
        const float av = fabsf(v);
        const float qf = av < 0.58f ? 0.0f : floorf(fminf(av, 32767.0f) + 0.5f);
        const int qa = (int)qf;
        if (ch == 1) {
          float adj = qa == 0 ? 0.0f : (qa == 1 ? kBias1 : qf - 0.145f / qf);
          if (v < 0.0f) adj = -adj;
          P[(size_t)x * R + ky] = adj * (yv[r] * inv_scale);
        }
        const float e = (av - qf) * sdv[r];
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
    }
    part[t] = cp;
  }
  (void)nb;
  if (bits) atomicAdd(&S.bits, bits);
  if (nzc) atomicAdd(&S.nz[ch], nzc);
  __syncthreads();
  // a chunk's column partials: pairwise tree over its C columns (tree_sum)
  for (int ls = 0; ls < lC; ls++) {
    const int st = 1 << ls, lper = lC - 1 - ls;  // per = C / (2 st) pairs per chunk
    for (int t = threadIdx.x; t < (nch << lper); t += kBT) {
      const int chunk = t >> lper, i = (chunk << lC) + ((t & ((1 << lper) - 1)) << (ls + 1));
      part[i] = part[i] + part[i + st];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float pc = part[0];
    for (int k = 1; k < nch; k++) pc = pc + part[k * C];
    S.pc[ch] = pc;
  }
  __syncthreads();
}

// transform + quantization of one candidate (scratch slot: planes X, Y, B);
// returns the estimate (thread 0's value is the one used).  cur: the region's
// current sum (eval) -- the candidate is dropped (+inf) when its estimate
// after Y alone already reaches it (the bits and the distortion sums only
// grow with X and B, every float op on them is monotone, so the final
// estimate would be >= cur >= the resolve's best and never chosen, alone or
// in a pair; hook F off -- its factor may be negative or NaN).  NaN cur or
// WRITE: no pruning.
template <bool WRITE>
__device__ __forceinline__ float vb_eval(const BigArgs& b, const BigShape& sh, int bx, int by, BigLds& S,
                                         float* pl, float cur) {
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
  vb_transform(a, sh, bx, by, pl, 1, 1, 0, S);  // Y (ends with a barrier)
  const float scale = (float)a.G * (float)S.raw / 65536.0f;
  // chroma from luma of the top-left block's tile (as the decoder applies it)
  const size_t tile = (size_t)(by >> 3) * a.tiles_x + (bx >> 3);
  const float kx = (float)a.cmap[tile] * (1.0f / 84.0f);
  const float kb = 1.0f + (float)a.cmap[a.ntiles_all + tile] * (1.0f / 84.0f);
  float* Yp = pl + 65536;  // planes: X, Y, B
  vb_quant<WRITE>(a, b.tab, b.nat, sh, bx, by, 1, Yp, Yp, scale, 0.0f, S);
  if (!WRITE && !(a.proposals & 2u)) {
    const float lb = ((float)(S.bits + (32 - __clz((uint32_t)S.nz[1]))) + 8.0f * S.pc[1]) * sh.tmul;
    if (lb >= cur) return __builtin_inff();  // (uniform: every thread reads the same LDS values)
  }
  vb_transform(a, sh, bx, by, pl, 2, 0, 2, S);  // X and B
  vb_quant<WRITE>(a, b.tab, b.nat, sh, bx, by, 0, pl, Yp, scale, kx, S);
  vb_quant<WRITE>(a, b.tab, b.nat, sh, bx, by, 2, pl + 2 * 65536, Yp, scale, kb, S);
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
// per group slot: level 128 (4 regions x 5), level 256 (5), then the regions'
// current sums (4 + 1, big_cur_kernel)
constexpr int kBigCost = 30;
__device__ __forceinline__ size_t cur_index(uint32_t gi, int L, int r) {
  return (size_t)gi * kBigCost + 25 + (L == 0 ? r : 4);
}

// one thread per region of level L: the sum of the decisions below in raster
// order (each varblock's estimate at its first block, 0 at covered blocks),
// which the eval kernel prunes against and the resolve kernel compares with
__global__ __launch_bounds__(256) void big_cur_kernel(Batch<BigArgs> bt_, int L) {
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
  b.cost[cur_index(gi, L, r)] = cur;
}

// the Lee tables into LDS (once per workgroup; the transforms read them per
// element and stage)
__device__ __forceinline__ void load_lee_tables(const float* tab, BigLds& S) {
  for (int i = threadIdx.x; i < 9 * 128; i += kBT) S.lee_c[i] = tab[kBigTabLeeC + i];
  for (int i = threadIdx.x; i < 9 * 256; i += kBT) S.lee_s[i] = tab[kBigTabLeeS + i];
  __syncthreads();
}

__global__ __launch_bounds__(kBT) __attribute__((amdgpu_waves_per_eu(4))) void big_eval_kernel(Batch<BigArgs> bt_, int L) {
  const BigArgs& b = bt_.a[blockIdx.z];
  __shared__ BigLds S;
  if (L == 0 && blockIdx.x == 0 && threadIdx.x == 0) b.work[0] = 0;  // big_list's count
  const int nreg = L == 0 ? 4 : 1;
  const uint32_t total = b.ng * (uint32_t)nreg * 5u;
  float* const pl = b.scratch + (size_t)blockIdx.x * kBigPlanes;  // X, Y, B planes
  load_lee_tables(b.tab, S);
  for (uint32_t w = blockIdx.x; w < total; w += gridDim.x) {
    const uint32_t gi = w / (nreg * 5), rem = w - gi * (nreg * 5);
    const int r = (int)rem / 5, j = (int)rem % 5;
    int bx0, by0;
    if (!big_region(b, L, gi, r, bx0, by0)) continue;  // (uniform)
    int bx, by;
    const BigShape& sh = big_cand(L, j, bx0, by0, bx, by);
    const float e = vb_eval<false>(b, sh, bx, by, S, pl, b.cost[cur_index(gi, L, r)]);
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
  const int nreg = L == 0 ? 4 : 1;
  const uint32_t idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= b.ng * (uint32_t)nreg) return;
  const uint32_t gi = idx / nreg;
  const int r = (int)(idx - gi * nreg);
  int bx0, by0;
  if (!big_region(b, L, gi, r, bx0, by0)) return;
  const float cur = b.cost[cur_index(gi, L, r)];
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
  if (t >= 21 && t <= 26) {
    b.work[1 + atomicAdd(b.work, 1u)] = gb;
    // kind 0 128X64 (22, 23), 1 128X128 (21), 2 256X128 (25, 26), 3 256X256 (24)
    const uint32_t k = t == 21 ? 1u : (t == 24 ? 3u : (t <= 23 ? 0u : 2u));
    atomicAdd(b.kinds + k, 1u);
  }
}

__global__ __launch_bounds__(kBT) __attribute__((amdgpu_waves_per_eu(4))) void big_write_kernel(Batch<BigArgs> bt_) {
  const BigArgs& b = bt_.a[blockIdx.z];
  const MergeArgs& a = b.m;
  __shared__ BigLds S;
  float* const pl = b.scratch + (size_t)blockIdx.x * kBigPlanes;  // X, Y, B planes
  const uint32_t n = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)b.work);
  const size_t nb = (size_t)a.bxs * a.bys;
  if (blockIdx.x < n) load_lee_tables(b.tab, S);
  for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
    const uint32_t gb0 = b.work[1 + w];
    const int bx = (int)(gb0 % a.bxs), by = (int)(gb0 / a.bxs);
    const uint8_t t = a.acs[gb0];
    int si = 0;
    for (int i = 0; i < 6; i++) si = kBig[i].type == t ? i : si;
    const BigShape& sh = kBig[si];
    (void)vb_eval<true>(b, sh, bx, by, S, pl, __builtin_nanf(""));
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
    const uint32_t nreg0 = ng * (L == 0 ? 4u : 1u);
    hipLaunchKernelGGL(big_cur_kernel, dim3((nreg0 + 255) / 256, 1, k), dim3(256), 0, s, bt, L);
    hipLaunchKernelGGL(big_eval_kernel, dim3(min(tasks, a[0].slots), 1, k), dim3(kBT), 0, s, bt, L);
    const uint32_t nreg = ng * (L == 0 ? 4u : 1u);
    hipLaunchKernelGGL(big_resolve_kernel, dim3((nreg + 255) / 256, 1, k), dim3(256), 0, s, bt, L);
  }
  hipLaunchKernelGGL(big_list_kernel, dim3(ng, 1, k), dim3(64), 0, s, bt);
  hipLaunchKernelGGL(big_write_kernel, dim3(min(ng * 16u, a[0].slots), 1, k), dim3(kBT), 0, s, bt);
  return hipGetLastError();
}

}  // namespace jxg
