// jxg_merge.hip -- merge stage of the AC-strategy search on gfx950:
// 8x8-class decisions -> 16x8 ... 64x64 varblocks, and the transform,
// quantization and LLF-derived DC of every merged varblock.
//
// One 512-thread workgroup per 64x64 tile (the unit libjxl's ProcessRectACS
// works on, combined.diff:346 context).  The tile's XYB planes are rebuilt in
// LDS from RGB8 (same pixel_xyb as the front kernel: 3 B/px re-read instead of
// keeping 12 B/px of XYB in HBM).  Per merge level s (16, 32, 64 px squares)
// the three candidate shapes (full, two tall halves, two wide halves) are
// evaluated for every region of the tile at once:
//   row pass    : lane = (varblock, channel, pixel row): C-point DCT in
//                 registers, written to an LDS coefficient plane (row stride 65:
//                 lanes on consecutive rows hit consecutive banks);
//   column pass : lane = (varblock, pixel column): R-point DCT of Y, X, B in
//                 registers, quantization with the CfL residual, rate bits and
//                 e*e partials; a C-lane XOR-butterfly tree gives the cost.
// One lane per region then resolves keep / full / tall / wide with the
// TryMergeAcs comparison (NaN accepted, combined.diff:294 context) and hook F
// (combined.diff:247-253) on every estimate.  Finally each chosen varblock is
// re-run in write mode (coefficients scattered to natural-order slices, LLF
// kept in LDS) and the DC of every covered block is derived from the LLF.
// Float op order == oracle/merge.c (jxo_varblock, jxo_llf_dc, jxo_merge_tile).
#include <float.h>

#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

__constant__ float c_mlut[256];
__constant__ float c_lee_c[7 * 32];  // [log2 N][i] = 1 / (2 cos(pi (2i+1) / 2N))
__constant__ float c_lee_s[7 * 64];  // [log2 N][k] = k ? sqrt2 / N : 1 / N
__constant__ float c_llf_p[4 * 8];   // [log2 M][k]
__constant__ float c_llf_ib[4 * 64]; // [log2 M][n][k]

constexpr int kMThreads = 512;
constexpr int kMS = 65;  // LDS row stride (floats)
constexpr int kMPlane = 64 * kMS;

template <int N>
constexpr int ilog2c() {
  return N <= 1 ? 0 : 1 + ilog2c<N / 2>();
}

// unnormalized DCT-II in registers, Lee's recursive even/odd split
// (== oracle/merge.c lee)
template <int N>
__device__ __forceinline__ void lee(float* x) {
  if constexpr (N > 1) {
    constexpr int h = N / 2, l = ilog2c<N>();
    float a[h], b[h];
#pragma unroll
    for (int i = 0; i < h; i++) {
      a[i] = x[i] + x[N - 1 - i];
      b[i] = (x[i] - x[N - 1 - i]) * c_lee_c[l * 32 + i];
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
template <int N>
__device__ __forceinline__ void dct_n(float* x) {
  lee<N>(x);
  constexpr int l = ilog2c<N>();
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = x[k] * c_lee_s[l * 64 + k];
}

// merged shapes (== oracle jxo_shapes): raw id, blocks down, blocks across,
// weight kind, cost multiplier
struct ShapeDesc {
  int type, cy, cx, kind;
  float tmul;
};
constexpr ShapeDesc kShapes[9] = {
    {6, 2, 1, 0, 1.0f},   {7, 1, 2, 0, 1.0f},   {4, 2, 2, 1, 1.0f},
    {10, 4, 2, 2, 1.02f}, {11, 2, 4, 2, 1.02f}, {5, 4, 4, 3, 1.03f},
    {19, 8, 4, 4, 1.05f}, {20, 4, 8, 4, 1.05f}, {18, 8, 8, 5, 1.05f}};

__device__ __forceinline__ int shape_index(int type) {
  switch (type) {
    case 6: return 0;
    case 7: return 1;
    case 4: return 2;
    case 10: return 3;
    case 11: return 4;
    case 5: return 5;
    case 19: return 6;
    case 20: return 7;
    case 18: return 8;
    default: return -1;
  }
}

__device__ __forceinline__ int bitlen_u(uint32_t v) { return 32 - __clz(v); }

struct MergeLds {
  float pix[3 * kMPlane];
  float co[3 * kMPlane];
  float cost[3][32];   // [candidate shape of the level][varblock grid index]
  float llf[3][64];    // LLF of merged varblocks at their covered blocks
  float ent[64];
  float r3[64][3];
  int raw[64];         // front-kernel quant field (raw, 1..256)
  int rmax[64];        // merged: max raw over the varblock (at covered blocks)
  uint8_t acs[64];
  uint8_t orig[64];    // merged: local index of the varblock's first block
  float lut[256];
};

struct MCtx {
  MergeLds* S;
  int tx, ty, nbx, nby;
};

// run-time description of one shape pass
struct Pass {
  int si, type, cy, cx, koff, s;
  float tmul;
  bool write;
  int slot;
  __device__ __forceinline__ int R() const { return 8 * cy; }
  __device__ __forceinline__ int C() const { return 8 * cx; }
  __device__ __forceinline__ int GX() const { return 8 / cx; }
  __device__ __forceinline__ int NV() const { return (8 / cx) * (8 / cy); }
};

// Eval validity: the level-s region containing the varblock lies inside the
// frame's blocks.  Write validity: the tile's final map holds the shape there.
__device__ __forceinline__ bool vb_valid(const Pass& P, const MCtx& m, int bx0, int by0) {
  if (P.write) return m.S->acs[by0 * 8 + bx0] == (uint8_t)P.type;
  const int rx = bx0 / P.s, ry = by0 / P.s;
  return (rx + 1) * P.s <= m.nbx && (ry + 1) * P.s <= m.nby;
}

// row pass: C-point DCT of every pixel row (3 channels) of every varblock
template <int C>
__device__ void row_pass(const Pass& P, const MCtx& m) {
  MergeLds& S = *m.S;
  const int R = P.R(), GX = P.GX(), n = P.NV() * 3 * R;
  for (int i = threadIdx.x; i < n; i += kMThreads) {
    const int v = i / (3 * R), rem = i - v * (3 * R), c = rem / R, y = rem - c * R;
    const int vx = v % GX, vy = v / GX;
    if (!vb_valid(P, m, vx * P.cx, vy * P.cy)) continue;
    const int off = c * kMPlane + (vy * R + y) * kMS + vx * C;
    float x[C];
#pragma unroll
    for (int k = 0; k < C; k++) x[k] = S.pix[off + k];
    dct_n<C>(x);
#pragma unroll
    for (int k = 0; k < C; k++) S.co[off + k] = x[k];
  }
}

// column pass: R-point DCT of Y, X, B per pixel column (lane), quantization
// with the CfL residual (the Y dequantized values go back into the lane's own
// Y column of the coefficient plane), rate bits and e*e partials; C-lane
// XOR-butterfly reductions.  Eval: cost per varblock; write: coefficients,
// LLF, non-zero counts, origins.
template <int R>
__device__ void col_pass(const MergeArgs& a, const Pass& P, const MCtx& m) {
  constexpr int KTOT = kKindOff[kNumKinds];
  MergeLds& S = *m.S;
  const int C = P.C(), GX = P.GX(), CY = P.cy, CX = P.cx, CB = CY * CX;
  const int n = P.NV() * C;  // multiple of 64
  for (int i = threadIdx.x; i < n; i += kMThreads) {
    const int v = i / C, x = i - v * C;
    const int vx = v % GX, vy = v / GX;
    const int bx0 = vx * CX, by0 = vy * CY;
    if (!vb_valid(P, m, bx0, by0)) continue;  // uniform over the varblock's C lanes
    int raw = 0;
    for (int iy = 0; iy < CY; iy++)
      for (int ix = 0; ix < CX; ix++) raw = max(raw, S.raw[(by0 + iy) * 8 + bx0 + ix]);
    const float scale = (float)a.G * (float)raw / 65536.0f;
    const float inv_scale = 1.0f / scale;
    float part = 0.0f;
    int bits = 0, nz0 = 0, nz1 = 0, nz2 = 0;
    const bool wide = CX >= CY;
#pragma unroll 1
    for (int ci = 0; ci < 3; ci++) {
      const int c = ci == 0 ? 1 : (ci == 1 ? 0 : 2);
      float* cplane = S.co + c * kMPlane + (vy * R) * kMS + vx * C + x;
      float* yplane = S.co + kMPlane + (vy * R) * kMS + vx * C + x;
      {
        // the column DCT in registers, written back to the lane's own column
        float col[R];
#pragma unroll
        for (int ky = 0; ky < R; ky++) col[ky] = cplane[ky * kMS];
        dct_n<R>(col);
#pragma unroll
        for (int ky = 0; ky < R; ky++) cplane[ky * kMS] = col[ky];
      }
      const float* wrow = a.wk + (size_t)c * KTOT + P.koff;
      int nzc = 0;
#pragma unroll 4
      for (int ky = 0; ky < R; ky++) {
        const float coef_v = cplane[ky * kMS];
        const int si = wide ? ky * C + x : x * R + ky;
        const bool is_llf = ky < CY && x < CX;
        int qq = 0;
        if (!is_llf) {
          const float w = wrow[si];
          const float ws = w * scale;
          float rv = coef_v;
          if (c == 2) rv = rv - yplane[ky * kMS];
          const float vq = rv * ws;
          const float av = fabsf(vq);
          const int qa = av < 0.58f ? 0 : (int)(fminf(av, 32767.0f) + 0.5f);
          qq = vq < 0.0f ? -qa : qa;
          if (c == 1) {
            constexpr float kBias1 = 1.0f - 0.07005449891748593f;
            float adj = qa == 0 ? 0.0f : (qa == 1 ? kBias1 : (float)qa - 0.145f / (float)qa);
            if (vq < 0.0f) adj = -adj;
            yplane[ky * kMS] = adj * (a.iwy[P.koff + si] * inv_scale);
          }
          const float e = av - (float)qa;
          part = fmaf(e, e, part);
          bits += qa ? 2 + 2 * bitlen_u((uint32_t)qa) : 0;
          nzc += qa != 0;
        } else if (P.write) {
          S.llf[c][(by0 + ky) * 8 + bx0 + x] = coef_v;
        }
        if (P.write) {
          const int p = a.nat[P.koff + si];
          const int sl = p >> 6;
          const int lbx = bx0 + sl % CX, lby = by0 + sl / CX;
          const size_t gb = (size_t)(m.ty * 8 + lby) * a.bxs + m.tx * 8 + lbx;
          a.ac[(gb * 3 + c) * 64 + (p & 63)] = (int16_t)qq;
        }
      }
      nz0 += c == 0 ? nzc : 0;
      nz1 += c == 1 ? nzc : 0;
      nz2 += c == 2 ? nzc : 0;
    }
    // C-lane reductions (aligned groups inside one wave)
    for (int msk = 1; msk < C; msk <<= 1) {
      part += __shfl_xor(part, msk, 64);
      bits += __shfl_xor(bits, msk, 64);
      nz0 += __shfl_xor(nz0, msk, 64);
      nz1 += __shfl_xor(nz1, msk, 64);
      nz2 += __shfl_xor(nz2, msk, 64);
    }
    if (!P.write) {
      if (x == 0) {
        const int tb = bitlen_u((uint32_t)nz0) + bitlen_u((uint32_t)nz1) + bitlen_u((uint32_t)nz2);
        float e = ((float)(bits + tb) + 8.0f * part) * P.tmul;
        if (a.proposals & 2u) {
          const float* h = S.r3[by0 * 8 + bx0];
          e = hook_f(e, h[0], h[1], h[2]);
        }
        S.cost[P.slot][v] = e;
      }
    } else if (x < CB) {
      // per covered block: non-zero counts, varblock origin, quant field
      const int lbx = bx0 + x % CX, lby = by0 + x / CX;
      const int lcb = CB == 2 ? 1 : CB == 4 ? 2 : CB == 8 ? 3 : CB == 16 ? 4 : CB == 32 ? 5 : 6;
      const size_t nb = (size_t)a.bxs * a.bys;
      const size_t gb = (size_t)(m.ty * 8 + lby) * a.bxs + m.tx * 8 + lbx;
      a.nz[gb] = (uint16_t)(x == 0 ? nz0 : (nz0 + CB - 1) >> lcb);
      a.nz[nb + gb] = (uint16_t)(x == 0 ? nz1 : (nz1 + CB - 1) >> lcb);
      a.nz[2 * nb + gb] = (uint16_t)(x == 0 ? nz2 : (nz2 + CB - 1) >> lcb);
      S.orig[lby * 8 + lbx] = (uint8_t)(by0 * 8 + bx0);
      S.rmax[lby * 8 + lbx] = raw;
    }
  }
}

// one shape: row pass, barrier, column pass, barrier
__device__ void run_shape(const MergeArgs& a, const MCtx& m, int si, int s, bool write,
                          int slot) {
  const ShapeDesc& D = kShapes[si];
  Pass P;
  P.si = si;
  P.type = D.type;
  P.cy = D.cy;
  P.cx = D.cx;
  P.koff = kKindOff[D.kind];
  P.s = s;
  P.tmul = D.tmul;
  P.write = write;
  P.slot = slot;
  switch (P.cx) {
    case 1: row_pass<8>(P, m); break;
    case 2: row_pass<16>(P, m); break;
    case 4: row_pass<32>(P, m); break;
    default: row_pass<64>(P, m); break;
  }
  __syncthreads();
  switch (P.cy) {
    case 1: col_pass<8>(a, P, m); break;
    case 2: col_pass<16>(a, P, m); break;
    case 4: col_pass<32>(a, P, m); break;
    default: col_pass<64>(a, P, m); break;
  }
  __syncthreads();
}

__global__ __launch_bounds__(kMThreads) void merge_kernel(MergeArgs a) {
  __shared__ __attribute__((aligned(16))) MergeLds S;
  const int tid = threadIdx.x;
  const int tx = blockIdx.x, ty = blockIdx.y;
  const int nbx = min(8, (int)a.bxs - tx * 8), nby = min(8, (int)a.bys - ty * 8);
  if (nbx < 2 || nby < 2) return;  // no 16x16 region fits: nothing to merge
  const size_t nb = (size_t)a.bxs * a.bys;
  if (tid < 256) S.lut[tid] = c_mlut[tid];
  if (tid < 64) {
    const int lbx = tid & 7, lby = tid >> 3;
    const bool in = lbx < nbx && lby < nby;
    const size_t gb = (size_t)(ty * 8 + lby) * a.bxs + tx * 8 + lbx;
    S.ent[tid] = in ? a.ent[gb] : 0.0f;
    S.raw[tid] = in ? (int)a.qf[gb] + 1 : 1;
    S.acs[tid] = in ? a.acs[gb] : 0;
    if (a.homog) {
      S.r3[tid][0] = in ? a.homog[gb * 3 + 0] : 0.0f;
      S.r3[tid][1] = in ? a.homog[gb * 3 + 1] : 0.0f;
      S.r3[tid][2] = in ? a.homog[gb * 3 + 2] : 0.0f;
    }
  }
  __syncthreads();
  // XYB tile (same conversion and edge handling as the front kernel)
  {
    const float cb = cbrt_det(kOpsinBias);
    const int ox = tx * 64, oy = ty * 64;
    for (int i = tid; i < 64 * 64; i += kMThreads) {
      const int ly = i >> 6, lx = i & 63;
      const int gx = ox + lx, gy = oy + ly;
      float X = 0.0f, Y = 0.0f, B = 0.0f;
      if (gx < (int)a.xp && gy < (int)a.yp) {
        const int sx = min(gx, (int)a.w - 1), sy = min(gy, (int)a.h - 1);
        const uint8_t* p = a.rgb + (size_t)sy * a.stride + 3 * (size_t)sx;
        pixel_xyb(S.lut, cb, p[0], p[1], p[2], X, Y, B);
      }
      const int o = ly * kMS + lx;
      S.pix[o] = X;
      S.pix[kMPlane + o] = Y;
      S.pix[2 * kMPlane + o] = B;
    }
  }
  __syncthreads();
  const MCtx m{&S, tx, ty, nbx, nby};
  bool merged = false;
  for (int s = 2; s <= a.max_s; s *= 2) {
    const int nr = 8 / s;
    if (s > nbx || s > nby) break;  // no region of this size (or larger) fits
    const int full = s == 2 ? 2 : (s == 4 ? 5 : 8);
    const int tall = s == 2 ? 0 : (s == 4 ? 3 : 6);
    run_shape(a, m, full, s, false, 0);
    run_shape(a, m, tall, s, false, 1);
    run_shape(a, m, tall + 1, s, false, 2);
    bool any = false;
    if (tid < nr * nr) {
      const int rx = tid % nr, ry = tid / nr;
      if ((rx + 1) * s <= nbx && (ry + 1) * s <= nby) {
        float cur = 0.0f;
        for (int iy = 0; iy < s; iy++)
          for (int ix = 0; ix < s; ix++) cur += S.ent[(ry * s + iy) * 8 + rx * s + ix];
        const float e0 = S.cost[0][ry * nr + rx];
        const int vl = ry * (16 / s) + 2 * rx;
        const float et = S.cost[1][vl] + S.cost[1][vl + 1];
        const int vt = (2 * ry) * nr + rx;
        const float ew = S.cost[2][vt] + S.cost[2][vt + nr];
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
        if (choice) {
          any = true;
          // varblocks of the choice: (shape, block origin, estimate)
          const int nv = choice == 1 ? 1 : 2;
          for (int j = 0; j < nv; j++) {
            int si, bx, by;
            float e;
            if (choice == 1) {
              si = full, bx = rx * s, by = ry * s, e = e0;
            } else if (choice == 2) {
              si = tall, bx = rx * s + j * (s / 2), by = ry * s, e = S.cost[1][vl + j];
            } else {
              si = tall + 1, bx = rx * s, by = ry * s + j * (s / 2), e = S.cost[2][vt + j * nr];
            }
            const int cy = kShapes[si].cy, cx = kShapes[si].cx, type = kShapes[si].type;
            for (int iy = 0; iy < cy; iy++)
              for (int ix = 0; ix < cx; ix++) {
                const int b = (by + iy) * 8 + bx + ix;
                S.acs[b] = (uint8_t)(type | ((iy | ix) ? 0x80 : 0));
                S.ent[b] = (iy | ix) ? 0.0f : e;
              }
          }
        }
      }
    }
    merged |= __syncthreads_or(any) != 0;
  }
  if (!merged) return;  // the front kernel's output stands
  // ---- emit the chosen varblocks ----
#pragma unroll 1
  for (int si = 0; si < 9; si++) {
    bool has = false;
    if (tid < 64) has = S.acs[tid] == (uint8_t)kShapes[si].type;
    if (__syncthreads_or(has)) run_shape(a, m, si, 0, true, 0);
  }
  // ---- per covered block: LLF-derived DC, quant field, strategy ----
  if (tid < 64) {
    const int lbx = tid & 7, lby = tid >> 3;
    if (lbx < nbx && lby < nby) {
      const size_t gb = (size_t)(ty * 8 + lby) * a.bxs + tx * 8 + lbx;
      const int t = S.acs[tid];
      a.acs[gb] = (uint8_t)t;
      const int si = shape_index(t & 0x7F);
      if (si >= 0) {
        const int o = S.orig[tid];
        const int oy = o >> 3, ox = o & 7;
        const int cy = kShapes[si].cy, cx = kShapes[si].cx;
        const int ly = cy == 1 ? 0 : (cy == 2 ? 1 : (cy == 4 ? 2 : 3));
        const int lx = cx == 1 ? 0 : (cx == 2 ? 1 : (cx == 4 ? 2 : 3));
        const int iy = lby - oy, ix = lbx - ox;
        float dc[3];
        for (int c = 0; c < 3; c++) {
          float acc = 0.0f;
          for (int ky = 0; ky < cy; ky++) {
            float u = 0.0f;
            for (int kx = 0; kx < cx; kx++) {
              const float tt = (S.llf[c][(oy + ky) * 8 + ox + kx] * c_llf_p[ly * 8 + ky]) *
                               c_llf_p[lx * 8 + kx];
              u = fmaf(tt, c_llf_ib[lx * 64 + ix * 8 + kx], u);
            }
            acc = fmaf(u, c_llf_ib[ly * 64 + iy * 8 + ky], acc);
          }
          dc[c] = acc;
        }
        int32_t q[3];
        quant_dc3(dc, a.dc_mul, a.dc_step, q);
        a.dc[gb] = q[0];
        a.dc[nb + gb] = q[1];
        a.dc[2 * nb + gb] = q[2];
        a.qf[gb] = (uint8_t)(S.rmax[tid] - 1);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// varblock lists of the LF groups (AC metadata channel of size count x 2):
// block indices of the varblocks' first blocks in LF-group raster order
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void vb_list_kernel(VbArgs a) {
  __shared__ uint32_t sWave[16];
  __shared__ uint32_t sBase;
  const uint32_t lg = blockIdx.x;
  const uint32_t bx0 = (lg % a.lfxs) * 256, by0 = (lg / a.lfxs) * 256;
  const uint32_t bw = min(256u, a.bxs - bx0), bh = min(256u, a.bys - by0);
  const uint32_t n = bw * bh;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) sBase = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < n; c0 += 1024) {
    const uint32_t i = c0 + threadIdx.x;
    size_t b = 0;
    uint32_t f = 0;
    if (i < n) {
      b = (size_t)(by0 + i / bw) * a.bxs + bx0 + i % bw;
      f = (a.acs[b] & 0x80) ? 0u : 1u;
    }
    const uint64_t bal = __ballot(f);
    const uint32_t below = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) sWave[wv] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = sBase, tot = 0;
    for (int w = 0; w < 16; w++) {
      before += w < wv ? sWave[w] : 0u;
      tot += sWave[w];
    }
    if (f) a.vb[(size_t)lg * 65536 + before + below] = (uint32_t)b;
    __syncthreads();
    if (threadIdx.x == 0) sBase += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) a.count[lg] = sBase;
}

void set_merge_constants(const float lut[256], const float* lee_c, const float* lee_s,
                         const float* llf_p, const float* llf_ib, hipStream_t s) {
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(c_mlut), lut, sizeof(float) * 256, 0,
                               hipMemcpyHostToDevice, s);
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(c_lee_c), lee_c, sizeof(float) * 7 * 32, 0,
                               hipMemcpyHostToDevice, s);
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(c_lee_s), lee_s, sizeof(float) * 7 * 64, 0,
                               hipMemcpyHostToDevice, s);
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(c_llf_p), llf_p, sizeof(float) * 4 * 8, 0,
                               hipMemcpyHostToDevice, s);
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(c_llf_ib), llf_ib, sizeof(float) * 4 * 64, 0,
                               hipMemcpyHostToDevice, s);
  (void)hipStreamSynchronize(s);
}
void launch_merge(const MergeArgs& a, uint32_t tiles_x, uint32_t tiles_y, hipStream_t s) {
  hipLaunchKernelGGL(merge_kernel, dim3(tiles_x, tiles_y), dim3(kMThreads), 0, s, a);
}
void launch_vb_list(const VbArgs& a, uint32_t nlf, hipStream_t s) {
  hipLaunchKernelGGL(vb_list_kernel, dim3(nlf), dim3(1024), 0, s, a);
}

}  // namespace jxg
