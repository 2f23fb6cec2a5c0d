// jxg_tables.cpp -- host-side constant tables (declared in jxg_tables.h)
#include "jxg_tables.h"

#include <cmath>
#include <cstring>

#include "jxg_bitstream.h"
#include "jxg_kernels.h"

namespace jxg {

// default dequantization weights (inverse steps) [ext libjxl quant_weights.cc]
// kinds: 0 DCT8, 1 DCT4X4, 2 DCT4X8 / DCT8X4, 3 IDENTITY, 4 DCT2X2
void quant_weights(float out[5][3][64]) {
  static const double dct8[3][6] = {{3150.0, 0.0, -0.4, -0.4, -0.4, -2.0},
                                    {560.0, 0.0, -0.3, -0.3, -0.3, -0.3},
                                    {512.0, -2.0, -1.0, 0.0, -1.0, -2.0}};
  static const double dct4[3][6] = {
      {2200.0, 0.0, 0.0, 0.0}, {392.0, 0.0, 0.0, 0.0}, {112.0, -0.25, -0.25, -0.5}};
  static const double dct4x8[3][6] = {
      {2198.050556016380522, -0.96269623020744692, -0.76194253026666783, -0.6551140670773547},
      {764.3655248643528689, -0.92630200888366945, -0.9675229603596517, -0.27845290869168118},
      {527.107573587542228, -1.4594385811273854, -1.450082094097871593, -1.5843722511996204}};
  auto weights = [](int rows, int cols, const double (*bands_in)[6], int nb, double* out3) {
    for (int c = 0; c < 3; c++) {
      double bands[6];
      bands[0] = bands_in[c][0];
      for (int i = 1; i < nb; i++) {
        const double v = bands_in[c][i];
        bands[i] = bands[i - 1] * (v > 0 ? 1.0 + v : 1.0 / (1.0 - v));
      }
      const double scale = (nb - 1) / (1.4142135623730951 + 1e-6);
      const double rc = scale / (cols - 1), rr = scale / (rows - 1);
      for (int y = 0; y < rows; y++) {
        const double dy = y * rr;
        for (int x = 0; x < cols; x++) {
          const double dx = x * rc;
          const double pos = std::sqrt(dx * dx + dy * dy);
          int idx = (int)pos;
          if (idx > nb - 2) idx = nb - 2;
          const double frac = pos - idx;
          const double a = bands[idx], b = bands[idx + 1];
          out3[c * 64 + y * cols + x] = a * std::pow(b / a, frac);
        }
      }
    }
  };
  double w[3 * 64];
  weights(8, 8, dct8, 6, w);
  for (int c = 0; c < 3; c++)
    for (int i = 0; i < 64; i++) out[0][c][i] = (float)w[c * 64 + i];
  weights(4, 4, dct4, 4, w);
  for (int c = 0; c < 3; c++)
    for (int y = 0; y < 8; y++)
      for (int x = 0; x < 8; x++) out[1][c][y * 8 + x] = (float)w[c * 64 + (y / 2) * 4 + x / 2];
  weights(4, 8, dct4x8, 4, w);
  for (int c = 0; c < 3; c++)
    for (int y = 0; y < 8; y++)
      for (int x = 0; x < 8; x++) out[2][c][y * 8 + x] = (float)w[c * 64 + (y / 2) * 8 + x];
  // IDENTITY: weight [0] everywhere, [1] at slots 1 / 8, [2] at slot 9;
  // DCT2X2: [0] slots 1 / 8, [1] slot 9, level-2 quadrants [2] / [3]
  // (off-diagonal / diagonal), level-1 quadrants [4] / [5]
  // [ext quant_weights.cc kQuantModeID / kQuantModeDCT2 defaults; == oracle]
  static const float id_w[3][3] = {{280.0f, 3160.0f, 3160.0f}, {60.0f, 864.0f, 864.0f},
                                   {18.0f, 200.0f, 200.0f}};
  static const float dct2_w[3][6] = {{3840.0f, 2560.0f, 1280.0f, 640.0f, 480.0f, 300.0f},
                                     {960.0f, 640.0f, 320.0f, 180.0f, 140.0f, 120.0f},
                                     {640.0f, 320.0f, 128.0f, 64.0f, 32.0f, 16.0f}};
  for (int c = 0; c < 3; c++) {
    for (int i = 0; i < 64; i++) out[3][c][i] = id_w[c][0];
    out[3][c][1] = out[3][c][8] = id_w[c][1];
    out[3][c][9] = id_w[c][2];
    for (int y = 0; y < 8; y++)
      for (int x = 0; x < 8; x++) {
        int k;
        if (y < 2 && x < 2) k = (y && x) ? 1 : 0;
        else if (y < 4 && x < 4) k = (y >= 2 && x >= 2) ? 3 : 2;
        else k = (y >= 4 && x >= 4) ? 5 : 4;
        out[4][c][y * 8 + x] = dct2_w[c][k];
      }
  }
}

// fuzzy-erosion weights of the masking quant field (== oracle/aq.c
// jxo_aq_erosion_weights, float ops in the same order) [ext, as recalled]
void aq_erosion_weights(float distance, float w[4]) {
  float mul = 0.0f;
  if (distance < 2.0f) mul = (2.0f - distance) * (1.0f / 2.0f);
  w[0] = 0.125f + mul * 0.0f;
  w[1] = 0.10f + mul * -0.10f;
  w[2] = 0.09f + mul * -0.09f;
  w[3] = 0.06f + mul * -0.06f;
  const float norm = 0.29959705784054957f / (((w[0] + w[1]) + w[2]) + w[3]);
  for (int i = 0; i < 4; i++) w[i] *= norm;
}

void srgb_lut(float lut[256]) {
  for (int u = 0; u < 256; u++) {
    const double v = u / 255.0;
    lut[u] = (float)(v <= 0.04045 ? v / 12.92 : std::pow((v + 0.055) / 1.055, 2.4));
  }
}

// ---- merge-stage tables [ext quant_weights.cc / coeff_order.cc]; same
// double-precision formulas as oracle/merge.c ----
static const double kKindBands[kNumKinds][3][8] = {
    {{7240.7734393502, -0.7, -0.7, -0.2, -0.2, -0.2, -0.5},
     {1448.15468787004, -0.5, -0.5, -0.5, -0.2, -0.2, -0.2},
     {506.854140754517, -1.4, -0.2, -0.5, -0.5, -1.5, -3.6}},
    {{8996.8725711814115328, -1.3000777393353804, -0.49424529824571225, -0.439093774457103443,
      -0.6350101832695744, -0.90177264050827612, -1.6162099239887414},
     {3191.48366296844234752, -0.67424582104194355, -0.80745813428471001,
      -0.44925837484843441, -0.35865440981033403, -0.31322389111877305, -0.37615025315725483},
     {1157.50408145487200256, -2.0531423165804414, -1.4, -0.50687130033378396,
      -0.42708730624733904, -1.4856834539296244, -4.9209142884401604}},
    {{13844.97076442300573, -0.97113799999999995, -0.658, -0.42026, -0.22712, -0.2206, -0.226,
      -0.6},
     {4798.964084220744293, -0.61125308982767057, -0.83770786552491361, -0.79014862079498627,
      -0.2692727459704829, -0.38272769465388551, -0.22924222653091453, -0.20719098826199578},
     {1807.236946760964614, -1.2, -1.2, -0.7, -0.7, -0.7, -0.4, -0.5}},
    {{15718.40830982518931456, -1.025, -0.98, -0.9012, -0.4, -0.48819395464, -0.421064, -0.27},
     {7305.7636810695983104, -0.8041958212306401, -0.7633036457487539, -0.55660379990111464,
      -0.49785304658857626, -0.43699592683512467, -0.40180866526242109, -0.27321683125358037},
     {3803.53173721215041536, -3.060733579805728, -2.0413270132490346, -2.0235650159727417,
      -0.5495389509954993, -0.4, -0.4, -0.3}},
    {{0.65 * 23629.073922049845, -1.025, -0.78, -0.65012, -0.19041574084286472, -0.20819395464,
      -0.421064, -0.32733845535848671},
     {0.65 * 8611.3238710010046, -0.3041958212306401, -0.3633036457487539, -0.35660379990111464,
      -0.3443074455424403, -0.33699592683512467, -0.30180866526242109, -0.27321683125358037},
     {0.65 * 4492.2486445538634, -1.2, -1.2, -0.8, -0.7, -0.7, -0.4, -0.5}},
    {{0.9 * 26629.073922049845, -1.025, -0.78, -0.65012, -0.19041574084286472, -0.20819395464,
      -0.421064, -0.32733845535848671},
     {0.9 * 9311.3238710010046, -0.3041958212306401, -0.3633036457487539, -0.35660379990111464,
      -0.3443074455424403, -0.33699592683512467, -0.30180866526242109, -0.27321683125358037},
     {0.9 * 4992.2486445538634, -1.2, -1.2, -0.8, -0.7, -0.7, -0.4, -0.5}},
};
static const int kKindNumBands[kNumKinds] = {7, 7, 8, 8, 8, 8};
static const int kKindDims[kNumKinds][2] = {{8, 16}, {16, 16}, {16, 32},
                                           {32, 32}, {32, 64}, {64, 64}};

MergeTables build_merge_tables() {
  MergeTables T;
  const int tot = kKindOff[kNumKinds];
  T.wk.assign((size_t)3 * tot, 0.0f);
  T.iwy.assign(tot, 0.0f);
  T.nat.assign(tot, 0);
  for (int k = 0; k < kNumKinds; k++) {
    const int rows = kKindDims[k][0], cols = kKindDims[k][1], nb = kKindNumBands[k];
    for (int c = 0; c < 3; c++) {
      double bands[8];
      bands[0] = kKindBands[k][c][0];
      for (int i = 1; i < nb; i++) {
        const double v = kKindBands[k][c][i];
        bands[i] = bands[i - 1] * (v > 0 ? 1.0 + v : 1.0 / (1.0 - v));
      }
      const double scale = (nb - 1) / (1.4142135623730951 + 1e-6);
      const double rc = scale / (cols - 1), rr = scale / (rows - 1);
      for (int y = 0; y < rows; y++)
        for (int x = 0; x < cols; x++) {
          const double dx = x * rc, dy = y * rr;
          const double pos = std::sqrt(dx * dx + dy * dy);
          int idx = (int)pos;
          if (idx > nb - 2) idx = nb - 2;
          const double frac = pos - idx;
          const double a = bands[idx], b = bands[idx + 1];
          T.wk[(size_t)c * tot + kKindOff[k] + y * cols + x] = (float)(a * std::pow(b / a, frac));
        }
    }
    for (int i = 0; i < rows * cols; i++) T.iwy[kKindOff[k] + i] = 1.0f / T.wk[(size_t)tot + kKindOff[k] + i];
    // natural order: LLF raster, then the y-scaled zigzag over cols x cols
    uint16_t* nat = &T.nat[kKindOff[k]];
    const int cs = rows / 8, cl = cols / 8, xf = cols / rows;
    int cur = 0;
    for (int y = 0; y < cs; y++)
      for (int x = 0; x < cl; x++) nat[y * cols + x] = (uint16_t)cur++;
    auto visit = [&](int x, int y, bool skip_llf) {
      if (y % xf) return;
      y /= xf;
      if (skip_llf && x < cl && y < cs) return;
      nat[y * cols + x] = (uint16_t)cur++;
    };
    for (int i = 0; i < cols; i++)
      for (int j = 0; j <= i; j++) {
        const bool odd = i & 1;
        visit(odd ? i - j : j, odd ? j : i - j, true);
      }
    for (int ip = cols - 1; ip > 0; ip--) {
      const int i = ip - 1;
      for (int j = 0; j <= i; j++) {
        const int x = cols - 1 - (i - j), y = cols - 1 - j;
        const bool odd = i & 1;
        visit(odd ? y : x, odd ? x : y, false);
      }
    }
  }
  // per-shape pixel-orientation copies in row quads ([ky / 4][kx][ky % 4]; tall
  // shapes read the stored table transposed) -- the lanes of a quantization
  // pass are consecutive columns kx, so one 16-byte load per lane brings a
  // lane's four rows and the wave's access is 1 KB contiguous: the cache lines
  // of four row-major loads in a quarter of the load instructions (per-lane
  // 16-byte column chunks [kx][ky] touched 64 cache lines per load and cost
  // merge_eval ~13 % in address processing)
  {
    static const int kShapeDims[kNumShapes][3] = {{2, 1, 0}, {1, 2, 0}, {2, 2, 1}, {4, 2, 2}, {2, 4, 2},
                                                 {4, 4, 3}, {8, 4, 4}, {4, 8, 4}, {8, 8, 5}};
    const int stot = kShapeOff[kNumShapes];
    std::vector<float> swk((size_t)3 * stot), ssdk((size_t)3 * stot), siwy(stot);
    std::vector<uint16_t> snat(stot);
    for (int sh = 0; sh < kNumShapes; sh++) {
      const int cy = kShapeDims[sh][0], cx = kShapeDims[sh][1], k = kShapeDims[sh][2];
      const int R = 8 * cy, C = 8 * cx;
      for (int ky = 0; ky < R; ky++)
        for (int kx = 0; kx < C; kx++) {
          const int si = cx >= cy ? ky * C + kx : kx * R + ky;
          const int pi = kShapeOff[sh] + ((ky >> 2) * C + kx) * 4 + (ky & 3);
          // LLF positions (the first cy x cx): weight 0, so they quantize to 0
          // and add nothing without a per-coefficient test in the kernels
          const bool llf = ky < cy && kx < cx;
          for (int c = 0; c < 3; c++) {
            const float wv = T.wk[(size_t)c * tot + kKindOff[k] + si];
            swk[(size_t)c * stot + pi] = llf ? 0.0f : wv;
            ssdk[(size_t)c * stot + pi] = llf ? 0.0f : dist_weight(c, R * C, wv);
          }
          siwy[pi] = T.iwy[kKindOff[k] + si];
          snat[pi] = T.nat[kKindOff[k] + si];
        }
    }
    T.wk.swap(swk);
    T.sdk.swap(ssdk);
    T.iwy.swap(siwy);
    T.nat.swap(snat);
  }
  const double pi = 3.14159265358979323846;
  std::memset(T.lee_c, 0, sizeof(T.lee_c));
  std::memset(T.lee_s, 0, sizeof(T.lee_s));
  for (int l = 0; l < 7; l++) {
    const int N = 1 << l;
    for (int i = 0; i < N / 2; i++)
      T.lee_c[l][i] = (float)(1.0 / (2.0 * std::cos(pi * (2 * i + 1) / (2.0 * N))));
    for (int k = 0; k < N; k++) T.lee_s[l][k] = (float)(k ? std::sqrt(2.0) / N : 1.0 / N);
  }
  std::memset(T.llf_p, 0, sizeof(T.llf_p));
  std::memset(T.llf_ib, 0, sizeof(T.llf_ib));
  for (int l = 0; l < 4; l++) {
    const int M = 1 << l;
    for (int k = 0; k < M; k++)
      T.llf_p[l][k] = (float)(std::cos(pi * k / (16.0 * M)) * std::cos(pi * k / (8.0 * M)) *
                              std::cos(pi * k / (4.0 * M)));
    for (int n = 0; n < M; n++)
      for (int k = 0; k < M; k++)
        T.llf_ib[l][n][k] =
            (float)(k ? std::sqrt(2.0) * std::cos(pi * (2 * n + 1) * k / (2.0 * M)) : 1.0);
  }
  return T;
}

double f16_round(double v) {
  const double a = std::fabs(v);
  if (a == 0.0) return 0.0;
  int e;
  (void)std::frexp(a, &e);  // a = m * 2^e, m in [0.5, 1)
  int ue = e - 11;          // ulp exponent of an 11-bit significand
  if (ue < -24) ue = -24;   // subnormal spacing
  const double q = std::ldexp(std::nearbyint(std::ldexp(a, -ue)), ue);
  return v < 0 ? -q : q;
}
uint32_t f16_bits(double v) {
  const uint32_t sign = v < 0 ? 0x8000u : 0u;
  const double a = std::fabs(v);
  if (a == 0.0) return sign;
  if (a < std::ldexp(1.0, -14)) return sign | (uint32_t)std::ldexp(a, 24);
  int e;
  const double m = std::frexp(a, &e);
  return sign | (uint32_t)(e - 1 + 15) << 10 | (uint32_t)std::ldexp(2.0 * m - 1.0, 10);
}

// DCT128X64, DCT128X128, DCT256X128, DCT256X256: the bands of DCT64X32 /
// DCT64X64 with the first band scaled up with the size (== oracle/merge.c),
// rounded to the binary16 parameters the stream carries for them
// (write_dequant_matrices): the first band 64 * f16(band / 64), the others
// f16(v)
static const double kBigY32[3] = {23629.073922049845, 8611.3238710010046, 4492.2486445538634};
static const double kBigY64[3] = {26629.073922049845, 9311.3238710010046, 4992.2486445538634};
static const double kBigRest[3][7] = {
    {-1.025, -0.78, -0.65012, -0.19041574084286472, -0.20819395464, -0.421064,
     -0.32733845535848671},
    {-0.3041958212306401, -0.3633036457487539, -0.35660379990111464, -0.3443074455424403,
     -0.33699592683512467, -0.30180866526242109, -0.27321683125358037},
    {-1.2, -1.2, -0.8, -0.7, -0.7, -0.4, -0.5}};
static const double kBigScale[4] = {1.3, 1.7, 2.2, 3.0};
static double big_param(int k, int c, int i) {
  if (i) return f16_round(kBigRest[c][i - 1]);
  return 64.0 * f16_round(kBigScale[k] * ((k & 1) ? kBigY64[c] : kBigY32[c]) / 64.0);
}

void write_dequant_matrices(BitWriter& w, uint32_t mask) {
  if (!mask) {
    w.put(1, 1);  // all_default
    return;
  }
  // quant table order DCT, IDENTITY, DCT2X2, DCT4X4, DCT16X16, DCT32X32,
  // DCT16X8, DCT32X8, DCT32X16, DCT64X64, DCT64X32, DCT4X8, AFV0, DCT128X128,
  // DCT128X64, DCT256X256, DCT256X128 -> big kind (0 128X64, 1 128X128,
  // 2 256X128, 3 256X256) or -1 (Library)
  static const int kTableBig[17] = {-1, -1, -1, -1, -1, -1, -1, -1, -1,
                                    -1, -1, -1, -1, 1,  0,  3,  2};
  w.put(1, 0);
  for (int t = 0; t < 17; t++) {
    const int k = kTableBig[t];
    if (k < 0 || !(mask >> k & 1)) {
      w.put(3, 0);  // Library
      continue;
    }
    w.put(3, 6);      // DCT
    w.put(4, 8 - 1);  // bands
    for (int c = 0; c < 3; c++)
      for (int i = 0; i < 8; i++) {
        const double v = big_param(k, c, i);
        w.put(16, f16_bits(i ? v : v / 64.0));
      }
  }
}

BigTables build_big_tables() {
  static const int kDims[4][2] = {{64, 128}, {128, 128}, {128, 256}, {256, 256}};
  BigTables T;
  const size_t n = kBigKindOff[4];
  T.tab.assign(kBigTabFloats, 0.0f);
  T.nat.assign(n, 0);
  for (int k = 0; k < 4; k++) {
    const int rows = kDims[k][0], cols = kDims[k][1], nb = 8, off = kBigKindOff[k];
    for (int c = 0; c < 3; c++) {
      double bands[8];
      bands[0] = big_param(k, c, 0);
      for (int i = 1; i < nb; i++) {
        const double v = big_param(k, c, i);
        bands[i] = bands[i - 1] * (v > 0 ? 1.0 + v : 1.0 / (1.0 - v));
      }
      const double scale = (nb - 1) / (1.4142135623730951 + 1e-6);
      const double rc = scale / (cols - 1), rr = scale / (rows - 1);
      for (int y = 0; y < rows; y++)
        for (int x = 0; x < cols; x++) {
          const double dx = x * rc, dy = y * rr;
          const double pos = std::sqrt(dx * dx + dy * dy);
          int idx = (int)pos;
          if (idx > nb - 2) idx = nb - 2;
          const double frac = pos - idx;
          const double a = bands[idx], b = bands[idx + 1];
          const float w = (float)(a * std::pow(b / a, frac));
          T.tab[kBigTabW + (size_t)c * n + off + y * cols + x] = w;
          T.tab[kBigTabSd + (size_t)c * n + off + y * cols + x] = dist_weight(c, rows * cols, w);
          if (c == 1) T.tab[kBigTabIw + off + y * cols + x] = 1.0f / w;
        }
    }
    uint16_t* nat = &T.nat[off];
    const int cs = rows / 8, cl = cols / 8, xf = cols / rows;
    int cur = 0;
    for (int y = 0; y < cs; y++)
      for (int x = 0; x < cl; x++) nat[y * cols + x] = (uint16_t)cur++;
    auto visit = [&](int x, int y, bool skip_llf) {
      if (y % xf) return;
      y /= xf;
      if (skip_llf && x < cl && y < cs) return;
      nat[y * cols + x] = (uint16_t)cur++;
    };
    for (int i = 0; i < cols; i++)
      for (int j = 0; j <= i; j++) {
        const bool odd = i & 1;
        visit(odd ? i - j : j, odd ? j : i - j, true);
      }
    for (int ip = cols - 1; ip > 0; ip--) {
      const int i = ip - 1;
      for (int j = 0; j <= i; j++) {
        const int x = cols - 1 - (i - j), y = cols - 1 - j;
        const bool odd = i & 1;
        visit(odd ? y : x, odd ? x : y, false);
      }
    }
  }
  const double pi = 3.14159265358979323846;
  for (int l = 0; l < 9; l++) {
    const int N = 1 << l;
    for (int i = 0; i < N / 2; i++)
      T.tab[kBigTabLeeC + l * 128 + i] = (float)(1.0 / (2.0 * std::cos(pi * (2 * i + 1) / (2.0 * N))));
    for (int k = 0; k < N; k++)
      T.tab[kBigTabLeeS + l * 256 + k] = (float)(k ? std::sqrt(2.0) / N : 1.0 / N);
  }
  for (int l = 0; l < 6; l++) {
    const int M = 1 << l;
    for (int k = 0; k < M; k++)
      T.tab[kBigTabLlfP + l * 32 + k] = (float)(std::cos(pi * k / (16.0 * M)) *
                                                std::cos(pi * k / (8.0 * M)) *
                                                std::cos(pi * k / (4.0 * M)));
    for (int nn = 0; nn < M; nn++)
      for (int k = 0; k < M; k++)
        T.tab[kBigTabLlfIb + (l * 32 + nn) * 32 + k] =
            (float)(k ? std::sqrt(2.0) * std::cos(pi * (2 * nn + 1) * k / (2.0 * M)) : 1.0);
  }
  return T;
}

}  // namespace jxg
