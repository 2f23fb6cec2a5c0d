// jxg_tables.h -- host-side constant tables of the encoder (built once per
// process, uploaded to __constant__ / device memory by jxg_host.cpp):
// default quantization weights, the sRGB8 -> linear table, the masking AQ's
// erosion weights, and the merge stage's per-shape weight / distortion /
// natural-order tables and DCT constants.  [ext libjxl quant_weights.cc,
// coeff_order.cc; == oracle/front.c, oracle/merge.c, oracle/aq.c]
#pragma once
#include <cstdint>
#include <vector>

namespace jxg {

struct MergeTables {
  std::vector<float> wk, sdk, iwy;
  std::vector<uint16_t> nat;
  float lee_c[7][32], lee_s[7][64], llf_p[4][8], llf_ib[4][8][8];
};

// kinds: 0 DCT8, 1 DCT4X4, 2 DCT4X8 / DCT8X4, 3 IDENTITY, 4 DCT2X2
void quant_weights(float out[5][3][64]);
void aq_erosion_weights(float distance, float w[4]);
void srgb_lut(float lut[256]);
MergeTables build_merge_tables();
// the 128 / 256 px levels' tables (kBigTab* layout, jxg_kernels.h) and their
// natural orders (== oracle/merge.c kinds 6-9)
struct BigTables {
  std::vector<float> tab;
  std::vector<uint16_t> nat;
};
BigTables build_big_tables();

// DequantMatrices of HfGlobal [ext quant_weights.cc]: all_default when mask is
// 0, else Library for every table but those of the big kinds in mask (bit 0
// 128X64, 1 128X128, 2 256X128, 3 256X256: the kinds the frame uses, effort
// >= 8), which are written in mode DCT with the binary16 parameters
// build_big_tables quantizes with (== oracle/encode.c put_dequant_matrices),
// so no decoder default is involved for them
class BitWriter;
void write_dequant_matrices(BitWriter& w, uint32_t mask);
// the binary16 value nearest v (ties to even) and its bits (== oracle/merge.c)
double f16_round(double v);
uint32_t f16_bits(double v);

}  // namespace jxg
