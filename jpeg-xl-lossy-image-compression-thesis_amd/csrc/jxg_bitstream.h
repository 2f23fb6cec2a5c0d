// jxg_bitstream.h -- host-side codestream writing: bit writer, prefix-code
// construction and serialisation, entropy-code headers, modular trees,
// image / frame headers and TOC.  [ext] JPEG XL codestream layout
// (ISO/IEC 18181-1); the byte-level contract is shared with the CPU oracle
// (oracle/encode.c, oracle/entropy.c) and checked bit-for-bit by the tests.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <array>
#include <vector>

namespace jxg {

class BitWriter {
 public:
  // a counting writer: put() only advances bits() (sizes without the bytes)
  static BitWriter counter() {
    BitWriter w;
    w.count_only_ = true;
    return w;
  }
  bool count_only() const { return count_only_; }
  void skip(size_t nbits) { bits_ += nbits; }  // (count-only writers)
  void put(uint32_t nbits, uint64_t v) {
    if (count_only_) {
      bits_ += nbits;
      return;
    }
    if (nbits == 0) return;
    if (nbits < 64) v &= (1ull << nbits) - 1;
    const size_t word = bits_ >> 6;
    const uint32_t off = (uint32_t)(bits_ & 63);
    if (word + 2 > words_.size()) words_.resize(word + 2 + words_.size() / 2, 0);
    words_[word] |= v << off;
    if (off && off + nbits > 64) words_[word + 1] |= v >> (64 - off);
    bits_ += nbits;
  }
  void pad_to_byte() { bits_ = (bits_ + 7) & ~(size_t)7; }
  size_t bits() const { return bits_; }
  // little-endian 32-bit words holding the bits (tail zero)
  std::vector<uint32_t> words32() const {
    std::vector<uint32_t> w((bits_ + 31) / 32, 0);
    for (size_t i = 0; i < w.size(); i++) w[i] = (uint32_t)(words_[i / 2] >> (32 * (i & 1)));
    return w;
  }
  std::vector<uint8_t> bytes() const {
    std::vector<uint8_t> b((bits_ + 7) / 8);
    for (size_t i = 0; i < b.size(); i++) b[i] = (uint8_t)(words_[i / 8] >> (8 * (i & 7)));
    return b;
  }
  void append(const BitWriter& o) {
    for (size_t i = 0; i < o.bits_; i += 64) {
      const uint32_t n = (uint32_t)(o.bits_ - i < 64 ? o.bits_ - i : 64);
      put(n, o.words_[i / 64]);
    }
  }

 private:
  std::vector<uint64_t> words_;
  size_t bits_ = 0;
  bool count_only_ = false;
};

struct UintCfg {
  uint32_t split_exp, msb, lsb;
};
constexpr UintCfg kCfg420{4, 2, 0};
constexpr UintCfg kCfgMap{8, 0, 0};

void hybrid_encode(uint32_t v, const UintCfg& c, uint32_t* tok, uint32_t* nb, uint32_t* bits);

// A Brotli-style prefix code over at most 256 symbols.
struct PrefixCode {
  uint32_t alphabet = 1;  // serialised alphabet size
  int nsym = 0;           // used symbols
  int simple = 0;         // simple-code NSYM (1..4) or 0 for a complex code
  int tree_select = 0;
  std::array<uint16_t, 4> ssyms{};
  std::array<uint8_t, 256> len{};
  std::array<uint16_t, 256> code{};  // bit-reversed canonical code
  // packed (code | len << 16) for device tables
  uint32_t packed(uint32_t sym) const { return code[sym] | ((uint32_t)len[sym] << 16); }
};
PrefixCode build_prefix_code(const uint32_t* counts, int n);
void write_prefix_code(BitWriter& w, const PrefixCode& p);

void write_token(BitWriter& w, const PrefixCode& p, const UintCfg& c, uint32_t v);
// DecodeHistograms: lz77 off, context map (ctxmap[nctx] dense ids), prefix codes
void write_histograms(BitWriter& w, const std::vector<uint8_t>& ctxmap, int nhist,
                      const std::vector<PrefixCode>& codes, const UintCfg& cfg,
                      const BitWriter* ctxmap_bits = nullptr);
// entropy-coded context map (the part of write_histograms that depends only
// on the map; callers may cache it)
void write_context_map(BitWriter& w, const std::vector<uint8_t>& map, int nhist);

// ANS (12-bit rANS, alias mapping, alphabet 128) for the AC stream: the
// restated encoder choices of oracle/ans.c (normalization, omitted symbol,
// full-precision histograms) -- the device kernels encode with these tables
struct AnsTable {
  std::array<uint16_t, 128> freq{};
  std::array<uint16_t, 128> cum{};
  std::vector<uint16_t> inv;  // [cum[s] + off] -> alias-table position (4096)
  int nused = 0, omit = 0, omit_code = 0;
};
// with_inverse false: the normalized frequencies only (enough to write the
// histogram; the encoder's alias inverse is left empty)
AnsTable build_ans_table(const uint32_t* counts /* [128] */, bool with_inverse = true);
// ANS histogram clustering (oracle/ans.c jxo_ans_cluster): hist[nh][128] ->
// assign[nh] (centre id, -1 for an empty histogram); returns the centre count
// (<= kAnsMaxHists: their alias inverses fill 64 KB of LDS in the encoder, so
// the rANS chain kernel co-resides with the transform kernels of the next
// frame; oracle/jxo_internal.h JXO_ANS_MAX_HISTS)
#ifndef JXG_ANS_HISTS  // (experiment builds override it: tools/build_variant.sh)
#define JXG_ANS_HISTS 8
#endif
constexpr int kAnsMaxHists = JXG_ANS_HISTS;
constexpr int64_t kAnsMinDist = 64ll << 16;  // Q16 bits
int cluster_ans_histograms(const uint32_t* hist, int nh, int* assign);
void write_ans_histogram(BitWriter& w, const AnsTable& t);
// DecodeHistograms for ANS: lz77 off, context map, use_prefix_code = 0,
// log_alpha 7, uint configs, histograms
void write_ans_histograms(BitWriter& w, const std::vector<uint8_t>& ctxmap, int nhist,
                          const std::vector<AnsTable>& tables, const UintCfg& cfg,
                          const BitWriter* ctxmap_bits = nullptr);

// Modular MA trees used by the LF-group streams (local trees, no transforms)
struct TreeNode {
  int prop, splitval, lchild, rchild, predictor, leaf;  // prop < 0: leaf
  int offset;                                          // leaf: value offset
};
extern const TreeNode kDcTree[5];
extern const TreeNode kMetaTree[7];
extern const TreeNode kMetaTreeEpf[7];  // the EPF leaf's offset = kEpfSharpness
constexpr int kEpfSharpness = 4;        // [ext] constant EPF sharpness per block
// GroupHeader + tree + data histograms (leaf codes); the residual tokens are
// emitted on the GPU
void write_modular_prelude(BitWriter& w, const TreeNode* tree, int nnodes, int nleaves,
                           const std::vector<PrefixCode>& leaf_codes);

// loop-filter code of the frame header: bit 0 Gaborish, bits 1-2 EPF
// iterations (oracle/xyb.c jxo_lf_code)
uint32_t lf_code(uint32_t flags, float distance);
// SizeHeader + all-default ImageMetadata + byte padding + FrameHeader
void write_headers(BitWriter& w, uint32_t xsize, uint32_t ysize, uint32_t lf = 0);
void write_toc(BitWriter& w, const std::vector<uint32_t>& section_bytes);
void write_u32_sel(BitWriter& w, uint32_t sel, uint32_t nbits, uint32_t v);

inline uint32_t ceil_log2(uint32_t x) {
  uint32_t n = 0;
  while ((1u << n) < x) n++;
  return n;
}

}  // namespace jxg
