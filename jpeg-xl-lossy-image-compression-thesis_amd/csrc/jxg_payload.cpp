// jxg_payload.cpp -- payload heads of sharded frames (jxg_payload.h)
#include "jxg_payload.h"

#include <cstring>

#include "jxg_bitstream.h"
#include "jxg_device.h"
#include "jxg_tables.h"

namespace jxg {

size_t head_words(const uint32_t* hw, size_t avail) {
  if (avail < 7 || hw[0] != kPayloadMagic) return 0;
  const size_t base = 7 + 2 * (size_t)hw[6];
  if (hw[1] == 1) return base;
  if (hw[1] != 2 || avail < base + 1) return 0;
  return base + 1 + hw[base];
}

// HfGlobal of a frame sharded with one HF preset per rank (payload heads of
// version 2): num_hf_presets = ranks, one context map over every preset's
// contexts (rank r's clusters after those of ranks < r), every rank's ANS
// histograms rebuilt from its clustered counts [ext HfGlobal / HfPass]
static jxg_status build_hf_presets(const std::vector<std::vector<uint32_t>>& heads,
                                   uint32_t ngroups, uint32_t big, BitWriter& hf) {
  const uint32_t n = (uint32_t)heads.size();
  const size_t cw = (kAcCtx + 3) / 4;
  std::vector<uint8_t> ctxmap((size_t)n * kAcCtx);
  std::vector<AnsTable> tables;
  uint32_t off = 0;
  for (uint32_t r = 0; r < n; r++) {
    const std::vector<uint32_t>& hw = heads[r];
    const size_t base = 7 + 2 * (size_t)hw[6];
    if (hw[1] != 2 || hw.size() < base + 2) return JXG_ERR_INVALID_ARG;
    const uint32_t B = hw[base], nh = hw[base + 1];
    if (nh < 1 || nh > (uint32_t)kAnsMaxHists || B != 1 + cw + nh * kAlpha ||
        hw.size() != base + 1 + B)
      return JXG_ERR_INVALID_ARG;
    const uint8_t* cm = reinterpret_cast<const uint8_t*>(hw.data() + base + 2);
    for (int k = 0; k < kAcCtx; k++) {
      if (cm[k] >= nh) return JXG_ERR_INVALID_ARG;
      ctxmap[(size_t)r * kAcCtx + k] = (uint8_t)(off + cm[k]);
    }
    const uint32_t* cnt = hw.data() + base + 2 + cw;
    for (uint32_t h = 0; h < nh; h++) tables.push_back(build_ans_table(cnt + (size_t)h * kAlpha, false));
    off += nh;
  }
  if (off > 255 || n - 1 >= (1u << ceil_log2(ngroups))) return JXG_ERR_INVALID_ARG;
  write_dequant_matrices(hf, big);         // DequantMatrices
  hf.put(ceil_log2(ngroups), n - 1);     // num_hf_presets - 1
  write_u32_sel(hf, 2, 0, 0);              // used_orders = 0
  write_ans_histograms(hf, ctxmap, (int)off, tables, kCfg420, nullptr);
  return JXG_OK;
}

// hf: with version-2 heads, the generated HfGlobal (section 1 + nlf, whose
// SectionRef then names payload n = "generated")
jxg_status parse_payload_heads(const std::vector<std::vector<uint32_t>>& heads,
                                      const std::vector<size_t>& psizes, uint32_t* w,
                                      uint32_t* h, std::vector<SectionRef>& secs,
                                      std::vector<uint8_t>& hf, uint32_t* lf, bool hf_bytes) {
  const uint32_t n = (uint32_t)heads.size();
  secs.clear();
  hf.clear();
  std::vector<bool> seen;
  for (uint32_t i = 0; i < n; i++) {
    const std::vector<uint32_t>& hw = heads[i];
    if (hw.size() < 7 || hw[0] != kPayloadMagic || (hw[1] != 1 && hw[1] != 2) ||
        hw[1] != heads[0][1] || hw[3] != n)
      return JXG_ERR_INVALID_ARG;
    // bits 16-23: loop-filter code (equal over the ranks), bits 24-27: the
    // big kinds of the rank's groups (shard_finish; their union is written)
    if (i == 0) {
      *w = hw[4];
      *h = hw[5];
      *lf = (hw[2] >> 16) & 0xFFu;
    } else if (hw[4] != *w || hw[5] != *h || ((hw[2] >> 16) & 0xFFu) != *lf) {
      return JXG_ERR_INVALID_ARG;
    }
    const size_t hwords = head_words(hw.data(), hw.size());
    if (!hwords || hw.size() != hwords) return JXG_ERR_INVALID_ARG;
    uint64_t off = 4 * (uint64_t)hwords;  // the body follows the whole head
    for (uint32_t k = 0; k < hw[6]; k++) {
      const uint32_t id = hw[7 + 2 * k], sz = hw[8 + 2 * k];
      if (off + sz > psizes[i]) return JXG_ERR_INVALID_ARG;
      if (id >= secs.size()) {
        secs.resize(id + 1, SectionRef{0, 0, 0});
        seen.resize(id + 1, false);
      }
      if (seen[id]) return JXG_ERR_INVALID_ARG;  // section twice
      seen[id] = true;
      secs[id] = SectionRef{i, off, sz};
      off += sz;
    }
  }
  uint32_t big = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (heads[i][2] >> 28) return JXG_ERR_INVALID_ARG;
    big |= heads[i][2] >> 24;
  }
  if (*w == 0 || *h == 0 || *lf > 7) return JXG_ERR_INVALID_ARG;
  const uint32_t ngroups = ((*w + 255) / 256) * ((*h + 255) / 256);
  const uint32_t nlf = ((*w + 2047) / 2048) * ((*h + 2047) / 2048);
  if (secs.size() != 2 + nlf + ngroups) return JXG_ERR_INVALID_ARG;
  if (heads[0][1] == 2) {  // per-rank presets: HfGlobal from the heads
    const uint32_t id = 1 + nlf;
    if (seen[id]) return JXG_ERR_INVALID_ARG;
    // (a rank that does not write HfGlobal needs its size only)
    BitWriter bw = hf_bytes ? BitWriter() : BitWriter::counter();
    const jxg_status st = build_hf_presets(heads, ngroups, big, bw);
    if (st) return st;
    if (hf_bytes) hf = bw.bytes();
    secs[id] = SectionRef{n, 0, (uint32_t)((bw.bits() + 7) / 8)};
    seen[id] = true;
  }
  for (size_t i = 0; i < secs.size(); i++)
    if (!seen[i]) return JXG_ERR_INVALID_ARG;  // section missing
  return JXG_OK;
}

std::vector<uint32_t> read_head(const uint8_t* p, size_t size) {
  if (size < 28) return {};
  std::vector<uint32_t> hw(7);
  std::memcpy(hw.data(), p, 28);
  const size_t base = 7 + 2 * (size_t)hw[6];
  if (hw[1] == 2 && size >= (base + 1) * 4) {  // version 2: the preset block's length
    hw.resize(base + 1);
    std::memcpy(hw.data(), p, (base + 1) * 4);
  }
  const size_t words = head_words(hw.data(), hw.size());
  if (!words || size < words * 4) return {};
  hw.resize(words);
  std::memcpy(hw.data(), p, words * 4);
  return hw;
}

}  // namespace jxg
