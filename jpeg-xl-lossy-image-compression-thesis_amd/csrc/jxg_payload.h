// jxg_payload.h -- a rank's payload head (group sharding, include/jxg.h
// jxg_shard_payload): parsing and validation of every rank's heads into the
// frame's section table, the HfGlobal of per-rank HF presets.  Host only;
// the heads are built by jxg_host.cpp shard_finish.
// payload: "JXGS" | version | rank (| loop-filter code << 16) | world | xsize | ysize | nsections |
//          nsections x (TOC index, bytes) [| version 2: the rank's HF preset]
//          | section bytes back to back
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "../../include/jxg.h"

namespace jxg {

constexpr uint32_t kPayloadMagic = 0x5347584Au;  // "JXGS"

// for each TOC index of the frame: (payload, byte offset inside it, size)
struct SectionRef {
  uint32_t payload;
  uint64_t off;
  uint32_t size;
};

// words of a payload head from its first words (avail of them; 0: malformed
// or more words needed to tell -- version 2 needs 7 + 2 nsections + 1)
size_t head_words(const uint32_t* hw, size_t avail);
// every rank's head (psizes: whole payload bytes) -> frame size, loop-filter
// code, section table; with version-2 heads also the generated HfGlobal
// (`hf`; its SectionRef names payload n = "generated"; hf_bytes false: its
// size only, `hf` left empty)
jxg_status parse_payload_heads(const std::vector<std::vector<uint32_t>>& heads,
                               const std::vector<size_t>& psizes, uint32_t* w, uint32_t* h,
                               std::vector<SectionRef>& secs, std::vector<uint8_t>& hf,
                               uint32_t* lf, bool hf_bytes = true);
// the head at the start of a payload in host memory (empty: malformed)
std::vector<uint32_t> read_head(const uint8_t* p, size_t size);

}  // namespace jxg
