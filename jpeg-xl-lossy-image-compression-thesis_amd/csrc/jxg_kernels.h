// jxg_kernels.h -- kernel argument blocks and device-symbol setup shared by
// the HIP translation units and the host orchestrator (jxg_host.cpp).
#pragma once
#include <cmath>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace jxg {

// Batched launches (the streaming pipeline's super-frames): up
// to kMaxBatch frames of one size go through each per-frame kernel as ONE
// launch -- the argument blocks of all of them in the kernel arguments,
// blockIdx.z = the frame.  One-at-a-time encodes launch batches of one.
constexpr uint32_t kMaxBatch = 4;
template <class A>
struct Batch {
  A a[kMaxBatch];
};
template <class A>
inline Batch<A> make_batch(const A* a, uint32_t k) {
  Batch<A> b{};
  for (uint32_t i = 0; i < k && i < kMaxBatch; i++) b.a[i] = a[i];
  return b;
}

struct FrontArgs {
  const uint8_t* rgb;
  uint32_t w, h;
  size_t stride;
  uint32_t bxs, bys, xp, yp, tiles_x;
  float distance;
  int effort;
  uint32_t proposals;
  int h1_int;
  int gab;        // inverse Gaborish on the XYB tile before every other stage
  float qf_base, inv_g;
  uint32_t G;
  float dc_mul[3], dc_step[3];
  uint8_t* acs;   // [nb] raw strategy
  uint8_t* qf;    // [nb] raw-1
  int32_t* dc;    // [3][nb] X,Y,B
  int16_t* ac;    // [nb][3 X,Y,B][64 zigzag]
  uint16_t* nz;   // [3][nb] non-zero AC count per block and channel
  float* homog;   // [nb][3] or null
  float* ent;     // [nb] best 8x8 estimate (merge stage input) or null
  float* xyb_out; // [tiles][3][64][64] XYB tiles (merge stage input) or null
  const uint32_t* tile_list;  // shard: tile ids (ty * tiles_x + tx), 1-D grid; or null
  int8_t* cmap;   // [2][tiles] chroma from luma ytox, ytob per 64x64 tile (out)
  uint32_t ntiles_all;  // tiles_x * tiles_y (cmap plane stride)
  uint4* zero;          // the frame's statistics arena, zeroed by the workgroups (or null)
  uint32_t zero_quads;  //   its size in 16-byte units
  const uint8_t* qf_in; // [nb] raw - 1 of the masking quant field (jxg_aq.hip), or null:
                        //   the activity heuristic
};
// libjxl-shaped masking quant field (jxg_aq.hip, oracle/aq.c)
struct AqArgs {
  const uint8_t* rgb;
  uint32_t w, h;
  size_t stride;
  uint32_t xp, yp, bxs, bys, tiles_x;
  const float* lut;      // [256] sRGB8 -> linear (device)
  float ew[4];           // fuzzy-erosion weights (aq_erosion_weights)
  float mul, add, inv_g; // quant field = pow2(...) mul + add; raw = round(qf inv_g)
  uint8_t* qf;           // [nb] raw - 1 (out)
  const uint32_t* tile_list;  // shard: tile ids, or null: every tile (1-D grid)
};
void launch_aq(const AqArgs* a, uint32_t k, uint32_t ntiles, hipStream_t s);

// merge stage (jxg_merge.hip): weight kinds (stored orientation) and the
// nine merged shapes' pixel-orientation tables, column-major ([kx * R + ky])
constexpr int kNumKinds = 6;
constexpr int kKindOff[kNumKinds + 1] = {0, 128, 384, 896, 1920, 3968, 8064};
constexpr int kNumShapes = 9;
constexpr int kShapeOff[kNumShapes + 1] = {0, 128, 256, 512, 1024, 1536, 2560, 4608, 6656, 10752};
struct MergeArgs {
  const float* xyb;     // [tiles][3][64][64] XYB tiles (front kernel)
  uint32_t bxs, bys, tiles_x, ntiles;  // ntiles: entries of tile_list (or all tiles)
  const uint32_t* tile_list;           // shard: tile ids, or null
  uint32_t proposals;
  int max_s;      // largest merged square in blocks (2, 4 or 8)
  uint32_t G;
  float dc_mul[3], dc_step[3];
  float* ent;           // [nb] per-block estimate (front kernel; resolve rewrites)
  const float* homog;   // [nb][3] (hook F) or null
  uint8_t* acs;         // in/out: raw id, bit 7 on covered non-first blocks
  uint8_t* qf;          // in/out: raw - 1
  int32_t* dc;          // out (merged varblocks)
  int16_t* ac;          // out (merged varblocks), natural order slices
  uint16_t* nz;         // out (merged varblocks): full count at the first block,
                        //   (nz + cb - 1) >> log2 cb at covered blocks
  float* cost;          // [tiles][9 shapes][32 varblocks] candidate estimates
  const float* wk;      // [3][kShapeOff[9]] weights per shape, pixel orientation, row quads ([ky/4][kx][ky%4])
  const float* iwy;     // [kShapeOff[9]] 1 / Y weight
  const float* sdk;     // [3][kShapeOff[9]] distortion weights (dist_weight), same layout
  const uint16_t* nat;  // [kShapeOff[9]] natural-order position
  uint32_t* work;       // [1 + tiles * 9]: count, then (tile << 4 | shape) of every
                        //   (tile, shape) holding a chosen varblock (resolve -> write)
  uint32_t nwrite;      // merge_write workgroups (persistent loop over work)
  const int8_t* cmap;   // [2][tiles_all] chroma from luma (front kernel)
  uint32_t ntiles_all;
};
// merge levels 128 / 256 px (effort >= 8; jxg_bigvb.hip): kinds 64x128,
// 128x128, 128x256, 256x256 (stored orientation rows <= cols), and the
// layout of their table blob (floats): weights [3][n], distortion weights
// [3][n], 1 / Y weight [n], Lee constants [9][128] / scales [9][256], LLF
// scales [6][32] and inverse basis [6][32][32]; natural orders separately
constexpr int kBigKindOff[5] = {0, 8192, 24576, 57344, 122880};
constexpr uint32_t kBigSlots = 512;          // persistent workgroups of the 128 / 256 px levels (two per CU)
constexpr size_t kBigPlanes = 3 * 65536;     // floats of a slot's scratch: X, Y, B planes of up to 256 x 256
constexpr size_t kBigTabW = 0, kBigTabSd = 3 * 122880, kBigTabIw = 6 * 122880,
                 kBigTabLeeC = 7 * 122880, kBigTabLeeS = kBigTabLeeC + 9 * 128,
                 kBigTabLlfP = kBigTabLeeS + 9 * 256, kBigTabLlfIb = kBigTabLlfP + 6 * 32,
                 kBigTabFloats = kBigTabLlfIb + 6 * 32 * 32;
struct BigArgs {
  MergeArgs m;             // the frame's merge arguments (xyb tiles, maps, outputs)
  const float* tab;        // kBigTab* blob
  const uint16_t* nat;     // [kBigKindOff[4]] natural-order position per stored index
  float* scratch;          // [slots][3][65536] column-major planes X, Y (dequantized after its quantization), B
  uint32_t slots;          // persistent workgroups (one scratch slot each)
  float* cost;             // [ng][30] candidate estimates (level 128: 4 x 5, level 256: 5), the regions' current sums (4 + 1)
  uint32_t* work;          // [1 + ng * 16]: count, then first blocks of the chosen varblocks
  uint32_t* kinds;         // [4] varblocks chosen per big kind (statistics arena; the host writes the used kinds' quant tables)
  const uint32_t* glist;   // the plan's pass groups: glist[i], or g0 + i
  uint32_t g0, ng, gxs;
};
hipError_t launch_big(const BigArgs* a, uint32_t k, hipStream_t s);

// per-LF-group varblock lists (AC metadata channel)
struct VbArgs {
  const uint8_t* acs;
  uint32_t bxs, bys, lfxs;
  const uint8_t* lf_mine;  // [nlf] 1 = this shard owns the LF group (null: all)
  uint32_t* vb;     // [nlf][65536] block index (frame raster) of each varblock
  uint32_t* count;  // [nlf]
};

struct HomogArgs {
  const float* xyb;  // [3][ysize][stride]
  uint32_t xsize, ysize;
  size_t stride, plane;
  float distance;
  int h1_int;
  float* r3;
  uint8_t* type;
};

// AC (pass group) token kernels
struct AcArgs {
  const uint8_t* acs;
  const int16_t* ac;  // [nb][3][64 zigzag]
  const uint16_t* nz;  // [3][nb] non-zero counts (front / merge kernels)
  uint32_t bxs, bys, gxs;
  uint32_t g0;           // first pass group of the launch (contiguous shard / whole frame)
  const uint32_t* glist; // [slots] pass group of each slot (a shard's non-contiguous
                         //   group set), or null: slot i = group g0 + i
  uint32_t* hist;        // [kMaxClusters][kAlpha]      (hist pass)
  uint32_t* bound;       // [ngroups] bit upper bound   (hist pass)
  uint32_t* ntok;        // [ngroups][3] token counts   (hist pass)
  const uint32_t* codes; // [kMaxClusters][kAlpha] (code | len << 16)  (emit pass)
  const uint64_t* base;  // [ngroups] scratch bit offset (emit pass)
  uint32_t* scratch;     // bit buffer (emit pass, zeroed)
  uint32_t* bits;        // [ngroups] exact bits (emit pass)
  uint32_t* tokens;      // token records (cluster | tok << 8 | nbits << 14 | bits << 18),
                         //   slot i (group glist[i] or g0 + i) at i * kGroupTokStride,
                         //   band j of it at + j * kBandTokStride (hist pass writes them)
  uint32_t* bandtok;     // [ngroups][4] tokens of each 8-block-row band (hist pass)
};
// records per pass group: 1024 blocks x 3 channels x <= 64 tokens per slice;
// per band (8 of the group's 32 block rows): a quarter of that
constexpr uint64_t kGroupTokStride = 1024ull * 3 * 64;
constexpr uint64_t kBandTokStride = 256ull * 3 * 64;

// ANS coding of the pass groups' token records (jxg_ac.hip)
#ifndef JXG_ANS_HISTS  // (jxg_bitstream.h kAnsMaxHists; experiment builds override it)
#define JXG_ANS_HISTS 8
#endif
constexpr uint32_t kAnsHists = JXG_ANS_HISTS;  // == kAnsMaxHists (jxg_bitstream.h)
constexpr uint32_t kAnsInvOff = kAnsHists * 128 * 4;
constexpr uint32_t kAnsMapOff = kAnsInvOff + kAnsHists * 4096 * 2;
constexpr uint32_t kAnsTabBytes = kAnsMapOff + 136;
struct AnsArgs {
  const uint32_t* tokens;  // token records of ac_hist_kernel (kGroupTokStride per group)
  uint32_t* val;           // [records] emitted bits: 16-bit chunk (if any) then raw bits
  uint8_t* len;            // [records] number of emitted bits
  const uint32_t* ntok;    // [ngroups][3]
  const uint32_t* bandtok; // [ngroups][4] tokens per band (the group's stream = its bands')
  const uint8_t* tab;      // table blob (kAnsInvOff / kAnsMapOff):
                           //  u32 [8][128] symbol: f - 1 | cum << 12
                           //  u16 [8][4096] alias inverse: slot of position cum + offset
                           //  u8 [132] static cluster -> histogram
  uint32_t nhist;          // histograms in use (<= kAnsMaxHists)
  uint32_t* state;         // [ngroups] final encoder state (= stream's first 32 bits)
  const uint64_t* base;    // [ngroups] scratch bit offset
  uint32_t* scratch;
  uint32_t* bits;          // [ngroups] exact bits
  uint32_t g0, n;          // slots [0, n): group glist[i], or g0 + i when glist is null
  const uint32_t* glist;
  const uint32_t* order;   // chain order of the n slots (longest group first)
  uint32_t* csum;          // [slots][kAnsMaxChunks] emitted bits of every 64-record chunk
  uint32_t max_tokens;     // most tokens of any group (ans_emit's segments per group)
};
constexpr uint32_t kAnsMaxChunks = (uint32_t)(kGroupTokStride / 64);
// rANS chains + bit placement of k frames (same plan)
void launch_ans(const AnsArgs* a, uint32_t k, hipStream_t s);

// LF-group modular streams: rows of (lf group, stream, channel, y)
// One segment of <= kLfSeg samples of a channel row (long rows -- the
// 2 x count AC-strategy/quant-field channel -- are split so every workgroup
// does one pass).
constexpr uint32_t kLfSeg = 256;
struct LfRow {
  uint32_t lg;      // LF group
  uint16_t stream;  // 0 = DC, 1 = AC metadata
  uint16_t chan;
  uint32_t y, x0, width;  // samples [x0, x0 + width) of row y
  uint32_t sid;           // stream index = lg*2 + stream
};
// A chunk: consecutive segments of ONE stream, <= kLfChunkSamples samples
// and <= kLfChunkRows segments; one workgroup (256 threads, <= 16 samples
// each, contiguous in stream order) per chunk.
constexpr uint32_t kLfChunkSamples = 4096, kLfChunkRows = 64, kLfPer = 16;
struct LfChunk {
  uint32_t row0, nrows, sid, nsamp;
};
struct LfArgs {
  const LfRow* rows;
  const LfChunk* chunks;
  const int32_t* dc;  // [3][nb]
  const uint8_t* acs;
  const uint8_t* qf;
  const uint32_t* vb;     // [nlf][65536] varblock -> block index
  const uint32_t* vcount; // [nlf] varblocks per LF group
  uint32_t bxs, bys, lfxs;
  const int8_t* cmap;     // [2][tiles_y][tiles_x] ytox, ytob (AC metadata channels 0, 1)
  uint32_t tiles_x, ntiles_all;
  uint32_t* hist;         // [nstreams][4 leaves][kAlpha]  (hist)
  uint32_t* sbound;       // [nstreams] (hist)
  const uint32_t* codes;  // [nstreams][4][kAlpha] (lf_code)
  uint64_t* status;       // [nchunks] look-back word (lf_hist clears, lf_code)
  const uint32_t* stream_chunks;  // [nstreams+1] first chunk of each stream
  const uint64_t* stream_base;  // [nstreams] scratch bit offset of each stream
  uint32_t* stream_bits;        // [nstreams] exact bits (lf_code)
  uint32_t* scratch;
};

struct ConcatPiece {
  uint64_t src_bit;  // bit offset into the source arena
  uint64_t dst_bit;  // bit offset into the output
  uint64_t nbits;
  uint32_t arena;    // 0 = device scratch, 1 = host-chunk upload, 2 = second scratch
  uint32_t pad;
};

// distortion weight of a coefficient in the strategy search's estimates
// (== oracle/front.c jxo_dist_weight): sqrt(area / 64) * w0[c] / w, in
// double, rounded once; w0 = the DCT8 band-0 weights of X, Y, B
inline float dist_weight(int c, int area, float w) {
  static const float kW0[3] = {3150.0f, 560.0f, 512.0f};
  return (float)(std::sqrt((double)area / 64.0) * ((double)kW0[c] / (double)w));
}
hipError_t set_front_constants(const float lut[256], const float wts[5][3][64], hipStream_t s);
void launch_front(const FrontArgs* a, uint32_t k, uint32_t tiles_x, uint32_t tiles_y, hipStream_t s);
void launch_front_list(const FrontArgs* a, uint32_t k, uint32_t ntiles, hipStream_t s);
// shard exchange: per-group block records (acs, qf, dc) <-> frame arrays
struct PackArgs {
  uint8_t* acs;
  uint8_t* qf;
  int32_t* dc;
  uint32_t bxs, bys, gxs;
  int8_t* cmap;           // [2][ntiles_all] chroma from luma of the group's 4 x 4 tiles
  uint32_t tiles_x, tiles_y;
  uint8_t* xbuf;          // n group records back to back
  const uint32_t* list;   // [n] group of each record
  uint32_t n;
};
void launch_pack(const PackArgs& a, hipStream_t s);    // frame arrays -> records
// a rank's sections (runs of consecutive section bytes of its payload body)
// -> their codestream offsets in mapped host memory; piece i takes workgroups
// [wg0, next wg0) of 1024 destination dwords each
struct ScatterPiece {
  uint64_t src, dst;
  uint32_t len, wg0;
};
constexpr int kMaxScatterPieces = 64;
struct ScatterArgs {
  const uint8_t* src;
  uint8_t* dst;
  uint32_t n;
  ScatterPiece p[kMaxScatterPieces];
};
void launch_scatter(const ScatterArgs& a, uint32_t nwg, hipStream_t s);
void launch_unpack(const PackArgs& a, hipStream_t s);  // records -> frame arrays
void launch_homog(const HomogArgs& a, uint32_t tiles_x, uint32_t tiles_y, hipStream_t s);
// whole_group: one 1024-thread workgroup per group (varblocks of 128 / 256 px
// span the 8-row bands; effort >= 8)
void launch_ac_hist(const AcArgs* a, uint32_t k, uint32_t ngroups, hipStream_t s,
                    bool whole_group = false);
void launch_ac_emit(const AcArgs& a, uint32_t ngroups, hipStream_t s);
void launch_lf_hist(const LfArgs* a, uint32_t k, uint32_t nchunks, hipStream_t s);
void launch_lf_code(const LfArgs* a, uint32_t k, uint32_t nchunks, hipStream_t s);
hipError_t set_cluster_table(const uint8_t* tab, hipStream_t s);
hipError_t set_merge_constants(const float* llf_p /*[4][8]*/, const float* llf_ib /*[4][8][8]*/,
                         hipStream_t s);
hipError_t launch_merge(const MergeArgs* a, uint32_t k, hipStream_t s);
void dump_merge_profile();  // JXG_MERGE_PROFILE experiment builds; no-op otherwise
void dump_front_profile();  // JXG_FRONT_PROFILE experiment builds; no-op otherwise
void dump_hist_profile();   // (the same builds: ac_hist's phase clock)
void launch_vb_list(const VbArgs* a, uint32_t k, uint32_t nlf, hipStream_t s);
// decode-side quality (jxg_metrics.hip): orig / comp RGB8 interleaved rows
struct MetricArgs {
  const uint8_t* orig;
  const uint8_t* comp;
  size_t so, sc;  // row strides (bytes)
  uint32_t w, h;
  uint64_t* sse;      // out: sum of squared sample differences (pre-zeroed)
  double* partials;   // [ssim_partials(w, h)] per-workgroup SSIM sums
  double* ssim;       // out: sum of window SSIMs over all channels, or null (skip SSIM)
};
uint32_t ssim_partials(uint32_t w, uint32_t h);
hipError_t set_gauss_table(const double* g, hipStream_t s);
void launch_metrics(const MetricArgs& a, hipStream_t s);
// synthetic benchmark input (jxg_synth.hip): RGB8 rows of `stride` bytes
hipError_t launch_synth(uint8_t* out, uint32_t w, uint32_t h, size_t stride, uint64_t seed,
                        hipStream_t s);
// every word of out[0, out_words) written once (bits no piece covers: 0)
void launch_concat(const ConcatPiece* pieces, uint32_t npieces, uint64_t out_words,
                   const uint32_t* scratch, const uint32_t* chunks, const uint32_t* scratch2,
                   uint32_t* out, hipStream_t s);

}  // namespace jxg
