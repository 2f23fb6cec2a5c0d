// jxg_host.cpp -- host orchestration and the C ABI (include/jxg.h).
//
// One encode = one stream-ordered pipeline on the context's HIP stream:
//   front (RGB8 -> ACS/QF/DC/AC)            [jxg_front.hip]
//   ac_hist + lf_hist (token statistics)     [jxg_entropy.hip]
//   -> D2H histograms; host builds prefix codes, LfGlobal/HfGlobal and the
//      LF-group stream preludes (a few KB of header bits)
//   ac_emit or the rANS chain + ans_emit, lf_code (bit emission into scratch)
//   -> D2H section sizes; host writes headers + TOC and the piece list
//   concat (bit-exact assembly) -> D2H codestream
// The byte stream equals the CPU oracle's (oracle/encode.c) bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/jxg.h"
#include "jxg_bitstream.h"
#include "jxg_device.h"
#include "jxg_kernels.h"
#include "jxg_helpers.h"
#include "jxg_payload.h"
#include "jxg_tables.h"

namespace jxg {

#define JXG_HIP(expr)                                                          \
  do {                                                                         \
    hipError_t e_ = (expr);                                                    \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "jxg: %s failed: %s\n", #expr, hipGetErrorString(e_)); \
      return JXG_ERR_HIP;                                                      \
    }                                                                          \
  } while (0)

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  bool n_grow = false;  // allocated before
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    // a regrowth gets 1/8 headroom: per-frame sizes (bit scratch, output)
    // vary a little between frames, and a reallocation in a streamed frame
    // costs ~0.1 ms of host time (hipFree + hipMalloc)
    size_t want = n_grow ? std::max<size_t>(count + count / 8, 1) : std::max<size_t>(count, 1);
    n_grow = true;
    hipError_t e = hipMalloc((void**)&p, want * sizeof(T));
    if (e == hipSuccess) n = want;
    return e;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

static_assert(kAnsHists == (uint32_t)kAnsMaxHists, "ANS table blob sized for kAnsMaxHists");

// A typed window into an arena (Ctx::stat / up and their host mirrors): the
// arena is laid out per frame by stage_alloc, so ensure() only checks.
template <class T>
struct View {
  T* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t count) const { return count <= n ? hipSuccess : hipErrorInvalidValue; }
  void set(void* base, size_t byte_off, size_t count) {
    p = reinterpret_cast<T*>(static_cast<uint8_t*>(base) + byte_off);
    n = count;
  }
};

template <class T>
struct PinBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    size_t want = std::max<size_t>(count, 1);
    hipError_t e = hipHostMalloc((void**)&p, want * sizeof(T), hipHostMallocDefault);
    if (e == hipSuccess) n = want;
    return e;
  }
  ~PinBuf() {
    if (p) (void)hipHostFree(p);
  }
};

// Output codestreams live in pinned host blocks so the final D2H copy lands
// in the caller's buffer directly (no bounce copy, no first-touch page
// faults).  Blocks carry a small header and are recycled through a
// process-wide pool by jxg_buffer_free.
struct OutHeader {
  uint64_t magic;
  size_t cap;     // usable bytes after the header
  uint64_t heap;  // 1: plain heap block (host-only paths), 0: pinned
};
constexpr uint64_t kOutMagic = 0x6a78674f75744275ull;  // "jxgOutBu"
constexpr size_t kOutHdr = 64;
static std::mutex g_pool_mu;
static std::vector<uint8_t*> g_pool;  // free blocks (header addresses)

static uint8_t* out_alloc(size_t bytes) {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    size_t best = g_pool.size();
    for (size_t i = 0; i < g_pool.size(); i++) {
      const size_t cap = reinterpret_cast<OutHeader*>(g_pool[i])->cap;
      if (cap >= bytes && (best == g_pool.size() ||
                           cap < reinterpret_cast<OutHeader*>(g_pool[best])->cap))
        best = i;
    }
    if (best < g_pool.size()) {
      uint8_t* b = g_pool[best];
      g_pool.erase(g_pool.begin() + best);
      return b + kOutHdr;
    }
  }
  const size_t cap = std::max<size_t>(bytes + bytes / 8, 1 << 16);
  void* p = nullptr;
  if (hipHostMalloc(&p, cap + kOutHdr, hipHostMallocDefault) != hipSuccess) return nullptr;
  OutHeader* hd = static_cast<OutHeader*>(p);
  hd->magic = kOutMagic;
  hd->cap = cap;
  hd->heap = 0;
  return static_cast<uint8_t*>(p) + kOutHdr;
}

// host-only outputs (jxg_shard_assemble runs without a device)
static uint8_t* out_alloc_heap(size_t bytes) {
  void* p = std::malloc(bytes + kOutHdr);
  if (!p) return nullptr;
  OutHeader* hd = static_cast<OutHeader*>(p);
  hd->magic = kOutMagic;
  hd->cap = bytes;
  hd->heap = 1;
  return static_cast<uint8_t*>(p) + kOutHdr;
}

// A codestream assembled at an offset inside its block (stage_concat_split:
// the AC block is copied first, the prefix lands right before it) carries a
// back reference to the block's data start in the kOutHdr bytes before it.
constexpr uint64_t kOutBackMagic = 0x6a7867426b526566ull;  // "jxgBkRef"
struct OutBackRef {
  uint64_t magic;
  uint8_t* data0;
};
static void out_set_backref(uint8_t* data, uint8_t* data0) {
  if (data == data0) return;
  OutBackRef* r = reinterpret_cast<OutBackRef*>(data - kOutHdr);
  r->magic = kOutBackMagic;
  r->data0 = data0;
}

static void out_release(uint8_t* data) {
  if (!data) return;
  if (reinterpret_cast<OutBackRef*>(data - kOutHdr)->magic == kOutBackMagic) {
    OutBackRef* r = reinterpret_cast<OutBackRef*>(data - kOutHdr);
    r->magic = 0;
    data = r->data0;
  }
  uint8_t* b = data - kOutHdr;
  if (reinterpret_cast<OutHeader*>(b)->magic != kOutMagic) return;  // not ours
  if (reinterpret_cast<OutHeader*>(b)->heap) {
    reinterpret_cast<OutHeader*>(b)->magic = 0;
    std::free(b);
    return;
  }
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (g_pool.size() < 8) {
    g_pool.push_back(b);
    return;
  }
  reinterpret_cast<OutHeader*>(b)->magic = 0;
  (void)hipHostFree(b);
}

using Clock = std::chrono::steady_clock;
static float ms_since(Clock::time_point t0) {
  return std::chrono::duration<float, std::milli>(Clock::now() - t0).count();
}

// frame-level scalars: same formulas as oracle jxo_frame_init (host, double)
struct Frame {
  uint32_t w, h, bxs, bys, xp, yp, tiles_x, tiles_y;
  uint32_t gxs, gys, ngroups, lfxs, lfys, nlf;
  float qf_base, inv_g;
  uint32_t G, qdc;
  float dc_mul[3], dc_step[3];
};

static Frame make_frame(uint32_t w, uint32_t h, float distance) {
  Frame f{};
  f.w = w;
  f.h = h;
  f.bxs = (w + 7) / 8;
  f.bys = (h + 7) / 8;
  f.xp = f.bxs * 8;
  f.yp = f.bys * 8;
  f.tiles_x = (f.bxs + 7) / 8;
  f.tiles_y = (f.bys + 7) / 8;
  f.gxs = (w + 255) / 256;
  f.gys = (h + 255) / 256;
  f.ngroups = f.gxs * f.gys;
  f.lfxs = (w + 2047) / 2048;
  f.lfys = (h + 2047) / 2048;
  f.nlf = f.lfxs * f.lfys;
  const double d = distance;
  const double qfb = 0.79 / d;
  f.qf_base = (float)qfb;
  long G = (long)std::floor(qfb * 1024.0 + 0.5);
  G = std::min<long>(std::max<long>(G, 1), 73727);
  f.G = (uint32_t)G;
  f.inv_g = (float)(65536.0 / (double)G);
  double t = 0.3 * std::pow(d / 0.3, 0.66);
  if (t > d) t = d;
  if (t < 0.5 * d) t = 0.5 * d;
  double qdc_f = 1.12 / t;
  if (qdc_f > 50.0) qdc_f = 50.0;
  long qdc = (long)std::floor(qdc_f * 65536.0 / (double)G + 0.5);
  qdc = std::min<long>(std::max<long>(qdc, 1), 65536);
  f.qdc = (uint32_t)qdc;
  const double m_lf[3] = {1.0 / 4096.0, 1.0 / 512.0, 1.0 / 256.0};
  for (int c = 0; c < 3; c++) {
    f.dc_mul[c] = (float)((double)G * (double)qdc / 65536.0 / m_lf[c]);
    f.dc_step[c] = (float)(65536.0 / (double)G / (double)qdc * m_lf[c]);
  }
  return f;
}

struct Ctx;
// batch lanes (jxg_encode_batch_rgb8[_device]): extra contexts of the same
// parameters, each with its own stream and pinned staging, owned by the
// context that ran the batch
struct CtxDeleter {
  void operator()(Ctx* c) const;
};
struct Ctx {
  jxg_params params{};
  std::vector<std::unique_ptr<Ctx, CtxDeleter>> lanes;
  PinBuf<uint8_t> h_stage;  // pinned staging of one host frame (pipeline lanes)
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // AC-block concat + D2H (stage_concat_split)
  // ev[6]: AC statistics downloaded (stage_download_ac); ev[7]: AC emission
  // done and its bit counts on the host; ev[8]: AC block in host memory;
  // ev[9]: masking quant field done (front kernel start)
  hipEvent_t ev[10] = {};
  bool constants_ready = false;
  // device
  DevBuf<uint8_t> rgb, acs, qf, aqf;  // aqf: masking quant field (JXG_FLAG_AQ_MASKING)
  DevBuf<float> lut;                   // sRGB8 -> linear (the AQ kernel)
  DevBuf<int8_t> cmap;  // [2][tiles] chroma from luma (front kernel)
  DevBuf<uint16_t> nz, mnat;
  DevBuf<float> ent, mwk, msdk, miwy, xyb_tiles, mcost;
  // merge levels 128 / 256 px (effort >= 8): tables (uploaded once), scratch
  // planes of the persistent workgroups, candidate estimates, chosen list
  DevBuf<float> big_tab, big_scratch, big_cost;
  DevBuf<uint16_t> big_nat;
  DevBuf<uint32_t> big_work;
  bool big_ready = false;
  DevBuf<uint32_t> vb, mwork, xlist;
  DevBuf<uint8_t> lf_mine;  // shard: [nlf] owned LF groups (vb_list)
  DevBuf<int32_t> dc;
  DevBuf<int16_t> ac;
  DevBuf<float> homog, xyb, r3;
  DevBuf<uint8_t> type;
  DevBuf<uint32_t> stream_chunks, scratch, scratch_lf, chunks, out, out_ac;
  DevBuf<uint64_t> lfstatus;  // [nchunks] lf_code look-back words
  // Per-frame statistics, zeroed by the front kernel and downloaded by two copies
  // (AC part, LF part): [hist_ac | bound | ntok | bandtok | bigcount][lfhist | sbound | vcount]
  DevBuf<uint8_t> stat;
  PinBuf<uint8_t> h_stat;
  View<uint32_t> hist_ac, bound, ntok, bandtok, bigcount, lfhist, sbound, vcount;
  View<uint32_t> h_hist_ac, h_bound, h_ntok, h_bigcount, h_lfhist, h_sbound, h_vcount;
  size_t stat_lf = 0, stat_bytes = 0;  // byte offset of the LF part, total
  // Per-frame code tables, uploaded by one copy (ANS) or two (prefix codes:
  // the AC part ahead of the AC emission): [codes_ac | gbase | ans_order |
  // ans_tab][lfcodes | stream_base]
  DevBuf<uint8_t> up;
  PinBuf<uint8_t> h_up;
  View<uint32_t> codes_ac, ans_order, lfcodes, h_codes_ac, h_ans_order, h_lfcodes;
  View<uint64_t> gbase, stream_base, h_gbase, h_sbase;
  View<uint8_t> ans_tab, h_ans_tab;
  size_t up_gbase = 0, up_ac = 0, up_lf = 0, up_bytes = 0;
  // emitted bit counts, one download: [gbits | stream_bits]
  DevBuf<uint32_t> bits;
  PinBuf<uint32_t> h_bits;
  View<uint32_t> gbits, stream_bits, h_gbits, h_sbits;
  uint32_t* lf_scratch = nullptr;  // LF-stream bit arena (scratch_lf, or in scratch)
  DevBuf<uint32_t> tile_list, glist;  // shard: tile ids, pass groups (non-contiguous plans)
  DevBuf<uint32_t> tokens, tval, ans_state, csum;  // ANS coder
  DevBuf<uint8_t> tlen;
  DevBuf<LfRow> rows;
  DevBuf<LfChunk> lfchunks;
  DevBuf<uint8_t> q_orig, q_comp;  // decode-side quality (jxg_compare_rgb8)
  DevBuf<uint64_t> q_sse;
  DevBuf<double> q_part, q_ssim;
  bool gauss_ready = false;
  DevBuf<ConcatPiece> pieces, pieces_ac;
  DevBuf<uint8_t> cat;  // stage_concat: [pieces | chunk words], one upload
  PinBuf<uint8_t> h_cat;
  PinBuf<ConcatPiece> h_pieces_ac;
  // host

  // LF row segments cached per frame size and shard
  uint32_t rows_w = 0, rows_h = 0, rows_rank = 0, rows_world = 1;
  std::vector<LfRow> rows_h_cache;
  std::vector<LfChunk> chunks_h_cache;
  std::vector<uint32_t> schunks_cache;
  // serialised AC context map of the previous frame (reused when equal)
  std::vector<uint8_t> cm_last;
  int cm_nhist = -1;
  BitWriter cm_bits;
  std::vector<uint8_t> m_acs, m_qf;
  std::vector<int32_t> m_dc, m_ac;
  std::vector<uint32_t> m_ntok;
  std::vector<float> m_homog;
  jxg_stats stats{};
  // ordering of device inputs (jxg_set_input_stream): the caller's stream
  // whose work so far every device-input entry point orders itself after
  hipStream_t in_stream = nullptr;
  hipEvent_t ev_in = nullptr;
  hipEvent_t ev_write = nullptr;  // jxg_shard_write_next: this slot's section copies
  uint32_t lane_cap = 0;          // jxg_set_pipeline_lanes (0: the queues' limit)
  bool owned_lane = false;  // a pipeline / batch lane of another context
  // a pipeline lane's extra slots: contexts with their own buffers that share
  // this context's stream (super-frames: k frames per batched launch)
  std::vector<std::unique_ptr<Ctx, CtxDeleter>> slots;
  bool shared_stream = false;  // `stream` belongs to the lane that owns this slot
  std::unique_ptr<struct Job> job;  // sharded encode in flight (begin -> end)
  std::unique_ptr<struct Pipe> pipe;  // streaming encode (jxg_submit_* / jxg_receive)
  std::vector<uint32_t> payload_head;  // last jxg_shard_end: payload head words
  size_t payload_body = 0;             //   and body bytes (in `out`)
};

void CtxDeleter::operator()(Ctx* c) const { jxg_destroy(reinterpret_cast<jxg_ctx*>(c)); }

static std::mutex g_const_mu;  // device __constant__ tables are shared by all contexts
// Live contexts of the process.  A HIP process has 4 hardware queues
// (GPU_MAX_HW_QUEUES); with several contexts their second streams would
// share queues with other contexts' main streams, so the split assembly
// (stage_concat_split, second stream) is used by a lone context only.
static std::atomic<int> g_live_ctx{0};  // caller-created contexts (owned lanes excluded)
static jxg_status init_constants(Ctx* c) {
  if (c->constants_ready) return JXG_OK;
  std::lock_guard<std::mutex> lock(g_const_mu);
  float lut[256];
  srgb_lut(lut);
  static float wts[5][3][64];
  quant_weights(wts);
  JXG_HIP(set_front_constants(lut, wts, c->stream));
  JXG_HIP(c->lut.ensure(256));
  JXG_HIP(hipMemcpyAsync(c->lut.p, lut, sizeof(lut), hipMemcpyHostToDevice, c->stream));
  uint8_t tab[kAcCtx];
  for (int i = 0; i < kAcCtx; i++) tab[i] = (uint8_t)ac_cluster(i);
  JXG_HIP(set_cluster_table(tab, c->stream));
  static const MergeTables mt = build_merge_tables();
  JXG_HIP(set_merge_constants(&mt.llf_p[0][0], &mt.llf_ib[0][0][0], c->stream));
  JXG_HIP(c->mwk.ensure(mt.wk.size()));
  JXG_HIP(c->msdk.ensure(mt.sdk.size()));
  JXG_HIP(c->miwy.ensure(mt.iwy.size()));
  JXG_HIP(c->mnat.ensure(mt.nat.size()));
  JXG_HIP(hipMemcpyAsync(c->mwk.p, mt.wk.data(), mt.wk.size() * 4, hipMemcpyHostToDevice, c->stream));
  JXG_HIP(hipMemcpyAsync(c->msdk.p, mt.sdk.data(), mt.sdk.size() * 4, hipMemcpyHostToDevice, c->stream));
  JXG_HIP(hipMemcpyAsync(c->miwy.p, mt.iwy.data(), mt.iwy.size() * 4, hipMemcpyHostToDevice, c->stream));
  JXG_HIP(hipMemcpyAsync(c->mnat.p, mt.nat.data(), mt.nat.size() * 2, hipMemcpyHostToDevice, c->stream));
  JXG_HIP(hipStreamSynchronize(c->stream));
  JXG_HIP(hipGetLastError());
  c->constants_ready = true;
  return JXG_OK;
}

// ---------------------------------------------------------------------------
// Work plan: which tiles, pass groups and LF groups this context encodes.
// world == 1: everything.  Sharded, make_partition:
//   1. balanced contiguous raster ranges of pass groups (rank r: [n*r/world,
//      n*(r+1)/world)), each LF group owned by the rank holding most of its
//      pass groups -- kept when that needs no record exchange (16384^2 over 8
//      ranks: LF-group rows fall on range boundaries);
//   2. otherwise whole LF groups per rank, when they balance: LF groups
//      assigned largest first (pixel area) to the least-loaded rank, kept if
//      the largest rank load is within 5 % of the mean (8K over 2 / 4 / 8
//      ranks: 1.1 %) -- every rank then owns the LF groups of all its pass
//      groups, so no per-block records move between ranks and a rank's frames
//      need no collective until assembly (the streaming shard pipeline);
//   3. else the ranges of 1 with the record exchange.
// ---------------------------------------------------------------------------
static uint32_t shard_g0(uint32_t ngroups, uint32_t r, uint32_t world) {
  return (uint32_t)(((uint64_t)ngroups * r) / world);
}
static uint32_t shard_of(uint32_t ngroups, uint32_t g, uint32_t world) {
  uint32_t r = (uint32_t)(((uint64_t)g * world) / ngroups);  // then correct the rounding
  while (r + 1 < world && shard_g0(ngroups, r + 1, world) <= g) r++;
  while (r > 0 && shard_g0(ngroups, r, world) > g) r--;
  return r;
}
static uint32_t lf_of_group(const Frame& f, uint32_t g) {
  return ((g / f.gxs) / 8) * f.lfxs + (g % f.gxs) / 8;
}
// LF-group owners under the contiguous ranges: the rank holding the most of
// the LF group's pass groups, less 16 per LF group already assigned to it (so
// near ties -- an LF group split over ranks' row ranges -- spread over ranks
// instead of piling onto one); ties go to the lower rank.
static std::vector<uint32_t> lf_owners_ranges(const Frame& f, uint32_t world) {
  std::vector<uint32_t> own(f.nlf, 0), nassigned(world, 0), cnt(world);
  if (world == 1) return own;
  for (uint32_t lg = 0; lg < f.nlf; lg++) {
    std::fill(cnt.begin(), cnt.end(), 0u);
    const uint32_t lx = lg % f.lfxs, ly = lg / f.lfxs;
    for (uint32_t gy = ly * 8; gy < std::min(ly * 8 + 8, f.gys); gy++)
      for (uint32_t gx = lx * 8; gx < std::min(lx * 8 + 8, f.gxs); gx++)
        cnt[shard_of(f.ngroups, gy * f.gxs + gx, world)]++;
    int best = -1;
    long bs = 0;
    for (uint32_t r = 0; r < world; r++) {
      if (!cnt[r]) continue;
      const long sc = (long)cnt[r] - 16 * (long)nassigned[r];
      if (best < 0 || sc > bs) {
        best = (int)r;
        bs = sc;
      }
    }
    own[lg] = (uint32_t)best;
    nassigned[best]++;
  }
  return own;
}
struct Partition {
  std::vector<uint32_t> group;  // [ngroups] owner rank of each pass group
  std::vector<uint32_t> lf;     // [nlf] owner rank of each LF group
  int kind = 0;                 // 0 ranges (no exchange), 1 whole LF groups, 2 ranges + exchange
};
static Partition make_partition(const Frame& f, uint32_t world) {
  Partition P;
  P.group.assign(f.ngroups, 0);
  P.lf.assign(f.nlf, 0);
  if (world <= 1) return P;
  for (uint32_t g = 0; g < f.ngroups; g++) P.group[g] = shard_of(f.ngroups, g, world);
  P.lf = lf_owners_ranges(f, world);
  bool exchange = false;
  for (uint32_t g = 0; g < f.ngroups && !exchange; g++)
    exchange = P.lf[lf_of_group(f, g)] != P.group[g];
  if (!exchange) return P;
  if (f.nlf >= world) {
    // whole LF groups, largest first (pixel area; ties: lower index) to the
    // least-loaded rank (ties: lower rank)
    std::vector<uint64_t> area(f.nlf);
    uint64_t total = 0;
    for (uint32_t lg = 0; lg < f.nlf; lg++) {
      const uint64_t x0 = (uint64_t)(lg % f.lfxs) * 2048, y0 = (uint64_t)(lg / f.lfxs) * 2048;
      area[lg] = std::min<uint64_t>(2048, f.w - x0) * std::min<uint64_t>(2048, f.h - y0);
      total += area[lg];
    }
    std::vector<uint32_t> order(f.nlf);
    for (uint32_t i = 0; i < f.nlf; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return area[a] > area[b]; });
    std::vector<uint64_t> load(world, 0);
    std::vector<uint32_t> lfo(f.nlf, 0);
    for (uint32_t lg : order) {
      uint32_t r = 0;
      for (uint32_t q = 1; q < world; q++)
        if (load[q] < load[r]) r = q;
      lfo[lg] = r;
      load[r] += area[lg];
    }
    const uint64_t most = *std::max_element(load.begin(), load.end());
    const uint64_t least = *std::min_element(load.begin(), load.end());
    if (least > 0 && most * 100 * world <= total * 105) {
      P.lf = lfo;
      for (uint32_t g = 0; g < f.ngroups; g++) P.group[g] = lfo[lf_of_group(f, g)];
      P.kind = 1;
      return P;
    }
  }
  P.kind = 2;
  return P;
}
// Record exchange of rank `rank`: send = its groups whose LF group another
// rank owns, ordered by (destination rank, group); recv = other ranks' groups
// inside its own LF groups, ordered by (source rank, group).  Counts per peer.
struct Exchange {
  std::vector<uint32_t> send, recv, nsend, nrecv;
};
static Exchange make_exchange(const Frame& f, const Partition& part, uint32_t rank,
                              uint32_t world) {
  Exchange X;
  X.nsend.assign(world, 0);
  X.nrecv.assign(world, 0);
  for (uint32_t p = 0; p < world; p++) {
    if (p == rank) continue;
    for (uint32_t g = 0; g < f.ngroups; g++) {
      const uint32_t lo = part.lf[lf_of_group(f, g)];
      if (part.group[g] == rank && lo == p) {
        X.send.push_back(g);
        X.nsend[p]++;
      }
      if (part.group[g] == p && lo == rank) {
        X.recv.push_back(g);
        X.nrecv[p]++;
      }
    }
  }
  return X;
}

struct Plan {
  uint32_t rank = 0, world = 1;
  std::vector<uint32_t> groups; // pass groups, ascending (launch slot i = groups[i])
  bool contiguous = true;       // groups == [groups[0], groups[0] + size)
  std::vector<uint32_t> tiles;  // shard: owned tile ids (ty * tiles_x + tx)
  std::vector<uint8_t> lf_mine; // shard: [nlf] 1 = owned LF group
  Exchange x;                   // shard: record exchange
  bool owns_lf(uint32_t lg) const { return world == 1 || lf_mine[lg]; }
  uint32_t g0() const { return groups.empty() ? 0 : groups[0]; }
  uint32_t ng() const { return (uint32_t)groups.size(); }
};
static Plan make_plan(const Frame& f, uint32_t rank, uint32_t world) {
  Plan P;
  P.rank = rank;
  P.world = world;
  if (world <= 1) {
    P.groups.resize(f.ngroups);
    for (uint32_t g = 0; g < f.ngroups; g++) P.groups[g] = g;
    return P;
  }
  const Partition part = make_partition(f, world);
  for (uint32_t g = 0; g < f.ngroups; g++)
    if (part.group[g] == rank) P.groups.push_back(g);
  P.contiguous = P.groups.empty() || P.groups.back() - P.groups.front() + 1 == P.groups.size();
  for (uint32_t g : P.groups) {
    const uint32_t gx = g % f.gxs, gy = g / f.gxs;
    for (uint32_t ty = gy * 4; ty < std::min(gy * 4 + 4, f.tiles_y); ty++)
      for (uint32_t tx = gx * 4; tx < std::min(gx * 4 + 4, f.tiles_x); tx++)
        P.tiles.push_back(ty * f.tiles_x + tx);
  }
  P.lf_mine.resize(f.nlf);
  for (uint32_t lg = 0; lg < f.nlf; lg++) P.lf_mine[lg] = part.lf[lg] == rank;
  P.x = make_exchange(f, part, rank, world);
  return P;
}
// exchange record of one pass group (jxg_shard.hip): acs, qf, 3 x int32 DC
constexpr size_t kGroupRecordBytes = 1024 * 2 + 1024 * 4 * 3 + 32;  // jxg_shard.hip

// LF-group row segments: (lf group, stream, channel, y, x0) in stream order,
// grouped into chunks of one stream (<= kLfChunkSamples samples,
// <= kLfChunkRows segments); only the plan's LF groups get rows (the stream
// table keeps an empty range for the others)
static void build_rows(const Frame& f, const Plan& P, std::vector<LfRow>& rows,
                       std::vector<LfChunk>& chunks, std::vector<uint32_t>& schunks) {
  rows.clear();
  chunks.clear();
  schunks.clear();
  auto add = [&](uint32_t lg, uint16_t stream, uint16_t ch, uint32_t y, uint32_t width) {
    for (uint32_t x0 = 0; x0 < width; x0 += kLfSeg) {
      const uint32_t wseg = std::min(kLfSeg, width - x0);
      const uint32_t sid = lg * 2 + stream;
      if (chunks.empty() || chunks.back().sid != sid || chunks.back().nrows == kLfChunkRows ||
          chunks.back().nsamp + wseg > kLfChunkSamples)
        chunks.push_back({(uint32_t)rows.size(), 0, sid, 0});
      chunks.back().nrows++;
      chunks.back().nsamp += wseg;
      rows.push_back({lg, stream, ch, y, x0, wseg, sid});
    }
  };
  for (uint32_t lg = 0; lg < f.nlf; lg++) {
    const uint32_t bx0 = (lg % f.lfxs) * 256, by0 = (lg / f.lfxs) * 256;
    const uint32_t bw = std::min(256u, f.bxs - bx0), bh = std::min(256u, f.bys - by0);
    const bool own = P.owns_lf(lg);
    schunks.push_back((uint32_t)chunks.size());
    if (own)
      for (uint16_t ch = 0; ch < 3; ch++)
        for (uint32_t y = 0; y < bh; y++) add(lg, 0, ch, y, bw);
    schunks.push_back((uint32_t)chunks.size());
    if (own) {
      const uint32_t cw = (bw + 7) / 8, chh = (bh + 7) / 8;
      for (uint16_t ch = 0; ch < 2; ch++)
        for (uint32_t y = 0; y < chh; y++) add(lg, 1, ch, y, cw);
      for (uint32_t y = 0; y < 2; y++) add(lg, 1, 2, y, bw * bh);
      for (uint32_t y = 0; y < bh; y++) add(lg, 1, 3, y, bw);
    }
  }
  schunks.push_back((uint32_t)chunks.size());
}

// Host waits on the library's events (helper threads waiting for statistics,
// emission, codestream copies): JXG_EVENT_BLOCKING=1 makes them blocking-sync
// events (the waiting thread sleeps until the GPU signals) instead of the
// runtime's default active wait -- an A/B switch for the host-CPU budget of
// several ranks per node
static hipError_t make_event(hipEvent_t* e, unsigned flags) {
  static const bool blocking = [] {
    const char* v = std::getenv("JXG_EVENT_BLOCKING");
    return v && v[0] == '1';
  }();
  return hipEventCreateWithFlags(e, flags | (blocking ? hipEventBlockingSync : 0u));
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

// state carried between the stages of one encode
struct Job {
  Frame f;
  Plan plan;
  uint32_t w = 0, h = 0;
  size_t stride = 0;
  const uint8_t* d_rgb = nullptr;
  int max_s = 0;
  bool homog = false;
  bool ans = false;  // ANS instead of prefix codes for the AC stream
  uint32_t lf = 0;   // frame header loop-filter code (lf_code: Gaborish / EPF)
  uint32_t nhist_ans = 0, max_tokens = 0;
  uint32_t nrows = 0, nchunks = 0, nstreams = 0;
  AcArgs aa{};
  LfArgs la{};
  // argument blocks of the front / merge / LF-list stages and the rANS coder
  // (build_front, build_emit): the batched launches gather them per frame
  FrontArgs fa{};
  AqArgs qa{};
  MergeArgs ma{};
  BigArgs ba{};
  bool big = false;  // merge levels 128 / 256 px (effort >= 8)
  VbArgs va{};
  AnsArgs na{};
  bool aq = false;  // masking quant field (aq_kernel before the front kernel)
  // host stage results
  std::vector<BitWriter> preA, preB;
  BitWriter lfglobal, hfglobal;
  // sharded ANS encode with one HF preset per rank: no histogram
  // all-reduce; the rank's clustered histograms travel in its payload head and
  // HfGlobal is written at assembly (build_hf_presets)
  bool presets = false;
  std::vector<uint8_t> pre_ctxmap;   // [kAcCtx] context -> the rank's dense histogram
  std::vector<uint32_t> pre_counts;  // [nhist][kAlpha] clustered counts
  std::vector<uint64_t> gbase, sbase;
  float ms_codes = 0.0f;
  float ms_layout = 0.0f;  // stage_concat_split host layout
  // enc_finish_start -> enc_finish_end: the codestream (pinned pool block,
  // D2H in flight), its size, the host layout time
  uint8_t* host_out = nullptr;
  size_t out_bytes = 0;
  float ms_finish_layout = 0.0f;
};

// the emission of J on c is done and its bit counts are on the host
static jxg_status wait_emission(Ctx* c, Job& J) {
  (void)J;
  JXG_HIP(hipStreamSynchronize(c->stream));
  return JXG_OK;
}

// ---- stage A: buffers for the frame / plan ----
static jxg_status stage_alloc(Ctx* c, Job& J) {
  hipStream_t s = c->stream;
  const jxg_params& P = c->params;
  const Frame& f = J.f;
  const size_t nb = (size_t)f.bxs * f.bys;
  J.homog = (P.proposals & 3u) != 0;
  J.ans = (P.flags & JXG_FLAG_ANS) != 0;
  J.lf = lf_code(P.flags, P.distance);
  jxg_status st = init_constants(c);
  if (st) return st;
  JXG_HIP(c->acs.ensure(nb));
  JXG_HIP(c->qf.ensure(nb));
  JXG_HIP(c->nz.ensure(nb * 3));
  JXG_HIP(c->dc.ensure(nb * 3));
  JXG_HIP(c->ac.ensure(nb * 192));
  if (J.homog) JXG_HIP(c->homog.ensure(nb * 3));
  J.max_s = P.effort >= 6 ? 8 : (P.effort >= 5 ? 4 : 0);  // merge levels
  const uint32_t ntiles = f.tiles_x * f.tiles_y;
  JXG_HIP(c->cmap.ensure((size_t)ntiles * 2));
  if (J.max_s) {
    JXG_HIP(c->ent.ensure(nb));
    JXG_HIP(c->xyb_tiles.ensure((size_t)ntiles * 3 * 4096));
    JXG_HIP(c->mcost.ensure((size_t)ntiles * kNumShapes * 32));
    JXG_HIP(c->mwork.ensure(1 + (size_t)ntiles * kNumShapes));
  }
  // the plan's tile, LF-group and pass-group lists: uploaded when the plan
  // changes (the same key as the LF row cache below)
  const bool new_plan = c->rows_w != J.w || c->rows_h != J.h || c->rows_rank != J.plan.rank ||
                        c->rows_world != J.plan.world;
  if (!J.plan.tiles.empty()) {
    JXG_HIP(c->tile_list.ensure(J.plan.tiles.size()));
    if (new_plan)
      JXG_HIP(hipMemcpyAsync(c->tile_list.p, J.plan.tiles.data(), J.plan.tiles.size() * 4,
                             hipMemcpyHostToDevice, s));
  }
  if (!J.plan.lf_mine.empty()) {
    JXG_HIP(c->lf_mine.ensure(J.plan.lf_mine.size()));
    if (new_plan)
      JXG_HIP(hipMemcpyAsync(c->lf_mine.p, J.plan.lf_mine.data(), J.plan.lf_mine.size(),
                             hipMemcpyHostToDevice, s));
  }
  JXG_HIP(c->vb.ensure((size_t)f.nlf * 65536));
  J.nstreams = f.nlf * 2;
  {
    // the statistics, code-table and bit-count arenas of this frame
    const uint32_t ns = J.nstreams;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t o = 0;
    const size_t o_hist = o;
    o = al(o + (size_t)kMaxClusters * kAlpha * 4);
    const size_t o_bound = o;
    o = al(o + (size_t)f.ngroups * 4);
    const size_t o_ntok = o;
    o = al(o + (size_t)f.ngroups * 12);
    const size_t o_bandtok = o;
    o = al(o + (size_t)f.ngroups * 16);
    const size_t o_bigcount = o;  // varblocks per big kind (big_list_kernel)
    o = al(o + 16);
    const size_t o_lfhist = o;
    o = al(o + (size_t)ns * 4 * kAlpha * 4);
    const size_t o_sbound = o;
    o = al(o + (size_t)ns * 4);
    const size_t o_vcount = o;
    o = al(o + (size_t)f.nlf * 4);
    JXG_HIP(c->stat.ensure(o));
    JXG_HIP(c->h_stat.ensure(o));
    c->stat_lf = o_lfhist;
    c->stat_bytes = o;
    c->hist_ac.set(c->stat.p, o_hist, (size_t)kMaxClusters * kAlpha);
    c->bound.set(c->stat.p, o_bound, f.ngroups);
    c->ntok.set(c->stat.p, o_ntok, (size_t)f.ngroups * 3);
    c->bandtok.set(c->stat.p, o_bandtok, (size_t)f.ngroups * 4);
    c->bigcount.set(c->stat.p, o_bigcount, 4);
    c->h_bigcount.set(c->h_stat.p, o_bigcount, 4);
    c->lfhist.set(c->stat.p, o_lfhist, (size_t)ns * 4 * kAlpha);
    c->sbound.set(c->stat.p, o_sbound, ns);
    c->vcount.set(c->stat.p, o_vcount, f.nlf);
    c->h_hist_ac.set(c->h_stat.p, o_hist, (size_t)kMaxClusters * kAlpha);
    c->h_bound.set(c->h_stat.p, o_bound, f.ngroups);
    c->h_ntok.set(c->h_stat.p, o_ntok, (size_t)f.ngroups * 3);
    c->h_lfhist.set(c->h_stat.p, o_lfhist, (size_t)ns * 4 * kAlpha);
    c->h_sbound.set(c->h_stat.p, o_sbound, ns);
    c->h_vcount.set(c->h_stat.p, o_vcount, f.nlf);
    const uint32_t ng = std::max(1u, J.plan.ng());
    o = 0;
    const size_t o_codes = o;
    o = al(o + (size_t)kMaxClusters * kAlpha * 4);
    const size_t o_gbase = o;
    o = al(o + (size_t)f.ngroups * 8);
    const size_t o_order = o;
    o = al(o + (size_t)ng * 4);
    const size_t o_tab = o;
    o = al(o + kAnsTabBytes);
    const size_t o_lfcodes = o;
    o = al(o + (size_t)ns * 4 * kAlpha * 4);
    const size_t o_sbase = o;
    o = al(o + (size_t)ns * 8);
    JXG_HIP(c->up.ensure(o));
    JXG_HIP(c->h_up.ensure(o));
    c->up_gbase = o_gbase;
    c->up_ac = o_order;
    c->up_lf = o_lfcodes;
    c->up_bytes = o;
    c->codes_ac.set(c->up.p, o_codes, (size_t)kMaxClusters * kAlpha);
    c->gbase.set(c->up.p, o_gbase, f.ngroups);
    c->ans_order.set(c->up.p, o_order, ng);
    c->ans_tab.set(c->up.p, o_tab, kAnsTabBytes);
    c->lfcodes.set(c->up.p, o_lfcodes, (size_t)ns * 4 * kAlpha);
    c->stream_base.set(c->up.p, o_sbase, ns);
    c->h_codes_ac.set(c->h_up.p, o_codes, (size_t)kMaxClusters * kAlpha);
    c->h_gbase.set(c->h_up.p, o_gbase, f.ngroups);
    c->h_ans_order.set(c->h_up.p, o_order, ng);
    c->h_ans_tab.set(c->h_up.p, o_tab, kAnsTabBytes);
    c->h_lfcodes.set(c->h_up.p, o_lfcodes, (size_t)ns * 4 * kAlpha);
    c->h_sbase.set(c->h_up.p, o_sbase, ns);
    const size_t nbits = (size_t)f.ngroups + ns;
    JXG_HIP(c->bits.ensure(nbits));
    JXG_HIP(c->h_bits.ensure(nbits));
    c->gbits.set(c->bits.p, 0, f.ngroups);
    c->stream_bits.set(c->bits.p, (size_t)f.ngroups * 4, ns);
    c->h_gbits.set(c->h_bits.p, 0, f.ngroups);
    c->h_sbits.set(c->h_bits.p, (size_t)f.ngroups * 4, ns);
  }
  const bool new_rows = c->rows_w != J.w || c->rows_h != J.h || c->rows_rank != J.plan.rank ||
                        c->rows_world != J.plan.world;
  if (new_rows) {
    build_rows(f, J.plan, c->rows_h_cache, c->chunks_h_cache, c->schunks_cache);
    c->rows_w = J.w;
    c->rows_h = J.h;
    c->rows_rank = J.plan.rank;
    c->rows_world = J.plan.world;
  }
  J.nrows = (uint32_t)c->rows_h_cache.size();
  J.nchunks = (uint32_t)c->chunks_h_cache.size();
  const uint32_t nstreams = J.nstreams;
  JXG_HIP(c->rows.ensure(J.nrows));
  JXG_HIP(c->lfchunks.ensure(J.nchunks));
  JXG_HIP(c->lfstatus.ensure(J.nchunks));
  JXG_HIP(c->stream_chunks.ensure(nstreams + 1));
  if (new_rows) {
    if (J.nrows)
      JXG_HIP(hipMemcpyAsync(c->rows.p, c->rows_h_cache.data(), J.nrows * sizeof(LfRow),
                             hipMemcpyHostToDevice, s));
    if (J.nchunks)
      JXG_HIP(hipMemcpyAsync(c->lfchunks.p, c->chunks_h_cache.data(), J.nchunks * sizeof(LfChunk),
                             hipMemcpyHostToDevice, s));
    JXG_HIP(hipMemcpyAsync(c->stream_chunks.p, c->schunks_cache.data(),
                           c->schunks_cache.size() * 4, hipMemcpyHostToDevice, s));
  }
  // kernel argument blocks
  AcArgs& aa = J.aa;
  aa = AcArgs{};
  aa.acs = c->acs.p;
  aa.ac = c->ac.p;
  aa.nz = c->nz.p;
  aa.bxs = f.bxs;
  aa.bys = f.bys;
  aa.gxs = f.gxs;
  aa.g0 = J.plan.g0();
  if (!J.plan.contiguous) {
    JXG_HIP(c->glist.ensure(J.plan.ng()));
    if (new_plan)
      JXG_HIP(hipMemcpyAsync(c->glist.p, J.plan.groups.data(), J.plan.ng() * 4,
                             hipMemcpyHostToDevice, s));
    aa.glist = c->glist.p;
  }
  aa.hist = c->hist_ac.p;
  aa.bound = c->bound.p;
  aa.ntok = c->ntok.p;
  aa.bandtok = c->bandtok.p;
  aa.codes = c->codes_ac.p;
  aa.base = c->gbase.p;
  aa.bits = c->gbits.p;
  JXG_HIP(c->tokens.ensure((uint64_t)std::max(1u, J.plan.ng()) * kGroupTokStride));
  aa.tokens = c->tokens.p;
  LfArgs& la = J.la;
  la = LfArgs{};
  la.rows = c->rows.p;
  la.chunks = c->lfchunks.p;
  la.dc = c->dc.p;
  la.acs = c->acs.p;
  la.qf = c->qf.p;
  la.vb = c->vb.p;
  la.vcount = c->vcount.p;
  la.bxs = f.bxs;
  la.bys = f.bys;
  la.lfxs = f.lfxs;
  la.cmap = c->cmap.p;
  la.tiles_x = f.tiles_x;
  la.ntiles_all = f.tiles_x * f.tiles_y;
  la.hist = c->lfhist.p;
  la.sbound = c->sbound.p;
  la.codes = c->lfcodes.p;
  la.status = c->lfstatus.p;
  la.stream_chunks = c->stream_chunks.p;
  la.stream_base = c->stream_base.p;
  la.stream_bits = c->stream_bits.p;
  return JXG_OK;
}

// ---- stage B: argument blocks of the front end, merge stage and LF lists
// over the plan's tiles (launched by launch_stats, batched over frames) ----
static jxg_status build_front(Ctx* c, Job& J) {
  const jxg_params& P = c->params;
  const Frame& f = J.f;
  FrontArgs& fa = J.fa;
  fa = FrontArgs{};
  fa.rgb = J.d_rgb;
  fa.w = J.w;
  fa.h = J.h;
  fa.stride = J.stride;
  fa.bxs = f.bxs;
  fa.bys = f.bys;
  fa.xp = f.xp;
  fa.yp = f.yp;
  fa.tiles_x = f.tiles_x;
  fa.distance = P.distance;
  fa.effort = P.effort;
  fa.proposals = P.proposals;
  fa.h1_int = (P.flags & JXG_FLAG_H1_INT_ABS) ? 1 : 0;
  fa.gab = (P.flags & JXG_FLAG_GABORISH) ? 1 : 0;
  fa.qf_base = f.qf_base;
  fa.inv_g = f.inv_g;
  fa.G = f.G;
  for (int i = 0; i < 3; i++) {
    fa.dc_mul[i] = f.dc_mul[i];
    fa.dc_step[i] = f.dc_step[i];
  }
  fa.acs = c->acs.p;
  fa.qf = c->qf.p;
  fa.dc = c->dc.p;
  fa.ac = c->ac.p;
  fa.nz = c->nz.p;
  fa.homog = J.homog ? c->homog.p : nullptr;
  fa.ent = J.max_s ? c->ent.p : nullptr;
  fa.xyb_out = J.max_s ? c->xyb_tiles.p : nullptr;
  const bool listed = !J.plan.tiles.empty();
  fa.tile_list = listed ? c->tile_list.p : nullptr;
  fa.cmap = c->cmap.p;
  fa.ntiles_all = f.tiles_x * f.tiles_y;
  // the statistics arena (256-byte aligned sections) is zeroed by the front
  // kernel's workgroups: no memset launch
  fa.zero = reinterpret_cast<uint4*>(c->stat.p);
  fa.zero_quads = (uint32_t)(c->stat_bytes / 16);
  if (P.flags & JXG_FLAG_AQ_MASKING) {
    // the libjxl-shaped masking quant field of the plan's tiles, before the
    // front kernel (== oracle/aq.c jxo_aq_masking)
    JXG_HIP(c->aqf.ensure((size_t)f.bxs * f.bys));
    J.aq = true;
    AqArgs& q = J.qa;
    q = AqArgs{};
    q.rgb = J.d_rgb;
    q.w = J.w;
    q.h = J.h;
    q.stride = J.stride;
    q.xp = f.xp;
    q.yp = f.yp;
    q.bxs = f.bxs;
    q.bys = f.bys;
    q.tiles_x = f.tiles_x;
    q.lut = c->lut.p;
    aq_erosion_weights(P.distance, q.ew);
    float dampen = 1.0f;
    if (P.distance >= 2.0f) {
      dampen = 1.0f - ((P.distance - 2.0f) / (14.0f - 2.0f));
      if (dampen < 0.0f) dampen = 0.0f;
    }
    q.mul = f.qf_base * dampen;
    q.add = (1.0f - dampen) * (0.48f * f.qf_base);
    q.inv_g = f.inv_g;
    q.qf = c->aqf.p;
    q.tile_list = listed ? c->tile_list.p : nullptr;
    fa.qf_in = c->aqf.p;
  } else {
    J.aq = false;
  }
  if (J.max_s) {
    MergeArgs& ma = J.ma;
    ma = MergeArgs{};
    ma.xyb = c->xyb_tiles.p;
    ma.bxs = f.bxs;
    ma.bys = f.bys;
    ma.tiles_x = f.tiles_x;
    ma.ntiles = listed ? (uint32_t)J.plan.tiles.size() : (J.plan.world == 1 ? f.tiles_x * f.tiles_y : 0);
    ma.tile_list = listed ? c->tile_list.p : nullptr;
    ma.proposals = P.proposals;
    ma.max_s = J.max_s;
    ma.G = f.G;
    for (int i = 0; i < 3; i++) {
      ma.dc_mul[i] = f.dc_mul[i];
      ma.dc_step[i] = f.dc_step[i];
    }
    ma.ent = c->ent.p;
    ma.cmap = c->cmap.p;
    ma.ntiles_all = f.tiles_x * f.tiles_y;
    ma.homog = J.homog ? c->homog.p : nullptr;
    ma.acs = c->acs.p;
    ma.qf = c->qf.p;
    ma.dc = c->dc.p;
    ma.ac = c->ac.p;
    ma.nz = c->nz.p;
    ma.cost = c->mcost.p;
    ma.wk = c->mwk.p;
    ma.sdk = c->msdk.p;
    ma.iwy = c->miwy.p;
    ma.nat = c->mnat.p;
    ma.work = c->mwork.p;
    ma.nwrite = 256 * 3 * 4;  // CUs x resident workgroups (3) x 4 rounds
  }
  // effort >= 8: the 128 / 256 px levels over the plan's pass groups
  J.big = J.max_s && P.effort >= 8;
  if (J.big) {
    if (!c->big_ready) {
      static const BigTables bt = build_big_tables();
      JXG_HIP(c->big_tab.ensure(bt.tab.size()));
      JXG_HIP(c->big_nat.ensure(bt.nat.size()));
      JXG_HIP(hipMemcpyAsync(c->big_tab.p, bt.tab.data(), bt.tab.size() * 4, hipMemcpyHostToDevice, c->stream));
      JXG_HIP(hipMemcpyAsync(c->big_nat.p, bt.nat.data(), bt.nat.size() * 2, hipMemcpyHostToDevice, c->stream));
      c->big_ready = true;
    }
    const uint32_t ng = std::max(1u, J.plan.ng());
    // one scratch slot per persistent workgroup; a frame of ng groups has at
    // most 20 ng tasks per level launch (a 512 x 512 frame needs 20
    // slots, not the 512 of an 8K one -- 402 MB per context otherwise)
    const uint32_t slots = std::min<uint32_t>(ng * 20u, kBigSlots);
    JXG_HIP(c->big_scratch.ensure((size_t)slots * kBigPlanes));
    JXG_HIP(c->big_cost.ensure((size_t)ng * 30));  // [group][25 estimates + 5 current sums]
    JXG_HIP(c->big_work.ensure(1 + (size_t)ng * 16));
    BigArgs& ba = J.ba;
    ba = BigArgs{};
    ba.m = J.ma;
    ba.tab = c->big_tab.p;
    ba.nat = c->big_nat.p;
    ba.scratch = c->big_scratch.p;
    ba.slots = slots;
    ba.cost = c->big_cost.p;
    ba.work = c->big_work.p;
    ba.kinds = c->bigcount.p;
    ba.glist = J.plan.contiguous ? nullptr : c->glist.p;
    ba.g0 = J.plan.g0();
    ba.ng = J.plan.ng();
    ba.gxs = f.gxs;
  }
  J.va = VbArgs{c->acs.p, f.bxs, f.bys, f.lfxs, J.plan.world > 1 ? c->lf_mine.p : nullptr, c->vb.p,
                c->vcount.p};
  return JXG_OK;
}

// bit k: the frame (or with a caller's summed histogram, the whole sharded
// frame) holds a varblock of big kind k
static uint32_t big_mask(const uint32_t* count) {
  uint32_t m = 0;
  for (int k = 0; k < 4; k++) m |= (count[k] != 0 ? 1u : 0u) << k;
  return m;
}

// ---- stage E: statistics to the host (AC histogram from `hist`) ----
// AC statistics (histogram, bit bounds, token counts) are downloaded as soon as
// ac_hist is done, so the host builds the AC prefix codes while the LF
// statistics kernels still run; the LF statistics follow in stage_download_lf.
static jxg_status stage_download_ac(Ctx* c, Job& J, const uint32_t* hist) {
  (void)J;
  hipStream_t s = c->stream;
  if (hist == c->hist_ac.p) {  // [hist_ac | bound | ntok]: one copy
    JXG_HIP(hipMemcpyAsync(c->h_stat.p, c->stat.p, c->stat_lf, hipMemcpyDeviceToHost, s));
  } else {  // a caller's (all-reduced) histogram
    const size_t hb = (size_t)kMaxClusters * kAlpha * 4, ob = (uint8_t*)c->bound.p - c->stat.p;
    JXG_HIP(hipMemcpyAsync(c->h_hist_ac.p, hist, hb, hipMemcpyDeviceToHost, s));
    JXG_HIP(hipMemcpyAsync(c->h_stat.p + ob, c->stat.p + ob, c->stat_lf - ob, hipMemcpyDeviceToHost, s));
    // the big-kind counts summed with it (jxg_shard_sizes: after the histogram)
    JXG_HIP(hipMemcpyAsync(c->h_bigcount.p, hist + (size_t)kMaxClusters * kAlpha, 16,
                           hipMemcpyDeviceToHost, s));
  }
  JXG_HIP(hipEventRecord(c->ev[6], s));
  return JXG_OK;
}
static jxg_status stage_download_lf(Ctx* c, Job& J) {
  (void)J;
  hipStream_t s = c->stream;
  // [lfhist | sbound | vcount]: one copy
  JXG_HIP(hipMemcpyAsync(c->h_stat.p + c->stat_lf, c->stat.p + c->stat_lf, c->stat_bytes - c->stat_lf,
                         hipMemcpyDeviceToHost, s));
  JXG_HIP(hipEventRecord(c->ev[2], s));
  return JXG_OK;
}

// ---- stages B-E of k frames of one size and plan whose contexts share one
// stream (a pipeline lane's slots; k = 1 for one-at-a-time encodes): one
// launch of each kernel for all of them, each frame's downloads after it ----
template <class A, class F>
static std::vector<A> gather(Job* const* js, uint32_t k, F f) {
  std::vector<A> v(k);
  for (uint32_t i = 0; i < k; i++) v[i] = f(*js[i]);
  return v;
}
// a batched launch sizes its grid from frame 0 and indexes the argument
// blocks by blockIdx.z: 1..kMaxBatch frames of one geometry and plan, one stream
static bool batch_ok(Ctx* const* cs, Job* const* js, uint32_t k) {
  if (k < 1 || k > kMaxBatch) return false;
  const Job& A = *js[0];
  for (uint32_t i = 1; i < k; i++) {
    const Job& B = *js[i];
    if (cs[i]->stream != cs[0]->stream || B.w != A.w || B.h != A.h || B.plan.rank != A.plan.rank ||
        B.plan.world != A.plan.world || B.plan.tiles.size() != A.plan.tiles.size() ||
        B.plan.ng() != A.plan.ng() || B.nchunks != A.nchunks || B.max_s != A.max_s || B.aq != A.aq)
      return false;
  }
  return true;
}
// front end (+ masking quant field), merge stage, AC token statistics
static jxg_status launch_transform(Ctx* const* cs, Job* const* js, uint32_t k) {
  if (!batch_ok(cs, js, k)) return JXG_ERR_INTERNAL;
  hipStream_t s = cs[0]->stream;
  const Job& J = *js[0];
  const Frame& f = J.f;
  const bool listed = !J.plan.tiles.empty();
  const uint32_t ntiles = listed ? (uint32_t)J.plan.tiles.size() : f.tiles_x * f.tiles_y;
  for (uint32_t i = 0; i < k; i++) JXG_HIP(hipEventRecord(cs[i]->ev[0], s));
  if (J.aq) {
    const auto q = gather<AqArgs>(js, k, [](Job& j) { return j.qa; });
    launch_aq(q.data(), k, ntiles, s);
  }
  for (uint32_t i = 0; i < k; i++) JXG_HIP(hipEventRecord(cs[i]->ev[9], s));
  const auto fa = gather<FrontArgs>(js, k, [](Job& j) { return j.fa; });
  if (listed)
    launch_front_list(fa.data(), k, ntiles, s);
  else if (J.plan.world == 1)
    launch_front(fa.data(), k, f.tiles_x, f.tiles_y, s);
  JXG_HIP(hipGetLastError());
  for (uint32_t i = 0; i < k; i++) JXG_HIP(hipEventRecord(cs[i]->ev[5], s));  // front kernel alone
  if (J.max_s) {
    const auto ma = gather<MergeArgs>(js, k, [](Job& j) { return j.ma; });
    JXG_HIP(launch_merge(ma.data(), k, s));
    if (J.big) {  // levels 128 / 256 px (effort >= 8)
      const auto ba = gather<BigArgs>(js, k, [](Job& j) { return j.ba; });
      JXG_HIP(launch_big(ba.data(), k, s));
      // test hook: JXG_DEBUG_BIGCOST=path writes frame 0's candidate estimates
      if (const char* dbg = std::getenv("JXG_DEBUG_BIGCOST")) {
        const size_t ngc = std::max(1u, J.plan.ng());
        std::vector<float> h(ngc * 30);
        JXG_HIP(hipMemcpyAsync(h.data(), ba[0].cost, h.size() * 4, hipMemcpyDeviceToHost, s));
        JXG_HIP(hipStreamSynchronize(s));
        if (FILE* fp = std::fopen(dbg, "wb")) {  // the 25 estimates of every group
          for (size_t g = 0; g < ngc; g++) std::fwrite(h.data() + g * 30, 4, 25, fp);
          std::fclose(fp);
        }
      }
    }
  }
  for (uint32_t i = 0; i < k; i++) JXG_HIP(hipEventRecord(cs[i]->ev[1], s));
  // (the statistics arenas were zeroed by the front kernel)
  const auto aa = gather<AcArgs>(js, k, [](Job& j) { return j.aa; });
  launch_ac_hist(aa.data(), k, J.plan.ng(), s, J.big);
  JXG_HIP(hipGetLastError());
  return JXG_OK;
}
// varblock lists, LF-stream histograms, and each frame's LF statistics download
static jxg_status launch_lf_stats(Ctx* const* cs, Job* const* js, uint32_t k) {
  if (!batch_ok(cs, js, k)) return JXG_ERR_INTERNAL;
  hipStream_t s = cs[0]->stream;
  const Job& J = *js[0];
  const auto va = gather<VbArgs>(js, k, [](Job& j) { return j.va; });
  launch_vb_list(va.data(), k, J.f.nlf, s);
  const auto la = gather<LfArgs>(js, k, [](Job& j) { return j.la; });
  launch_lf_hist(la.data(), k, J.nchunks, s);
  JXG_HIP(hipGetLastError());
  for (uint32_t i = 0; i < k; i++) {
    const jxg_status st = stage_download_lf(cs[i], *js[i]);
    if (st) return st;
  }
  return JXG_OK;
}
// all of stages B-E (each frame's own AC histogram)
static jxg_status launch_stats(Ctx* const* cs, Job* const* js, uint32_t k) {
  jxg_status st = launch_transform(cs, js, k);
  for (uint32_t i = 0; i < k && !st; i++) st = stage_download_ac(cs[i], *js[i], cs[i]->hist_ac.p);
  return st ? st : launch_lf_stats(cs, js, k);
}

// ---- stage F (host): prefix codes, LF preludes, LfGlobal / HfGlobal,
// scratch layout for the plan's groups and streams ----
static jxg_status stage_codes(Ctx* c, Job& J) {
  hipStream_t s = c->stream;
  const Frame& f = J.f;
  const uint32_t nstreams = J.nstreams;
  JXG_HIP(hipEventSynchronize(c->ev[6]));  // AC statistics on the host; LF kernels may still run
  const Clock::time_point t_codes = Clock::now();
  // prefix codes: one histogram per (used) static cluster; ANS: the static
  // clusters are clustered again into <= kAnsMaxHists groups (the alias
  // inverses must fit the encoder's LDS).  Dense ids in order of first
  // appearance over contexts (oracle/encode.c).
  int group[kMaxClusters];
  if (J.ans) {
    cluster_ans_histograms(c->h_hist_ac.p, kMaxClusters, group);
  } else {
    int ng = 0;
    for (int cl = 0; cl < kMaxClusters; cl++) {
      uint64_t tot = 0;
      for (int k = 0; k < kAlpha; k++) tot += c->h_hist_ac.p[cl * kAlpha + k];
      group[cl] = tot ? ng++ : -1;
    }
  }
  int dense[kMaxClusters];
  std::fill(dense, dense + kMaxClusters, -1);
  int nhist = 0;
  std::vector<uint8_t> ctxmap(kAcCtx);
  for (int ctx = 0; ctx < kAcCtx; ctx++) {
    const int gr = group[ac_cluster(ctx)];
    if (gr >= 0 && dense[gr] < 0) dense[gr] = nhist++;
    ctxmap[ctx] = (uint8_t)(gr < 0 ? 0 : dense[gr]);
  }
  std::vector<PrefixCode> codes(std::max(nhist, 1));
  std::vector<AnsTable> ans_tables(J.ans ? std::max(nhist, 1) : 0);
  std::vector<uint32_t> packed(kMaxClusters * kAlpha, 0);
  if (J.ans) {
    std::vector<uint32_t> dh((size_t)std::max(nhist, 1) * kAlpha, 0);
    for (int cl = 0; cl < kMaxClusters; cl++)
      if (group[cl] >= 0)
        for (int k = 0; k < kAlpha; k++) dh[dense[group[cl]] * kAlpha + k] += c->h_hist_ac.p[cl * kAlpha + k];
    // device table blob (AnsArgs::tab): freq | cum << 16, alias inverses,
    // static cluster -> dense histogram
    JXG_HIP(c->h_ans_tab.ensure(kAnsTabBytes));
    uint8_t* blob = c->h_ans_tab.p;
    std::memset(blob, 0, kAnsTabBytes);
    uint32_t* sym = reinterpret_cast<uint32_t*>(blob);
    uint16_t* inv = reinterpret_cast<uint16_t*>(blob + kAnsInvOff);
    for (int h = 0; h < nhist; h++) {
      AnsTable& t = ans_tables[h];
      t = build_ans_table(dh.data() + h * kAlpha);
      std::copy(t.inv.begin(), t.inv.end(), inv + (size_t)h * 4096);
      for (int k = 0; k < 128; k++) {
        const uint32_t f = t.freq[k];
        if (!f) continue;
        sym[h * 128 + k] = (f - 1) | (uint32_t)t.cum[k] << 12;
      }
    }
    for (int cl = 0; cl < kMaxClusters; cl++)
      blob[kAnsMapOff + cl] = (uint8_t)(group[cl] >= 0 ? dense[group[cl]] : 0);
    J.nhist_ans = (uint32_t)nhist;
    if (J.presets) {
      J.pre_ctxmap = ctxmap;
      J.pre_counts.assign(dh.begin(), dh.begin() + (size_t)nhist * kAlpha);
    }
  } else {
    for (int cl = 0; cl < kMaxClusters; cl++) {
      if (group[cl] < 0) continue;
      const int h = dense[group[cl]];
      codes[h] = build_prefix_code(c->h_hist_ac.p + cl * kAlpha, kAlpha);
      for (int k = 0; k < kAlpha; k++) packed[cl * kAlpha + k] = codes[h].packed(k);
    }
  }
  // LfGlobal / HfGlobal (rank 0): need the AC codes only
  J.lfglobal = BitWriter();
  J.hfglobal = BitWriter();
  if (J.plan.rank == 0) {
    BitWriter& lfglobal = J.lfglobal;
    BitWriter& hfglobal = J.hfglobal;
    lfglobal.put(1, 1);  // LfChannelDequantization.all_default
    if (f.G <= 2048)
      write_u32_sel(lfglobal, 0, 11, f.G - 1);
    else if (f.G <= 4096)
      write_u32_sel(lfglobal, 1, 11, f.G - 2049);
    else if (f.G <= 8192)
      write_u32_sel(lfglobal, 2, 12, f.G - 4097);
    else
      write_u32_sel(lfglobal, 3, 16, f.G - 8193);
    if (f.qdc == 16)
      lfglobal.put(2, 0);
    else if (f.qdc <= 32)
      write_u32_sel(lfglobal, 1, 5, f.qdc - 1);
    else if (f.qdc <= 256)
      write_u32_sel(lfglobal, 2, 8, f.qdc - 1);
    else
      write_u32_sel(lfglobal, 3, 16, f.qdc - 1);
    lfglobal.put(1, 1);  // BlockCtxMap default
    lfglobal.put(1, 1);  // colour correlation default
    lfglobal.put(1, 0);  // GlobalModular: no tree, no channels
    if (!J.presets) {  // (per-rank presets: HfGlobal at assembly, build_hf_presets)
      // the quant tables of the 128 / 256 px kinds the frame uses (e >= 8)
      write_dequant_matrices(hfglobal, J.big ? big_mask(c->h_bigcount.p) : 0u);
      hfglobal.put(ceil_log2(f.ngroups), 0);  // num_hf_presets - 1
      write_u32_sel(hfglobal, 2, 0, 0);        // used_orders = 0
      if (nhist != c->cm_nhist || ctxmap != c->cm_last) {
        c->cm_bits = BitWriter();
        write_context_map(c->cm_bits, ctxmap, nhist);
        c->cm_last = ctxmap;
        c->cm_nhist = nhist;
      }
      if (J.ans)
        write_ans_histograms(hfglobal, ctxmap, nhist, ans_tables, kCfg420, &c->cm_bits);
      else
        write_histograms(hfglobal, ctxmap, nhist, codes, kCfg420, &c->cm_bits);
    }
  }
  // AC layout: the plan's groups in the scratch arena (32-bit aligned); the AC
  // emission is launched at once and runs while the host builds the LF-group
  // codes below
  J.gbase.assign(f.ngroups, 0);
  uint64_t cursor = 0;
  for (uint32_t g : J.plan.groups) {
    J.gbase[g] = cursor;
    const uint64_t nt = (uint64_t)c->h_ntok.p[g * 3] + c->h_ntok.p[g * 3 + 1] + c->h_ntok.p[g * 3 + 2];
    // ANS: <= 16 + raw bits per token (prefix: <= 15 + raw) and the 32-bit state
    const uint64_t bound = (uint64_t)c->h_bound.p[g] + (J.ans ? nt + 32 : 0);
    cursor += (bound + 63) & ~31ull;
  }
  const uint64_t ac_words = (cursor / 32 + 2 + 63) & ~63ull;
  if (!J.ans) JXG_HIP(c->scratch.ensure(ac_words));  // (ANS: with the LF arena below)
  // pinned upload sources: valid until the next frame's stage_codes, which
  // runs after this frame's emission has completed
  JXG_HIP(c->h_codes_ac.ensure(packed.size()));
  std::copy(packed.begin(), packed.end(), c->h_codes_ac.p);
  JXG_HIP(c->h_gbase.ensure(J.gbase.size()));
  std::copy(J.gbase.begin(), J.gbase.end(), c->h_gbase.p);
  if (J.ans) {
    const uint64_t nrec = (uint64_t)std::max(1u, J.plan.ng()) * kGroupTokStride;
    JXG_HIP(c->tval.ensure(nrec));
    JXG_HIP(c->tlen.ensure(nrec));
    JXG_HIP(c->ans_state.ensure(f.ngroups));
    JXG_HIP(c->csum.ensure((uint64_t)std::max(1u, J.plan.ng()) * kAnsMaxChunks));
    JXG_HIP(c->ans_tab.ensure(kAnsTabBytes));
    // chain order: the plan's groups by token count, longest first, so a
    // chain workgroup holds groups of similar length and the workgroups of
    // short groups give their CUs (and 68 KB of LDS each) back early -- the
    // kernel still lasts as long as the longest group
    const uint32_t ng = J.plan.ng();
    JXG_HIP(c->h_ans_order.ensure(ng));
    JXG_HIP(c->ans_order.ensure(ng));
    uint32_t* ord = c->h_ans_order.p;
    for (uint32_t i = 0; i < ng; i++) ord[i] = i;  // launch slots
    const uint32_t* nt = c->h_ntok.p;
    const uint32_t* gl = J.plan.groups.data();
    std::stable_sort(ord, ord + ng, [nt, gl](uint32_t x, uint32_t y) {
      const uint32_t gx = gl[x], gy = gl[y];
      return nt[gx * 3] + nt[gx * 3 + 1] + nt[gx * 3 + 2] > nt[gy * 3] + nt[gy * 3 + 1] + nt[gy * 3 + 2];
    });
    J.max_tokens = 0;
    for (uint32_t g : J.plan.groups)
      J.max_tokens = std::max(J.max_tokens, nt[g * 3] + nt[g * 3 + 1] + nt[g * 3 + 2]);
  }
  const float ms_ac_codes = ms_since(t_codes);
  if (!J.ans) {
    // prefix codes: the AC code tables now, so the AC emission runs while the
    // host builds the LF-group codes (ANS: every table in one upload below)
    JXG_HIP(hipMemcpyAsync(c->up.p, c->h_up.p, c->up_ac, hipMemcpyHostToDevice, s));
    J.aa.scratch = c->scratch.p;
    launch_ac_emit(J.aa, J.plan.ng(), s);
    JXG_HIP(hipGetLastError());
    JXG_HIP(hipMemcpyAsync(c->h_gbits.p, c->gbits.p, f.ngroups * 4, hipMemcpyDeviceToHost, s));
    JXG_HIP(hipEventRecord(c->ev[7], s));
  }
  // (the rANS coder -- a long latency-bound chain that hides the LF-code
  // construction anyway -- is launched by stage_emit)

  // LF-group stream codes and preludes (the plan's LF groups)
  JXG_HIP(hipEventSynchronize(c->ev[2]));  // LF statistics (stage_download_lf)
  const Clock::time_point t_lf = Clock::now();
  const size_t nlfcodes = (size_t)nstreams * 4 * kAlpha;
  JXG_HIP(c->h_lfcodes.ensure(nlfcodes));
  uint32_t* lfpacked = c->h_lfcodes.p;
  std::fill(lfpacked, lfpacked + nlfcodes, 0u);
  J.preA.assign(f.nlf, BitWriter());
  J.preB.assign(f.nlf, BitWriter());
  for (uint32_t lg = 0; lg < f.nlf; lg++) {
    if (!J.plan.owns_lf(lg)) continue;
    const uint32_t bx0 = (lg % f.lfxs) * 256, by0 = (lg / f.lfxs) * 256;
    const uint32_t bw = std::min(256u, f.bxs - bx0), bh = std::min(256u, f.bys - by0);
    for (int sidx = 0; sidx < 2; sidx++) {
      const uint32_t sid = lg * 2 + sidx;
      const int nleaves = sidx == 0 ? 3 : 4;
      std::vector<PrefixCode> lc(nleaves);
      for (int l = 0; l < nleaves; l++) {
        lc[l] = build_prefix_code(c->h_lfhist.p + ((size_t)sid * 4 + l) * kAlpha, kAlpha);
        for (int k = 0; k < kAlpha; k++) lfpacked[((size_t)sid * 4 + l) * kAlpha + k] = lc[l].packed(k);
      }
      if (sidx == 0) {
        J.preA[lg].put(2, 0);  // extra_precision
        write_modular_prelude(J.preA[lg], kDcTree, 5, 3, lc);
      } else {
        J.preB[lg].put(ceil_log2(bw * bh), c->h_vcount.p[lg] - 1);  // varblock count - 1
        write_modular_prelude(J.preB[lg], (J.lf >> 1) ? kMetaTreeEpf : kMetaTree, 7, 4, lc);
      }
    }
  }
  // LF layout: the plan's LF streams in their own arena (32-bit aligned)
  J.sbase.assign(nstreams, 0);
  cursor = 0;
  for (uint32_t i = 0; i < nstreams; i++) {
    J.sbase[i] = cursor;
    if (J.plan.owns_lf(i / 2)) cursor += ((uint64_t)c->h_sbound.p[i] + 63) & ~31ull;
  }
  const uint64_t lf_words = cursor / 32 + 2;
  JXG_HIP(c->h_sbase.ensure(J.sbase.size()));
  std::copy(J.sbase.begin(), J.sbase.end(), c->h_sbase.p);
  if (J.ans) {
    // one arena for the AC and LF bits (no fill: the chains clear their
    // ranges, lf_code stores whole words) and every table in one upload
    JXG_HIP(c->scratch.ensure(ac_words + lf_words));
    c->lf_scratch = c->scratch.p + ac_words;
    J.aa.scratch = c->scratch.p;
    JXG_HIP(hipMemcpyAsync(c->up.p + c->up_gbase, c->h_up.p + c->up_gbase,
                           c->up_bytes - c->up_gbase, hipMemcpyHostToDevice, s));
  } else {
    JXG_HIP(c->scratch_lf.ensure(lf_words));
    c->lf_scratch = c->scratch_lf.p;
    JXG_HIP(hipMemcpyAsync(c->up.p + c->up_lf, c->h_up.p + c->up_lf, c->up_bytes - c->up_lf,
                           hipMemcpyHostToDevice, s));
  }
  J.ms_codes = ms_ac_codes + ms_since(t_lf);
  return JXG_OK;
}

// ---- stage G: rANS coder (the prefix-code AC emission was launched by
// stage_codes), LF-stream bit emission, bit counts to the host ----
static void build_emit(Ctx* c, Job& J) {
  J.la.scratch = c->lf_scratch;
  if (!J.ans) return;
  AnsArgs& na = J.na;
  na = AnsArgs{};
  na.tokens = c->tokens.p;
  na.val = c->tval.p;
  na.len = c->tlen.p;
  na.ntok = c->ntok.p;
  na.bandtok = c->bandtok.p;
  na.tab = c->ans_tab.p;
  na.nhist = J.nhist_ans;
  na.state = c->ans_state.p;
  na.base = c->gbase.p;
  na.scratch = c->scratch.p;
  na.bits = c->gbits.p;
  na.g0 = J.plan.g0();
  na.n = J.plan.ng();
  na.glist = J.aa.glist;
  na.order = c->ans_order.p;
  na.csum = c->csum.p;
  na.max_tokens = J.max_tokens;
}
// the emission of k frames sharing a stream (codes built): rANS chains + bit
// placement and LF streams as one launch each, then each frame's bit counts
// to the host
static jxg_status launch_emit(Ctx* const* cs, Job* const* js, uint32_t k) {
  if (!batch_ok(cs, js, k)) return JXG_ERR_INTERNAL;
  hipStream_t s = cs[0]->stream;
  const Job& J = *js[0];
  for (uint32_t i = 0; i < k; i++) build_emit(cs[i], *js[i]);
  if (J.ans) {
    const auto na = gather<AnsArgs>(js, k, [](Job& j) { return j.na; });
    launch_ans(na.data(), k, s);
    JXG_HIP(hipGetLastError());
  }
  const auto la = gather<LfArgs>(js, k, [](Job& j) { return j.la; });
  launch_lf_code(la.data(), k, J.nchunks, s);
  JXG_HIP(hipGetLastError());
  for (uint32_t i = 0; i < k; i++) {
    Ctx* c = cs[i];
    const Frame& f = js[i]->f;
    if (J.ans) {  // [gbits | stream_bits]: one copy
      JXG_HIP(hipMemcpyAsync(c->h_bits.p, c->bits.p, ((size_t)f.ngroups + js[i]->nstreams) * 4,
                             hipMemcpyDeviceToHost, s));
      JXG_HIP(hipEventRecord(c->ev[7], s));
    } else {
      JXG_HIP(hipMemcpyAsync(c->h_sbits.p, c->stream_bits.p, js[i]->nstreams * 4,
                             hipMemcpyDeviceToHost, s));
    }
    JXG_HIP(hipEventRecord(c->ev[3], s));
  }
  return JXG_OK;
}
static jxg_status stage_emit(Ctx* c, Job& J, bool sync = true) {
  Job* jp = &J;
  jxg_status st = launch_emit(&c, &jp, 1);
  if (!st && sync) st = wait_emission(c, J);
  return st;
}

// ---- stage H: concatenation.  Sections are bit-exact piece lists (host
// chunks + device scratch ranges).  full: headers + TOC + all sections into
// one codestream; shard: the plan's sections, each byte-aligned, back to back
// (`section_ids` receives their TOC indices) ----
struct Piece {
  int arena;  // 0 AC scratch, 1 host chunk, 2 LF scratch
  uint64_t src, nbits;
};
static jxg_status stage_concat(Ctx* c, Job& J, bool full, std::vector<uint32_t>* section_ids,
                               std::vector<uint32_t>* section_bytes, uint8_t** host_out,
                               size_t* out_bytes) {
  hipStream_t s = c->stream;
  const Frame& f = J.f;
  std::vector<std::vector<Piece>> sections;
  std::vector<uint32_t> ids;
  std::vector<uint32_t> chunk_words;
  auto add_chunk = [&](const BitWriter& bw) -> Piece {
    Piece p{1, (uint64_t)chunk_words.size() * 32, bw.bits()};
    auto wv = bw.words32();
    chunk_words.insert(chunk_words.end(), wv.begin(), wv.end());
    return p;
  };
  if (J.plan.rank == 0) {
    sections.push_back({add_chunk(J.lfglobal)});
    ids.push_back(0);
  }
  for (uint32_t lg = 0; lg < f.nlf; lg++) {
    if (!J.plan.owns_lf(lg)) continue;
    sections.push_back({add_chunk(J.preA[lg]), Piece{2, J.sbase[lg * 2], c->h_sbits.p[lg * 2]},
                        add_chunk(J.preB[lg]),
                        Piece{2, J.sbase[lg * 2 + 1], c->h_sbits.p[lg * 2 + 1]}});
    ids.push_back(1 + lg);
  }
  if (J.plan.rank == 0 && !J.presets) {
    sections.push_back({add_chunk(J.hfglobal)});
    ids.push_back(1 + f.nlf);
  }
  // per-rank presets: every pass group starts with its preset index
  BitWriter sel;
  if (J.presets) sel.put(ceil_log2(J.plan.world), J.plan.rank);
  for (uint32_t g : J.plan.groups) {
    if (J.presets)
      sections.push_back({add_chunk(sel), Piece{0, J.gbase[g], c->h_gbits.p[g]}});
    else
      sections.push_back({Piece{0, J.gbase[g], c->h_gbits.p[g]}});
    ids.push_back(2 + f.nlf + g);
  }
  const bool single = full && f.ngroups == 1;
  std::vector<uint32_t> sizes;
  if (single) {
    uint64_t total = 0;
    for (auto& sec : sections)
      for (auto& p : sec) total += p.nbits;
    sizes.push_back((uint32_t)((total + 7) / 8));
  } else {
    for (auto& sec : sections) {
      uint64_t t = 0;
      for (auto& p : sec) t += p.nbits;
      sizes.push_back((uint32_t)((t + 7) / 8));
    }
  }
  std::vector<ConcatPiece> cps;
  uint64_t dst = 0, max_words = 0;
  auto emit_piece = [&](const Piece& p) {
    if (p.nbits) {
      cps.push_back({p.src, dst, p.nbits, (uint32_t)p.arena, 0});
      max_words = std::max<uint64_t>(max_words, (p.nbits + 31) / 32);
    }
    dst += p.nbits;
  };
  if (full) {
    BitWriter head;
    write_headers(head, J.w, J.h, J.lf);
    write_toc(head, sizes);
    emit_piece(add_chunk(head));
  }
  for (auto& sec : sections) {
    for (auto& p : sec) emit_piece(p);
    if (!single) dst = (dst + 7) & ~7ull;
  }
  dst = (dst + 7) & ~7ull;
  const size_t nbytes = (size_t)(dst / 8);
  const size_t out_words = (nbytes + 3) / 4 + 1;
  chunk_words.push_back(0);  // read-ahead guard
  // pieces and chunk words through one pinned staging buffer, one upload
  // (the previous frame of this context has completed: the staging is free)
  const size_t pb = (std::max<size_t>(cps.size(), 1) * sizeof(ConcatPiece) + 255) & ~(size_t)255;
  const size_t wb = chunk_words.size() * 4;
  JXG_HIP(c->cat.ensure(pb + wb));
  JXG_HIP(c->h_cat.ensure(pb + wb));
  JXG_HIP(c->out.ensure(out_words));
  uint8_t* ho = nullptr;
  if (host_out) {  // else the bytes stay in c->out (device)
    ho = out_alloc(out_words * 4);
    if (!ho) return JXG_ERR_OOM;
  }
  if (!cps.empty()) std::memcpy(c->h_cat.p, cps.data(), cps.size() * sizeof(ConcatPiece));
  std::memcpy(c->h_cat.p + pb, chunk_words.data(), wb);
  JXG_HIP(hipMemcpyAsync(c->cat.p, c->h_cat.p, pb + wb, hipMemcpyHostToDevice, s));
  launch_concat(reinterpret_cast<const ConcatPiece*>(c->cat.p), (uint32_t)cps.size(), out_words,
                c->scratch.p, reinterpret_cast<const uint32_t*>(c->cat.p + pb), c->lf_scratch,
                c->out.p, s);
  JXG_HIP(hipGetLastError());
  if (ho && hipMemcpyAsync(ho, c->out.p, out_words * 4, hipMemcpyDeviceToHost, s) != hipSuccess) {
    out_release(ho);
    return JXG_ERR_HIP;
  }
  JXG_HIP(hipEventRecord(c->ev[4], s));
  if (host_out) *host_out = ho;
  *out_bytes = nbytes;
  if (section_ids) *section_ids = ids;
  if (section_bytes) *section_bytes = sizes;
  return JXG_OK;
}

// Full codestream of a multi-group frame with the AC block moved early: the
// pass-group sections (the bulk of the bytes) are concatenated on stream2 as
// soon as the AC emission is done and copied to the END region of the host
// block while the LF streams are still being emitted; the prefix (headers,
// TOC, LfGlobal, LF groups, HfGlobal) follows on the main stream and lands
// right before it.  Same bytes as stage_concat(full).
static jxg_status stage_concat_split(Ctx* c, Job& J, uint8_t** host_out, size_t* out_bytes) {
  if (!c->stream2 && hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess)
    return JXG_ERR_HIP;  // created on first use: only lone contexts take this path
  hipStream_t s = c->stream, s2 = c->stream2;
  const Frame& f = J.f;
  JXG_HIP(hipEventSynchronize(c->ev[7]));  // AC emission done, its bit counts on the host
  const uint32_t g0 = J.plan.g0(), ng = J.plan.ng();  // (one context: all groups)
  JXG_HIP(c->h_pieces_ac.ensure(std::max<uint32_t>(ng, 1)));
  std::vector<uint32_t> ac_sizes(ng);
  uint64_t dst = 0, max_words = 0;
  uint32_t np = 0;
  for (uint32_t i = 0; i < ng; i++) {
    const uint64_t nb = c->h_gbits.p[g0 + i];
    ac_sizes[i] = (uint32_t)((nb + 7) / 8);
    if (nb) {
      c->h_pieces_ac.p[np++] = {J.gbase[g0 + i], dst, nb, 0u, 0u};
      max_words = std::max<uint64_t>(max_words, (nb + 31) / 32);
    }
    dst += (uint64_t)ac_sizes[i] * 8;
  }
  const size_t ac_bytes = (size_t)(dst / 8);
  // prefix upper bound: chunks + LF stream bounds + headers / TOC + slack for
  // the back reference
  uint64_t pbits = J.lfglobal.bits() + J.hfglobal.bits() + 16;
  for (uint32_t lg = 0; lg < f.nlf; lg++)
    if (J.plan.owns_lf(lg))
      pbits += J.preA[lg].bits() + J.preB[lg].bits() + c->h_sbound.p[lg * 2] +
               c->h_sbound.p[lg * 2 + 1] + 8;
  const size_t nsec = 2 + (size_t)f.nlf + f.ngroups;
  size_t pmax = (size_t)(pbits / 8) + 256 + 4 * nsec + 16 + kOutHdr;
  pmax = (pmax + 63) & ~(size_t)63;
  uint8_t* ho = out_alloc(pmax + ac_bytes + 8);
  if (!ho) return JXG_ERR_OOM;
  auto fail = [&](jxg_status e) {
    (void)hipStreamSynchronize(s2);
    (void)hipStreamSynchronize(s);
    out_release(ho);
    return e;
  };
  const size_t ac_words = ac_bytes / 4 + 2;
  if (c->out_ac.ensure(ac_words) != hipSuccess ||
      c->pieces_ac.ensure(std::max<uint32_t>(np, 1)) != hipSuccess)
    return fail(JXG_ERR_HIP);
  if (hipStreamWaitEvent(s2, c->ev[7], 0) != hipSuccess ||
      (np && hipMemcpyAsync(c->pieces_ac.p, c->h_pieces_ac.p, np * sizeof(ConcatPiece),
                            hipMemcpyHostToDevice, s2) != hipSuccess))
    return fail(JXG_ERR_HIP);
  launch_concat(c->pieces_ac.p, np, ac_words, c->scratch.p, c->chunks.p, nullptr, c->out_ac.p, s2);
  if (hipGetLastError() != hipSuccess ||
      (ac_bytes && hipMemcpyAsync(ho + pmax, c->out_ac.p, ac_bytes, hipMemcpyDeviceToHost, s2) !=
                       hipSuccess) ||
      hipEventRecord(c->ev[8], s2) != hipSuccess)
    return fail(JXG_ERR_HIP);

  // prefix, after the LF emission (stage_emit without its sync)
  if (hipStreamSynchronize(s) != hipSuccess) return fail(JXG_ERR_HIP);
  const Clock::time_point t_layout = Clock::now();
  std::vector<std::vector<Piece>> sections;
  std::vector<uint32_t> chunk_words;
  auto add_chunk = [&](const BitWriter& bw) -> Piece {
    Piece p{1, (uint64_t)chunk_words.size() * 32, bw.bits()};
    auto wv = bw.words32();
    chunk_words.insert(chunk_words.end(), wv.begin(), wv.end());
    return p;
  };
  sections.push_back({add_chunk(J.lfglobal)});
  for (uint32_t lg = 0; lg < f.nlf; lg++)
    sections.push_back({add_chunk(J.preA[lg]), Piece{2, J.sbase[lg * 2], c->h_sbits.p[lg * 2]},
                        add_chunk(J.preB[lg]),
                        Piece{2, J.sbase[lg * 2 + 1], c->h_sbits.p[lg * 2 + 1]}});
  sections.push_back({add_chunk(J.hfglobal)});
  std::vector<uint32_t> sizes;
  for (auto& sec : sections) {
    uint64_t t = 0;
    for (auto& p : sec) t += p.nbits;
    sizes.push_back((uint32_t)((t + 7) / 8));
  }
  sizes.insert(sizes.end(), ac_sizes.begin(), ac_sizes.end());
  std::vector<ConcatPiece> cps;
  dst = 0;
  max_words = 0;
  auto emit_piece = [&](const Piece& p) {
    if (p.nbits) {
      cps.push_back({p.src, dst, p.nbits, (uint32_t)p.arena, 0});
      max_words = std::max<uint64_t>(max_words, (p.nbits + 31) / 32);
    }
    dst += p.nbits;
  };
  BitWriter head;
  write_headers(head, J.w, J.h, J.lf);
  write_toc(head, sizes);
  emit_piece(add_chunk(head));
  for (auto& sec : sections) {
    for (auto& p : sec) emit_piece(p);
    dst = (dst + 7) & ~7ull;
  }
  const size_t pbytes = (size_t)(dst / 8);
  // prefix bound violated (or forced, JXG_FLAG_FORCE_ONE_STREAM): one-stream
  // assembly instead
  if (pbytes + kOutHdr > pmax || (c->params.flags & JXG_FLAG_FORCE_ONE_STREAM)) {
    if (hipStreamSynchronize(s2) != hipSuccess) return fail(JXG_ERR_HIP);
    out_release(ho);
    const jxg_status st = stage_concat(c, J, true, nullptr, nullptr, host_out, out_bytes);
    J.ms_layout = ms_since(t_layout);
    return st;
  }
  const size_t out_words = (pbytes + 3) / 4 + 1;
  chunk_words.push_back(0);  // read-ahead guard
  if (c->chunks.ensure(chunk_words.size()) != hipSuccess ||
      c->pieces.ensure(std::max<size_t>(cps.size(), 1)) != hipSuccess ||
      c->out.ensure(out_words) != hipSuccess)
    return fail(JXG_ERR_HIP);
  uint8_t* data = ho + pmax - pbytes;
  if (hipMemcpyAsync(c->chunks.p, chunk_words.data(), chunk_words.size() * 4,
                     hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(c->pieces.p, cps.data(), cps.size() * sizeof(ConcatPiece),
                     hipMemcpyHostToDevice, s) != hipSuccess)
    return fail(JXG_ERR_HIP);
  launch_concat(c->pieces.p, (uint32_t)cps.size(), out_words, c->scratch.p, c->chunks.p,
                c->lf_scratch, c->out.p, s);
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(data, c->out.p, pbytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamWaitEvent(s, c->ev[8], 0) != hipSuccess ||
      hipEventRecord(c->ev[4], s) != hipSuccess)
    return fail(JXG_ERR_HIP);
  J.ms_layout = ms_since(t_layout);
  out_set_backref(data, ho);
  *host_out = data;
  *out_bytes = pbytes + ac_bytes;
  return JXG_OK;
}

// Device inputs (jxg_set_input_stream): `lane`'s stream is ordered after the
// work the caller has submitted to its input stream so far; without an input
// stream the caller's writes must be complete before the call (include/jxg.h).
static jxg_status order_input(Ctx* owner, Ctx* lane) {
  if (!owner->in_stream) return JXG_OK;
  if (!lane->ev_in && make_event(&lane->ev_in, hipEventDisableTiming) != hipSuccess)
    return JXG_ERR_HIP;
  JXG_HIP(hipEventRecord(lane->ev_in, owner->in_stream));
  JXG_HIP(hipStreamWaitEvent(lane->stream, lane->ev_in, 0));
  return JXG_OK;
}

// ---- one frame, in three phases (encode_device runs them back to back; the
// streaming pipeline interleaves the phases of consecutive frames) ----
// phase 1: buffers, front end + merge stage + AC / LF statistics and their
// downloads, all launched asynchronously on the context's stream
// (rank, world): a shard of a frame whose plan needs no record exchange and,
// with world > 1, ANS (one HF preset per rank): no collective before assembly
// the frame's plan, buffers and argument blocks (nothing launched)
static jxg_status enc_prepare(Ctx* c, Job& J, const uint8_t* d_rgb, uint32_t w, uint32_t h,
                              size_t stride, uint32_t rank, uint32_t world) {
  J.f = make_frame(w, h, c->params.distance);
  J.plan = make_plan(J.f, rank, world);
  J.w = w;
  J.h = h;
  J.stride = stride;
  J.d_rgb = d_rgb;
  jxg_status st = stage_alloc(c, J);
  if (st) return st;
  J.presets = J.ans && world > 1;
  return build_front(c, J);
}
static jxg_status enc_launch(Ctx* c, Job& J, const uint8_t* d_rgb, uint32_t w, uint32_t h,
                             size_t stride, uint32_t rank = 0, uint32_t world = 1) {
  jxg_status st = enc_prepare(c, J, d_rgb, w, h, stride, rank, world);
  if (st) return st;
  Job* jp = &J;
  return launch_stats(&c, &jp, 1);
}

// phase 2: (host, after the statistics arrive) codes and headers; AC / LF
// emission launched
static jxg_status enc_codes(Ctx* c, Job& J, bool sync) {
  const jxg_status st = stage_codes(c, J);
  if (st) return st;
  return stage_emit(c, J, sync);
}

// phase 3: assembly, the codestream in host memory, stats
// phase 3 in two halves: enc_finish_start (the emission's bit counts on the
// host -> layout, concat and the codestream's D2H enqueued) and enc_finish_end
// (wait for them, stats).  The streaming pipeline starts a frame's assembly
// as soon as its emission is done and ends it when the frame is taken.
static jxg_status enc_finish_start(Ctx* c, Job& J, bool split) {
  const Clock::time_point t_layout = Clock::now();
  J.host_out = nullptr;
  J.out_bytes = 0;
  jxg_status st;
  if (split) {
    if ((st = stage_concat_split(c, J, &J.host_out, &J.out_bytes))) return st;
  } else {
    // the emission's bit counts on the host (stage_emit may have returned
    // without waiting)
    if ((st = wait_emission(c, J))) return st;
    if ((st = stage_concat(c, J, true, nullptr, nullptr, &J.host_out, &J.out_bytes))) return st;
  }
  J.ms_finish_layout = split ? J.ms_layout : ms_since(t_layout);
  return JXG_OK;
}
// the frame's stats (the lane's jxg_stats); `assembled`: the assembly has
// completed (ev[4]), else its time is left out
static void enc_stats(Ctx* c, Job& J, size_t out_bytes, float ms_layout, bool assembled,
                      const std::vector<int16_t>* m_ac16, Clock::time_point t_call) {
  const jxg_params& P = c->params;
  const Frame& f = J.f;
  const size_t nb = (size_t)f.bxs * f.bys;
  jxg_stats& S = c->stats;
  S = jxg_stats{};
  S.xsize = J.w;
  S.ysize = J.h;
  S.xsize_blocks = f.bxs;
  S.ysize_blocks = f.bys;
  S.num_groups = f.ngroups;
  S.num_lf_groups = f.nlf;
  S.global_scale = f.G;
  S.quant_dc = f.qdc;
  S.bytes = out_bytes;
  c->m_ntok.assign(c->h_ntok.p, c->h_ntok.p + f.ngroups * 3);
  S.ac_tokens = c->m_ntok.data();
  if ((P.flags & JXG_FLAG_KEEP_MAPS) && m_ac16) {
    // coefficients in natural-order slices, widened to int32 for the caller
    for (size_t i = 0; i < nb * 192; i++) c->m_ac[i] = (*m_ac16)[i];
    S.ac_strategy = c->m_acs.data();
    S.quant_field = c->m_qf.data();
    S.dc = c->m_dc.data();
    S.ac = c->m_ac.data();
    S.homogeneity = J.homog ? c->m_homog.data() : nullptr;
  }
  S.ms_front = elapsed(c->ev[0], c->ev[1]);
  S.ms_front_kernel = elapsed(c->ev[9], c->ev[5]);
  S.ms_aq = elapsed(c->ev[0], c->ev[9]);
  S.ms_histogram = elapsed(c->ev[1], c->ev[2]);
  S.ms_emit = elapsed(c->ev[2], c->ev[3]);
  S.ms_assemble = assembled ? elapsed(c->ev[3], c->ev[4]) : 0.0f;
  S.ms_total = elapsed(c->ev[0], assembled ? c->ev[4] : c->ev[3]);
  S.ms_host_codes = J.ms_codes;
  S.ms_host_layout = ms_layout;
  S.ms_host_call = ms_since(t_call);
}
static jxg_status enc_finish_end(Ctx* c, Job& J, jxg_buffer* out, Clock::time_point t_call) {
  hipStream_t s = c->stream;
  const jxg_params& P = c->params;
  const Frame& f = J.f;
  const size_t nb = (size_t)f.bxs * f.bys;
  uint8_t* host_out = J.host_out;
  const size_t out_bytes = J.out_bytes;
  J.host_out = nullptr;
  std::vector<int16_t> m_ac16_tmp;
  if (P.flags & JXG_FLAG_KEEP_MAPS) {
    c->m_acs.resize(nb);
    c->m_qf.resize(nb);
    c->m_dc.resize(nb * 3);
    c->m_ac.resize(nb * 192);
    JXG_HIP(hipMemcpyAsync(c->m_acs.data(), c->acs.p, nb, hipMemcpyDeviceToHost, s));
    JXG_HIP(hipMemcpyAsync(c->m_qf.data(), c->qf.p, nb, hipMemcpyDeviceToHost, s));
    JXG_HIP(hipMemcpyAsync(c->m_dc.data(), c->dc.p, nb * 12, hipMemcpyDeviceToHost, s));
    m_ac16_tmp.resize(nb * 192);
    JXG_HIP(hipMemcpyAsync(m_ac16_tmp.data(), c->ac.p, nb * 192 * 2, hipMemcpyDeviceToHost, s));
    if (J.homog) {
      c->m_homog.resize(nb * 3);
      JXG_HIP(hipMemcpyAsync(c->m_homog.data(), c->homog.p, nb * 12, hipMemcpyDeviceToHost, s));
    }
  }
  if (hipStreamSynchronize(s) != hipSuccess) {
    out_release(host_out);
    return JXG_ERR_HIP;
  }
  out->data = host_out;
  out->size = out_bytes;
  enc_stats(c, J, out_bytes, J.ms_finish_layout, true, &m_ac16_tmp, t_call);
  return JXG_OK;
}
static jxg_status enc_finish(Ctx* c, Job& J, bool split, jxg_buffer* out,
                             Clock::time_point t_call) {
  const jxg_status st = enc_finish_start(c, J, split);
  return st ? st : enc_finish_end(c, J, out, t_call);
}

static bool pipe_busy(const Ctx* c);
// a lane of another context (its own stream); not counted in g_live_ctx
static jxg_status ctx_new_lane(const jxg_params& params, Ctx** out) {
  *out = nullptr;
  Ctx* c = new (std::nothrow) Ctx();
  if (!c) return JXG_ERR_OOM;
  c->params = params;
  c->owned_lane = true;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return JXG_ERR_HIP;
  }
  for (auto& e : c->ev)
    if (make_event(&e, 0) != hipSuccess) {
      jxg_destroy(reinterpret_cast<jxg_ctx*>(c));
      return JXG_ERR_HIP;
    }
  *out = c;
  return JXG_OK;
}

static jxg_status encode_device(Ctx* c, const uint8_t* d_rgb, uint32_t w, uint32_t h,
                                size_t stride, jxg_buffer* out, Clock::time_point t_call) {
  // streamed frames in flight use this context as a lane (and its helper
  // threads its host state): one-at-a-time calls wait until they are received
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  Job J;
  jxg_status st = enc_launch(c, J, d_rgb, w, h, stride);
  if (st) return st;
  // split assembly for a single context of a multi-group frame (single-group
  // frames are one section; several contexts keep the one-stream assembly)
  const bool split = J.f.ngroups > 1 && g_live_ctx.load() <= 1;
  if ((st = enc_codes(c, J, !split))) return st;
  return enc_finish(c, J, split, out, t_call);
}

// ---------------------------------------------------------------------------
// streaming encode (jxg_submit_rgb8[_device] / jxg_receive): a software
// pipeline over lanes (the caller's context plus lanes it owns, one stream
// each), driven by the caller's one host thread.  A frame's rANS chains last
// as long as its longest pass group's whatever the frame size, and a lane's
// stream is held by a frame from its front end to its assembly, so the
// frames in flight -- not the GPU's throughput -- bound small frames
// (profiles/r04f: ms per 1080p frame falls as 1 / lanes up to the 12 lanes
// the hardware queues allow).  So a lane carries a SUPER-FRAME: up to
// kMaxBatch frames of one size in slots (contexts with their own buffers
// sharing the lane's stream) that go through every per-frame kernel as one
// batched launch (blockIdx.z = the frame): front end, merge stage,
// statistics, then -- once a helper thread has built the codes of every
// frame of the batch -- rANS chains + bit placement and LF streams.  submit:
//   the frame joins the open batch (a free lane's next slot; completing the
//   oldest frames frees one) -> a full batch (or one of another size) is
//   launched, its codes queued on the helper threads; the last helper to
//   finish launches the batch's emission.
// Frames complete in submission order (deferred finish: layout, concat and
// the codestream's D2H enqueued; jxg_receive waits for the copy).  ~3570 pass
// groups in flight: 8K 7 lanes x 1, 1080p 12 lanes x 4.  Every lane needs
// its own hardware queue (GPU_MAX_HW_QUEUES > lanes, bench.py sets 16).
// ---------------------------------------------------------------------------
#ifndef JXG_PIPE_CHAIN_GROUPS  // (experiment builds override it: tools/build_variant.sh)
#define JXG_PIPE_CHAIN_GROUPS 3570
#endif
constexpr uint32_t kPipeMaxLanes = 12, kPipeMinLanes = 4, kPipeChainGroups = JXG_PIPE_CHAIN_GROUPS;
// Hardware queues of this process (GPU_MAX_HW_QUEUES as HIP read it at start
// up; HIP's default is 4).  Lanes beyond queues - 1 (one is left for the
// caller's own stream) would share a queue with another lane and serialise
// its kernels (5.5 vs 6.7 GPix/s at 8K), so the depth never
// exceeds it: a caller that wants the full depth raises the variable (at most
// 32) before HIP initialises, as bench.py and tests/conftest.py do.
static uint32_t hw_queues() {
  const char* e = std::getenv("GPU_MAX_HW_QUEUES");
  const long q = e && *e ? std::strtol(e, nullptr, 10) : 4;
  return (uint32_t)std::min<long>(32, std::max<long>(1, q));
}
// lanes and frames per lane (batch) for a frame / shard of `ngroups` pass
// groups and `ntiles` 64x64 tiles.  Batches only for frames of at most
// kPipeBatchTiles tiles (1080p: 510, a rank's eighth of 8K: 1080): 4K in
// batches of 3 fell from 8.1 to 4.8 GPix/s (profiles/r04h) -- a frame that
// fills the chip gains nothing from sharing a launch and its lane's latency
// grows with every frame in the batch; the 8K eighth gains 0.63 -> 0.56 ms
// per frame, a quarter (2160 tiles) nothing (profiles/r04k).
#ifndef JXG_PIPE_BATCH_TILES  // (experiment builds override it: tools/build_variant.sh)
#define JXG_PIPE_BATCH_TILES 1280
#endif
constexpr uint32_t kPipeBatchTiles = JXG_PIPE_BATCH_TILES;
struct PipeShape {
  uint32_t lanes, batch;
  uint32_t frames() const { return lanes * batch; }
  // shard frames that may be pending with the next submit always accepted:
  // unwritten frames (written oldest first, so only the oldest batch is
  // partly written) leave a lane free while they fill at most lanes - 1
  // batches -- jxg_pipeline_depth
  uint32_t pending() const { return (lanes - 1) * batch + 1; }
};
// (cap: jxg_set_pipeline_lanes, 0 = none)
static PipeShape pipe_shape(uint32_t ngroups, uint32_t ntiles, uint32_t cap) {
  const uint32_t want = (kPipeChainGroups + ngroups - 1) / std::max(1u, ngroups);  // frames
  uint32_t lmax = std::max(2u, std::min(kPipeMaxLanes, hw_queues() - 1));
  if (cap) lmax = std::min(lmax, cap);
  const uint32_t kt = ntiles <= kPipeBatchTiles ? kMaxBatch : 1u;
  const uint32_t k = std::min(kt, std::max(1u, (want + lmax - 1) / lmax));
  const uint32_t lanes = std::min(lmax, std::max(std::min(kPipeMinLanes, lmax), (want + k - 1) / k));
  return PipeShape{lanes, k};
}
// a completed frame: its codestream (pinned host block) and stats; `ev`: the
// codestream's D2H, still in flight when the frame was completed (deferred
// finish) -- jxg_receive waits for it
struct PipeDone {
  jxg_buffer buf;
  jxg_stats stats;
  hipEvent_t ev;
};
struct PipeBatch;
struct PipeFrame {
  Ctx* lane = nullptr;   // the frame's slot (its buffers; the lane's stream)
  Ctx* owner = nullptr;  // the lane
  std::shared_ptr<PipeBatch> batch;
  Job J;
  int phase = 0;  // 0: in the open batch; 1: statistics launched; 2: emission launched
  bool shard = false;
  Clock::time_point t0;
  const uint8_t* src = nullptr;  // the device input (phase 0)
  uint32_t w = 0, h = 0, rank = 0, world = 1;
  size_t stride = 0;
  std::future<jxg_status> codes;  // valid while a helper builds the codes
};
// frames launched together on one lane; the last of their codes launches the
// batch's emission
struct PipeBatch {
  Ctx* owner = nullptr;
  uint32_t w = 0, h = 0, rank = 0, world = 1;
  bool shard = false;
  std::vector<PipeFrame*> frames;
  std::atomic<int> left{0};         // codes not yet built
  std::atomic<int> err{JXG_OK};     // a frame's codes or the emission failed
};
// the codes of frame fr of its batch (a helper thread, or inline); the
// batch's last one launches the emission of all its frames
static jxg_status pipe_codes(PipeFrame* fr) {
  PipeBatch& B = *fr->batch;
  jxg_status st = stage_codes(fr->lane, fr->J);
  if (st) B.err.store(st);
  if (B.left.fetch_sub(1) == 1 && !B.err.load()) {
    std::vector<Ctx*> cs;
    std::vector<Job*> js;
    for (PipeFrame* q : B.frames) {
      cs.push_back(q->lane);
      js.push_back(&q->J);
    }
    const jxg_status e = launch_emit(cs.data(), js.data(), (uint32_t)cs.size());
    if (e) B.err.store(e);
  }
  return st;
}
// the helper's codes of a frame -> phase 2 (on an error the caller aborts)
static jxg_status pipe_join_codes(PipeFrame& fr) {
  jxg_status st = JXG_OK;
  if (fr.codes.valid()) {
    st = fr.codes.get();
    fr.phase = 2;
  }
  if (!st && fr.batch) st = (jxg_status)fr.batch->err.load();
  return st;
}
constexpr int kPipeHelpers = 6;  // codes of a batch (<= kMaxBatch) and the next one's in parallel

struct Pipe {
  std::vector<std::unique_ptr<PipeFrame>> inflight;  // submission order
  std::vector<PipeDone> done;                        // submission order
  std::vector<hipEvent_t> evfree;                    // PipeDone::ev pool
  // shard frames whose sections are emitted and payload head built; each
  // holds its lane (sections in lane->out) until jxg_shard_write_next
  std::vector<std::unique_ptr<PipeFrame>> ready;
  uint64_t submitted = 0;
  int mode = 0;  // 1 whole frames, 2 shards (while any frame is pending)
  uint32_t depth = 0;  // frames in flight (lanes x batch)
  std::shared_ptr<PipeBatch> open;   // frames submitted, not yet launched
  std::deque<hipEvent_t> writes;    // jxg_shard_write_next copies in flight, oldest first
  std::unique_ptr<Helpers> helpers;  // created with the first helper task
  ~Pipe() {
    for (auto& d : done)
      if (d.ev) {
        (void)hipEventSynchronize(d.ev);  // its D2H writes the codestream block
        (void)hipEventDestroy(d.ev);
      }
    for (hipEvent_t e : evfree) (void)hipEventDestroy(e);
  }
};
// the oldest completed frame's codestream is on the host (its D2H done)
static jxg_status pipe_done_wait(Pipe& p, PipeDone& d) {
  if (!d.ev) return JXG_OK;
  const hipError_t e = hipEventSynchronize(d.ev);
  p.evfree.push_back(d.ev);
  d.ev = nullptr;
  return e == hipSuccess ? JXG_OK : JXG_ERR_HIP;
}
// drop every completed frame (their D2H copies finish first)
static void pipe_drop_done(Pipe& p) {
  for (auto& d : p.done) {
    (void)pipe_done_wait(p, d);
    jxg_buffer_free(&d.buf);
  }
  p.done.clear();
}
static bool pipe_busy(const Ctx* c) {
  return c->pipe && (!c->pipe->inflight.empty() || !c->pipe->done.empty() ||
                     !c->pipe->ready.empty());
}

static jxg_status ensure_lanes(Ctx* c, uint32_t extra) {
  while (c->lanes.size() < extra) {
    Ctx* l = nullptr;
    const jxg_status st = ctx_new_lane(c->params, &l);
    if (st) return st;
    c->lanes.emplace_back(l);
  }
  return JXG_OK;
}
// slot i of lane L (0: the lane itself; others share its stream)
static jxg_status ensure_slots(Ctx* L, uint32_t k) {
  while (L->slots.size() + 1 < k) {
    Ctx* q = new (std::nothrow) Ctx();
    if (!q) return JXG_ERR_OOM;
    q->params = L->params;
    q->owned_lane = true;
    q->shared_stream = true;
    q->stream = L->stream;
    L->slots.emplace_back(q);
    for (auto& e : q->ev)
      if (make_event(&e, 0) != hipSuccess) return JXG_ERR_HIP;
  }
  return JXG_OK;
}
static Ctx* lane_slot(Ctx* L, uint32_t i) { return i == 0 ? L : L->slots[i - 1].get(); }

// drop every frame in flight (after an error): wait for the helpers and the
// lanes' streams
static void pipe_abort(Ctx* c) {
  Pipe& p = *c->pipe;
  p.open.reset();
  for (auto& fr : p.inflight) (void)pipe_join_codes(*fr);
  for (auto& fr : p.inflight) (void)hipStreamSynchronize(fr->lane->stream);
  for (auto& fr : p.ready) (void)hipStreamSynchronize(fr->lane->stream);
  for (auto& fr : p.inflight)  // codestreams of frames whose assembly had started
    if (fr->J.host_out) {
      out_release(fr->J.host_out);
      fr->J.host_out = nullptr;
    }
  p.inflight.clear();
  p.ready.clear();
}

// A rank's sections of a frame (codes built, emission launched) -> payload
// head (host, lane->payload_head) + body (device, lane->out); the stream is
// synchronised.
// payload: "JXGS" | version | rank (| loop-filter code << 16) | world | xsize | ysize | nsections |
//          nsections x (TOC index, bytes) [| version 2: the rank's HF preset]
//          | section bytes back to back
// (sync false: the body may still be in flight on the context's stream; the
// streaming path enqueues its D2H behind it -- shard_write_host -- so the head
// goes out one GPU round trip earlier)
static jxg_status shard_finish(Ctx* c, Job& J, size_t* payload_bytes, bool sync = true) {
  hipStream_t s = c->stream;
  jxg_status st0 = wait_emission(c, J);  // the emission's bit counts on the host
  if (st0) return st0;
  std::vector<uint32_t> ids, sizes;
  size_t nbytes = 0;
  jxg_status st;
  if ((st = stage_concat(c, J, false, &ids, &sizes, nullptr, &nbytes))) return st;
  std::vector<uint32_t>& hw = c->payload_head;
  hw.assign(7 + 2 * ids.size(), 0);
  hw[0] = kPayloadMagic;
  hw[1] = J.presets ? 2 : 1;
  // the rank, the frame's loop-filter code, the 128 / 256 px kinds the rank's
  // groups use (their quant tables go into HfGlobal, effort >= 8)
  hw[2] = J.plan.rank | J.lf << 16 | (J.big ? big_mask(c->h_bigcount.p) : 0u) << 24;
  hw[3] = J.plan.world;
  hw[4] = J.w;
  hw[5] = J.h;
  hw[6] = (uint32_t)ids.size();
  for (size_t i = 0; i < ids.size(); i++) {
    hw[7 + 2 * i] = ids[i];
    hw[8 + 2 * i] = sizes[i];
  }
  if (J.presets) {
    // version 2: the rank's HF preset -- [B][nhist][context map, bytes packed
    // in words][clustered counts nhist x kAlpha], B = words after B
    const uint32_t nh = J.nhist_ans, cw = (kAcCtx + 3) / 4;
    hw.push_back(1 + cw + nh * kAlpha);
    hw.push_back(nh);
    const size_t o = hw.size();
    hw.resize(o + cw, 0);
    std::memcpy(hw.data() + o, J.pre_ctxmap.data(), kAcCtx);
    hw.insert(hw.end(), J.pre_counts.begin(), J.pre_counts.end());
  }
  c->payload_body = nbytes;
  *payload_bytes = hw.size() * 4 + nbytes;
  if (sync) JXG_HIP(hipStreamSynchronize(s));
  return JXG_OK;
}

// a shard frame's stats (its lane's) once its sections are emitted
static void shard_frame_stats(PipeFrame& fr, size_t bytes) {
  jxg_stats& S = fr.lane->stats;
  S = jxg_stats{};
  S.xsize = fr.J.w;
  S.ysize = fr.J.h;
  S.num_groups = fr.J.f.ngroups;
  S.num_lf_groups = fr.J.f.nlf;
  S.bytes = bytes;
  S.ms_front_kernel = elapsed(fr.lane->ev[9], fr.lane->ev[5]);
  S.ms_aq = elapsed(fr.lane->ev[0], fr.lane->ev[9]);
  S.ms_front = elapsed(fr.lane->ev[0], fr.lane->ev[1]);
  S.ms_host_codes = fr.J.ms_codes;
  S.ms_host_call = ms_since(fr.t0);
}

// the open batch -> launched: every frame's plan and buffers, the batched
// front end / merge / statistics kernels, the frames' codes queued on the
// helper threads (inline without threads: codes, then the emission)
static jxg_status pipe_launch_open(Ctx* c) {
  Pipe& p = *c->pipe;
  std::shared_ptr<PipeBatch> B = std::move(p.open);
  p.open.reset();
  if (!B || B->frames.empty()) return JXG_OK;
  const uint32_t k = (uint32_t)B->frames.size();
  std::vector<Ctx*> cs;
  std::vector<Job*> js;
  for (PipeFrame* fr : B->frames) {
    const jxg_status st = enc_prepare(fr->lane, fr->J, fr->src, fr->w, fr->h, fr->stride,
                                      fr->rank, fr->world);
    if (st) return st;
    cs.push_back(fr->lane);
    js.push_back(&fr->J);
  }
  jxg_status st = launch_stats(cs.data(), js.data(), k);
  if (st) return st;
  B->left.store((int)k);
  for (PipeFrame* fr : B->frames) fr->phase = 1;
  try {
    if (!p.helpers) p.helpers.reset(new Helpers(c->params.device, kPipeHelpers));
    for (PipeFrame* fr : B->frames) fr->codes = p.helpers->run([fr]() { return pipe_codes(fr); });
  } catch (...) {  // no thread: the codes (and the emission) on this one
    for (PipeFrame* fr : B->frames) {
      if (fr->codes.valid()) continue;
      if ((st = pipe_codes(fr))) return st;
      fr->phase = 2;
    }
  }
  return JXG_OK;
}

// oldest frame in flight -> done (a whole frame: assembled, codestream on
// the host) or ready (a shard: sections emitted, payload head built); on an
// error the caller aborts the pipe
static jxg_status pipe_complete_oldest(Ctx* c) {
  Pipe& p = *c->pipe;
  jxg_status st = JXG_OK;
  if (p.inflight.front()->phase == 0 && (st = pipe_launch_open(c))) return st;
  PipeFrame& fr = *p.inflight.front();
  // every frame of its batch: the last codes launch the batch's emission
  // (the batch's frames are the oldest in flight, consecutive)
  for (size_t i = 0; i < p.inflight.size() && p.inflight[i]->batch == fr.batch; i++) {
    const jxg_status e = pipe_join_codes(*p.inflight[i]);
    if (!st) st = e;
  }
  if (fr.shard) {
    size_t bytes = 0;
    if (!st) st = shard_finish(fr.lane, fr.J, &bytes, false);
    if (st) return st;
    shard_frame_stats(fr, bytes);
    p.ready.push_back(std::move(p.inflight.front()));
    p.inflight.erase(p.inflight.begin());
    return JXG_OK;
  }
  PipeDone d{{nullptr, 0}, {}, nullptr};
  if (fr.lane->params.flags & JXG_FLAG_KEEP_MAPS) {
    if (!st) st = enc_finish(fr.lane, fr.J, false, &d.buf, fr.t0);
  } else if (!st) {
    // deferred finish: layout, concat and the codestream's D2H are enqueued on
    // the lane's stream and the lane is free at once (the next frame's work
    // queues behind them); only jxg_receive waits for the D2H.  Saves this
    // thread one GPU round trip per frame.
    if (p.evfree.empty()) {
      hipEvent_t e = nullptr;
      if (make_event(&e, hipEventDisableTiming) != hipSuccess) return JXG_ERR_HIP;
      p.evfree.push_back(e);
    }
    st = enc_finish_start(fr.lane, fr.J, false);
    if (!st && hipEventRecord(p.evfree.back(), fr.lane->stream) != hipSuccess) st = JXG_ERR_HIP;
    if (st) {
      (void)hipStreamSynchronize(fr.lane->stream);
      out_release(fr.J.host_out);
      fr.J.host_out = nullptr;
      return st;
    }
    d.ev = p.evfree.back();
    p.evfree.pop_back();
    d.buf = jxg_buffer{fr.J.host_out, fr.J.out_bytes};
    fr.J.host_out = nullptr;
    enc_stats(fr.lane, fr.J, d.buf.size, fr.J.ms_finish_layout, false, nullptr, fr.t0);
  }
  if (st) return st;
  d.stats = fr.lane->stats;
  p.done.push_back(d);
  p.inflight.erase(p.inflight.begin());
  return JXG_OK;
}

static Ctx* pipe_lane(Ctx* c, uint32_t li) { return li == 0 ? c : c->lanes[li - 1].get(); }

// submit one frame (world == 1) or this rank's shard of one frame
static jxg_status pipe_submit(Ctx* c, const uint8_t* src, bool on_device, uint32_t w,
                              uint32_t h, size_t stride, uint32_t rank = 0, uint32_t world = 1,
                              bool shard = false) {
  if (!c->pipe) c->pipe.reset(new (std::nothrow) Pipe());
  if (!c->pipe) return JXG_ERR_OOM;
  Pipe& p = *c->pipe;
  const int mode = shard ? 2 : 1;
  if (pipe_busy(c) && p.mode != mode) return JXG_ERR_INVALID_ARG;  // one kind at a time
  const Frame f0 = make_frame(w, h, c->params.distance);
  uint32_t ngroups = f0.ngroups, ntiles = f0.tiles_x * f0.tiles_y;
  if (shard) {
    if (world < 1 || rank >= world || f0.ngroups < world || (world > 1 && f0.ngroups < 2))
      return JXG_ERR_INVALID_ARG;
    // no collective inside the pipeline: no record exchange, and with more
    // than one rank one HF preset per rank (ANS)
    const Plan P = make_plan(f0, rank, world);
    if (!P.x.send.empty() || !P.x.recv.empty() ||
        (world > 1 && !(c->params.flags & JXG_FLAG_ANS)))
      return JXG_ERR_UNSUPPORTED;
    ngroups = P.ng();
    if (!P.tiles.empty()) ntiles = (uint32_t)P.tiles.size();
  }
  const PipeShape shape = pipe_shape(ngroups, ntiles, c->lane_cap);
  jxg_status st = ensure_lanes(c, shape.lanes - 1);
  if (st) return st;
  const Clock::time_point t0 = Clock::now();
  // a shard frame holds its slot until its sections are written: the caller
  // must take one first (jxg_shard_next_head / jxg_shard_write_next)
  if (shard && p.inflight.size() + p.ready.size() >= shape.pending()) return JXG_ERR_INVALID_ARG;
  p.mode = mode;
  p.depth = shape.frames();
  auto fail = [&](jxg_status e) {
    pipe_abort(c);
    return e;
  };
  // an open batch of another size / plan, or a full one, goes out first
  if (p.open && (p.open->w != w || p.open->h != h || p.open->rank != rank ||
                 p.open->world != world || p.open->frames.size() >= shape.batch))
    if ((st = pipe_launch_open(c))) return fail(st);
  if (!p.open) {
    // a free lane (no frame in flight or ready on it): complete the oldest
    // frames until one is
    Ctx* L = nullptr;
    for (;;) {
      for (uint32_t li = 0; li < shape.lanes && !L; li++) {
        Ctx* cand = pipe_lane(c, li);
        bool used = false;
        for (auto& q : p.inflight) used = used || q->owner == cand;
        for (auto& q : p.ready) used = used || q->owner == cand;
        if (!used) L = cand;
      }
      if (L) break;
      if (p.inflight.empty()) return shard ? JXG_ERR_INVALID_ARG : fail(JXG_ERR_INTERNAL);
      if ((st = pipe_complete_oldest(c))) return fail(st);
    }
    if ((st = ensure_slots(L, shape.batch))) return fail(st);
    p.open = std::make_shared<PipeBatch>();
    PipeBatch& B = *p.open;
    B.owner = L;
    B.w = w;
    B.h = h;
    B.rank = rank;
    B.world = world;
    B.shard = shard;
  }
  PipeBatch& B = *p.open;
  std::unique_ptr<PipeFrame> fr(new (std::nothrow) PipeFrame());
  if (!fr) return fail(JXG_ERR_OOM);
  Ctx* S = lane_slot(B.owner, (uint32_t)B.frames.size());
  fr->lane = S;
  fr->owner = B.owner;
  fr->batch = p.open;
  fr->t0 = t0;
  fr->shard = shard;
  fr->w = w;
  fr->h = h;
  fr->stride = stride;
  fr->rank = rank;
  fr->world = world;
  if (!on_device) {
    // the slot's previous frame has completed, so its staging is free
    const size_t bytes = stride * (h - 1) + (size_t)w * 3;
    if (S->h_stage.ensure(bytes) != hipSuccess || S->rgb.ensure(bytes) != hipSuccess)
      return fail(JXG_ERR_OOM);
    std::memcpy(S->h_stage.p, src, bytes);
    if (hipMemcpyAsync(S->rgb.p, S->h_stage.p, bytes, hipMemcpyHostToDevice, S->stream) !=
        hipSuccess)
      return fail(JXG_ERR_HIP);
    src = S->rgb.p;
  } else if ((st = order_input(c, S))) {
    return fail(st);
  }
  fr->src = src;
  B.frames.push_back(fr.get());
  p.inflight.push_back(std::move(fr));
  p.submitted++;
  if (B.frames.size() >= shape.batch && (st = pipe_launch_open(c))) return fail(st);
  // frames one per lane: this thread waits for the codes of frame j - lag
  // (their emission launched), which paces the launches by the codes and
  // rANS chains instead of filling every lane with transform work at once
  // (8K: +4 %, profiles/r04j); batched small frames are paced by their lanes
  if (shape.batch == 1) {
    const size_t lag = ngroups >= 256 ? 1 : 3;
    if (p.inflight.size() > lag) {
      PipeFrame& fj = *p.inflight[p.inflight.size() - 1 - lag];
      if (fj.phase >= 1 && (st = pipe_join_codes(fj))) return fail(st);
    }
  }
  return JXG_OK;
}

static jxg_status pipe_receive(Ctx* c, jxg_buffer* out) {
  if (!c->pipe || c->pipe->mode != 1) return JXG_ERR_INVALID_ARG;
  Pipe& p = *c->pipe;
  if (p.done.empty()) {
    if (p.inflight.empty()) return JXG_ERR_INVALID_ARG;
    const jxg_status st = pipe_complete_oldest(c);
    if (st) {
      pipe_abort(c);
      return st;
    }
  }
  const jxg_status st = pipe_done_wait(p, p.done.front());
  if (st) return st;
  *out = p.done.front().buf;
  c->stats = p.done.front().stats;
  p.done.erase(p.done.begin());
  return JXG_OK;
}

// streaming shards: the oldest pending shard frame, completed if needed
static jxg_status pipe_shard_oldest(Ctx* c, PipeFrame** fr) {
  if (!c->pipe || c->pipe->mode != 2) return JXG_ERR_INVALID_ARG;
  Pipe& p = *c->pipe;
  if (p.ready.empty()) {
    if (p.inflight.empty()) return JXG_ERR_INVALID_ARG;
    const jxg_status st = pipe_complete_oldest(c);
    if (st) {
      pipe_abort(c);
      return st;
    }
  }
  *fr = p.ready.front().get();
  return JXG_OK;
}

// ---------------------------------------------------------------------------
// sharded encode, one frame at a time (jxg_shard_begin / jxg_shard_end), with
// the caller's collectives in between
// ---------------------------------------------------------------------------
static jxg_status shard_begin(Ctx* c, const uint8_t* d_rgb, uint32_t w, uint32_t h,
                              size_t stride, uint32_t rank, uint32_t world, uint32_t* d_hist,
                              uint8_t* d_xbuf) {
  hipStream_t s = c->stream;
  c->job = std::make_unique<Job>();
  Job& J = *c->job;
  J.f = make_frame(w, h, c->params.distance);
  if (world < 1 || rank >= world || J.f.ngroups < world || J.f.ngroups < 2)
    return JXG_ERR_INVALID_ARG;
  J.plan = make_plan(J.f, rank, world);
  J.w = w;
  J.h = h;
  J.stride = stride;
  J.d_rgb = d_rgb;
  jxg_status st = stage_alloc(c, J);
  if (st) return st;
  // ANS: one HF preset per rank (its own histograms; the caller need not
  // all-reduce d_hist).  Prefix codes keep one preset from the summed
  // histogram (N x 132 clusters would not fit one context map).
  J.presets = J.ans && world > 1;
  if ((st = order_input(c, c))) return st;
  if ((st = build_front(c, J))) return st;
  Job* jp = &J;
  if ((st = launch_transform(&c, &jp, 1))) return st;
  JXG_HIP(hipMemcpyAsync(d_hist, c->hist_ac.p, kMaxClusters * kAlpha * 4, hipMemcpyDeviceToDevice, s));
  JXG_HIP(hipMemcpyAsync(d_hist + (size_t)kMaxClusters * kAlpha, c->bigcount.p, 16,
                         hipMemcpyDeviceToDevice, s));
  // the send list (then the receive list) of the record exchange
  const Exchange& X = J.plan.x;
  JXG_HIP(c->xlist.ensure(X.send.size() + X.recv.size() + 1));
  if (!X.send.empty())
    JXG_HIP(hipMemcpyAsync(c->xlist.p, X.send.data(), X.send.size() * 4, hipMemcpyHostToDevice, s));
  if (!X.recv.empty())
    JXG_HIP(hipMemcpyAsync(c->xlist.p + X.send.size(), X.recv.data(), X.recv.size() * 4,
                           hipMemcpyHostToDevice, s));
  PackArgs pa{c->acs.p, c->qf.p, c->dc.p, J.f.bxs, J.f.bys, J.f.gxs, c->cmap.p, J.f.tiles_x,
              J.f.tiles_y, d_xbuf, c->xlist.p, (uint32_t)X.send.size()};
  launch_pack(pa, s);
  JXG_HIP(hipGetLastError());
  JXG_HIP(hipEventRecord(c->ev[1], s));
  JXG_HIP(hipStreamSynchronize(s));
  return JXG_OK;
}

static jxg_status shard_end(Ctx* c, const uint32_t* d_hist, const uint8_t* d_xbuf,
                            size_t* payload_bytes) {
  if (!c->job) return JXG_ERR_INVALID_ARG;
  const Clock::time_point t_call = Clock::now();
  Job& J = *c->job;
  hipStream_t s = c->stream;
  const Exchange& X = J.plan.x;
  PackArgs pa{c->acs.p, c->qf.p, c->dc.p, J.f.bxs, J.f.bys, J.f.gxs, c->cmap.p, J.f.tiles_x,
              J.f.tiles_y, const_cast<uint8_t*>(d_xbuf), c->xlist.p + X.send.size(),
              (uint32_t)X.recv.size()};
  launch_unpack(pa, s);
  JXG_HIP(hipGetLastError());
  jxg_status st;
  if ((st = stage_download_ac(c, J, d_hist))) return st;
  Job* jp = &J;
  if ((st = launch_lf_stats(&c, &jp, 1))) return st;
  if ((st = stage_codes(c, J))) return st;
  if ((st = stage_emit(c, J))) return st;
  if ((st = shard_finish(c, J, payload_bytes))) return st;
  c->stats = jxg_stats{};
  c->stats.xsize = J.w;
  c->stats.ysize = J.h;
  c->stats.num_groups = J.f.ngroups;
  c->stats.num_lf_groups = J.f.nlf;
  c->stats.bytes = *payload_bytes;
  c->stats.ms_front = elapsed(c->ev[0], c->ev[1]);
  c->stats.ms_front_kernel = elapsed(c->ev[9], c->ev[5]);
  c->stats.ms_aq = elapsed(c->ev[0], c->ev[9]);
  c->stats.ms_total = elapsed(c->ev[0], c->ev[4]);
  c->stats.ms_host_call = ms_since(t_call);
  c->job.reset();
  return JXG_OK;
}

// copy the payload of the last jxg_shard_end to dst (device or host memory)
static jxg_status shard_payload(Ctx* c, void* dst, bool on_device) {
  hipStream_t s = c->stream;
  const size_t head = c->payload_head.size() * 4;
  if (!head) return JXG_ERR_INVALID_ARG;
  uint8_t* d = static_cast<uint8_t*>(dst);
  if (on_device) {
    JXG_HIP(hipMemcpyAsync(d, c->payload_head.data(), head, hipMemcpyHostToDevice, s));
    JXG_HIP(hipMemcpyAsync(d + head, c->out.p, c->payload_body, hipMemcpyDeviceToDevice, s));
  } else {
    std::memcpy(d, c->payload_head.data(), head);
    JXG_HIP(hipMemcpyAsync(d + head, c->out.p, c->payload_body, hipMemcpyDeviceToHost, s));
  }
  JXG_HIP(hipStreamSynchronize(s));
  return JXG_OK;
}

// device-resident payloads (payload i at d_base + offsets[i]) -> codestream in
// host memory: headers + TOC on the host, every section moved by the concat
// kernel, one D2H of the result
static jxg_status shard_assemble_device(Ctx* c, const uint8_t* d_base, const size_t* offsets,
                                        const size_t* psizes, uint32_t n, jxg_buffer* out) {
  hipStream_t s = c->stream;
  // payload heads to the host (a few KB each)
  std::vector<std::vector<uint32_t>> heads(n);
  std::vector<size_t> ps(psizes, psizes + n);
  for (uint32_t i = 0; i < n; i++) {
    std::vector<uint32_t>& hw = heads[i];
    if (psizes[i] < 28) return JXG_ERR_INVALID_ARG;
    hw.resize(7);
    JXG_HIP(hipMemcpy(hw.data(), d_base + offsets[i], 28, hipMemcpyDeviceToHost));
    const size_t base = 7 + 2 * (size_t)hw[6];
    if (hw[1] == 2) {  // version 2: read up to the preset block's length
      if (psizes[i] < (base + 1) * 4) return JXG_ERR_INVALID_ARG;
      hw.resize(base + 1);
      JXG_HIP(hipMemcpy(hw.data(), d_base + offsets[i], (base + 1) * 4, hipMemcpyDeviceToHost));
    }
    const size_t words = head_words(hw.data(), hw.size());
    if (!words || psizes[i] < words * 4) return JXG_ERR_INVALID_ARG;
    hw.resize(words);
    JXG_HIP(hipMemcpy(hw.data(), d_base + offsets[i], words * 4, hipMemcpyDeviceToHost));
  }
  uint32_t w = 0, h = 0;
  std::vector<SectionRef> secs;
  std::vector<uint8_t> hf;
  uint32_t lf = 0;
  jxg_status st = parse_payload_heads(heads, ps, &w, &h, secs, hf, &lf);
  if (st) return st;
  std::vector<uint32_t> sizes(secs.size());
  for (size_t i = 0; i < secs.size(); i++) sizes[i] = secs[i].size;
  BitWriter head;
  write_headers(head, w, h, lf);
  write_toc(head, sizes);
  std::vector<uint32_t> chunk_words = head.words32();
  // a generated HfGlobal (per-rank presets) follows the headers in the chunk arena
  const uint64_t hf_src = (uint64_t)chunk_words.size() * 32;
  for (size_t i = 0; i < hf.size(); i += 4) {
    uint32_t wv = 0;
    for (size_t b = 0; b < 4 && i + b < hf.size(); b++) wv |= (uint32_t)hf[i + b] << (8 * b);
    chunk_words.push_back(wv);
  }
  chunk_words.push_back(0);
  std::vector<ConcatPiece> cps;
  uint64_t dst = 0, max_words = 0;
  cps.push_back({0, 0, head.bits(), 1, 0});
  max_words = (head.bits() + 31) / 32;
  dst = (head.bits() + 7) & ~7ull;
  // payloads are read as one 32-bit-word arena starting at d_base
  for (const SectionRef& r : secs) {
    if (r.size) {
      if (r.payload == n)
        cps.push_back({hf_src, dst, (uint64_t)r.size * 8, 1, 0});
      else
        cps.push_back({(offsets[r.payload] + r.off) * 8, dst, (uint64_t)r.size * 8, 0, 0});
      max_words = std::max<uint64_t>(max_words, ((uint64_t)r.size * 8 + 31) / 32);
    }
    dst += (uint64_t)r.size * 8;
  }
  const size_t nbytes = (size_t)(dst / 8);
  const size_t out_words = (nbytes + 3) / 4 + 1;
  JXG_HIP(c->chunks.ensure(chunk_words.size()));
  JXG_HIP(c->pieces.ensure(cps.size()));
  JXG_HIP(c->out.ensure(out_words));
  uint8_t* ho = out_alloc(out_words * 4);
  if (!ho) return JXG_ERR_OOM;
  JXG_HIP(hipMemcpyAsync(c->chunks.p, chunk_words.data(), chunk_words.size() * 4, hipMemcpyHostToDevice, s));
  JXG_HIP(hipMemcpyAsync(c->pieces.p, cps.data(), cps.size() * sizeof(ConcatPiece), hipMemcpyHostToDevice, s));
  // arena 0 = the payload base (word aligned: offsets are multiples of 4)
  launch_concat(c->pieces.p, (uint32_t)cps.size(), out_words,
                reinterpret_cast<const uint32_t*>(d_base), c->chunks.p, nullptr, c->out.p, s);
  JXG_HIP(hipGetLastError());
  if (hipMemcpyAsync(ho, c->out.p, out_words * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    out_release(ho);
    return JXG_ERR_HIP;
  }
  out->data = ho;
  out->size = nbytes;
  return JXG_OK;
}

// Distributed host assembly: with every rank's payload head (host), each rank
// writes its own sections straight from its device body into one host buffer
// shared by all ranks (one D2H per contiguous run: its pass groups are one
// run, its LF groups one each); rank 0 also writes headers + TOC.  Same bytes
// as shard_assemble_device, without the payload gather and the serial D2H of
// the whole codestream on rank 0.
// (sync false: the copies are left in flight on the context's stream)
static jxg_status shard_write_host(Ctx* c, const uint32_t* const* heads_in, const size_t* words,
                                   uint32_t n, uint8_t* dst, size_t dst_size, size_t* total,
                                   bool sync = true) {
  if (c->payload_head.size() < 7) return JXG_ERR_INVALID_ARG;
  std::vector<std::vector<uint32_t>> heads(n);
  std::vector<size_t> ps(n);
  for (uint32_t i = 0; i < n; i++) {
    if (!heads_in[i] || words[i] < 7) return JXG_ERR_INVALID_ARG;
    heads[i].assign(heads_in[i], heads_in[i] + words[i]);
    if (head_words(heads[i].data(), words[i]) != words[i]) return JXG_ERR_INVALID_ARG;
    size_t body = 0;
    for (uint32_t k = 0; k < heads[i][6]; k++) body += heads[i][8 + 2 * k];
    ps[i] = words[i] * 4 + body;
  }
  const uint32_t me = c->payload_head[2] & 0xFFFFu;
  if (me >= n || heads[me] != c->payload_head) return JXG_ERR_INVALID_ARG;
  uint32_t w = 0, h = 0;
  std::vector<SectionRef> secs;
  std::vector<uint8_t> hf;
  uint32_t lf = 0;
  // a generated HfGlobal (per-rank presets) is written by rank 0; the others
  // need its size only
  jxg_status st = parse_payload_heads(heads, ps, &w, &h, secs, hf, &lf, me == 0);
  if (st) return st;
  std::vector<uint32_t> sec_size(secs.size());
  for (size_t i = 0; i < secs.size(); i++) sec_size[i] = secs[i].size;
  BitWriter head;
  write_headers(head, w, h, lf);
  write_toc(head, sec_size);
  const std::vector<uint8_t> hb = head.bytes();
  std::vector<uint64_t> out_off(secs.size());
  uint64_t pos = hb.size();
  for (size_t i = 0; i < secs.size(); i++) {
    out_off[i] = pos;
    pos += sec_size[i];
  }
  *total = (size_t)pos;
  if (!dst || pos > dst_size) return JXG_ERR_INVALID_ARG;  // *total tells the size needed
  hipStream_t s = c->stream;
  const std::vector<uint32_t>& hw = c->payload_head;
  // runs of consecutive sections (payload body -> codestream offsets)
  std::vector<ScatterPiece> runs;
  uint64_t body = 0;
  for (uint32_t k = 0; k < hw[6]; k++) {
    const uint32_t id = hw[7 + 2 * k], sz = hw[8 + 2 * k];
    ScatterPiece* r = runs.empty() ? nullptr : &runs.back();
    if (r && r->src + r->len == body && r->dst + r->len == out_off[id])
      r->len += sz;
    else if (sz)
      runs.push_back({body, out_off[id], sz, 0});
    body += sz;
  }
  // one scatter launch through the buffer's device mapping (page-locked with
  // jxg_host_register); D2H copies per run otherwise
  void* dmap = nullptr;
  if (!runs.empty() && runs.size() <= (size_t)kMaxScatterPieces &&
      hipHostGetDevicePointer(&dmap, dst, 0) == hipSuccess && dmap) {
    ScatterArgs sa{};
    sa.src = reinterpret_cast<const uint8_t*>(c->out.p);
    sa.dst = static_cast<uint8_t*>(dmap);
    sa.n = (uint32_t)runs.size();
    uint32_t nwg = 0;
    for (size_t i = 0; i < runs.size(); i++) {
      sa.p[i] = runs[i];
      sa.p[i].wg0 = nwg;
      const uint64_t w0 = runs[i].dst >> 2, w1 = (runs[i].dst + runs[i].len + 3) >> 2;
      nwg += (uint32_t)((w1 - w0 + 1023) / 1024);
    }
    launch_scatter(sa, nwg, s);
    JXG_HIP(hipGetLastError());
  } else {
    (void)hipGetLastError();  // (an unmapped buffer: hipHostGetDevicePointer failed)
    for (const ScatterPiece& r : runs)
      JXG_HIP(hipMemcpyAsync(dst + r.dst, reinterpret_cast<const uint8_t*>(c->out.p) + r.src, r.len,
                             hipMemcpyDeviceToHost, s));
  }
  if (me == 0) {
    std::memcpy(dst, hb.data(), hb.size());
    for (size_t i = 0; i < secs.size(); i++)  // a generated HfGlobal (per-rank presets)
      if (secs[i].payload == n && secs[i].size) std::memcpy(dst + out_off[i], hf.data(), hf.size());
  }
  if (sync) JXG_HIP(hipStreamSynchronize(s));
  return JXG_OK;
}

// host only: payloads of every rank -> codestream (same layout as
// shard_assemble_device; no device needed)
static jxg_status shard_assemble(const uint8_t* const* payloads, const size_t* sizes, uint32_t n,
                                 jxg_buffer* out) {
  if (!payloads || !sizes || !out || n == 0) return JXG_ERR_INVALID_ARG;
  std::vector<std::vector<uint32_t>> heads(n);
  std::vector<size_t> ps(sizes, sizes + n);
  for (uint32_t i = 0; i < n; i++) {
    if (!payloads[i]) return JXG_ERR_INVALID_ARG;
    heads[i] = read_head(payloads[i], sizes[i]);
    if (heads[i].empty()) return JXG_ERR_INVALID_ARG;
  }
  uint32_t w = 0, h = 0;
  std::vector<SectionRef> secs;
  std::vector<uint8_t> hf;
  uint32_t lf = 0;
  jxg_status st = parse_payload_heads(heads, ps, &w, &h, secs, hf, &lf);
  if (st) return st;
  std::vector<uint32_t> sec_size(secs.size());
  size_t total = 0;
  for (size_t i = 0; i < secs.size(); i++) {
    sec_size[i] = secs[i].size;
    total += secs[i].size;
  }
  BitWriter head;
  write_headers(head, w, h, lf);
  write_toc(head, sec_size);
  const std::vector<uint8_t> hb = head.bytes();
  uint8_t* o = out_alloc_heap(hb.size() + total);
  if (!o) return JXG_ERR_OOM;
  std::memcpy(o, hb.data(), hb.size());
  size_t pos = hb.size();
  for (const SectionRef& r : secs) {
    std::memcpy(o + pos, r.payload == n ? hf.data() : payloads[r.payload] + r.off, r.size);
    pos += r.size;
  }
  out->data = o;
  out->size = pos;
  return JXG_OK;
}

}  // namespace jxg

using namespace jxg;

extern "C" {

const char* jxg_status_str(jxg_status s) {
  switch (s) {
    case JXG_OK: return "ok";
    case JXG_ERR_INVALID_ARG: return "invalid argument";
    case JXG_ERR_NO_DEVICE: return "no HIP device";
    case JXG_ERR_HIP: return "HIP runtime error";
    case JXG_ERR_OOM: return "out of memory";
    case JXG_ERR_UNSUPPORTED: return "unsupported";
    default: return "internal error";
  }
}


jxg_status jxg_create(const jxg_params* params, jxg_ctx** out) {
  if (!params || !out) return JXG_ERR_INVALID_ARG;
  *out = nullptr;
  if (!(params->distance > 0.0f) || params->distance > 25.0f) return JXG_ERR_INVALID_ARG;
  if (params->effort < 1 || params->effort > 10) return JXG_ERR_INVALID_ARG;
  if (params->proposals & ~3u) return JXG_ERR_INVALID_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return JXG_ERR_NO_DEVICE;
  if (params->device < 0 || params->device >= ndev) return JXG_ERR_INVALID_ARG;
  if (hipSetDevice(params->device) != hipSuccess) return JXG_ERR_HIP;
  Ctx* c = nullptr;
  const jxg_status st = ctx_new_lane(*params, &c);
  if (st) return st;
  c->owned_lane = false;
  g_live_ctx++;
  *out = reinterpret_cast<jxg_ctx*>(c);
  return JXG_OK;
}

void jxg_destroy(jxg_ctx* ctx) {
  if (!ctx) return;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c->pipe) {  // frames still in the pipeline (their lanes are released below)
    pipe_abort(c);
    pipe_drop_done(*c->pipe);
    c->pipe.reset();
  }
  (void)hipSetDevice(c->params.device);
  // written shard frames' section copies may still read a slot's buffers
  (void)hipStreamSynchronize(c->stream);
  if (c->stream2) (void)hipStreamSynchronize(c->stream2);
  c->lanes.clear();  // pipeline lanes (jxg_destroy each)
  c->slots.clear();  // their extra slots (sharing this context's stream)
  if (!c->owned_lane) g_live_ctx--;
#ifdef JXG_MERGE_PROFILE
  dump_merge_profile();
#endif
#ifdef JXG_FRONT_PROFILE
  dump_front_profile();
  dump_hist_profile();
#endif
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->ev_in) (void)hipEventDestroy(c->ev_in);
  if (c->ev_write) (void)hipEventDestroy(c->ev_write);
  if (c->stream && !c->shared_stream) (void)hipStreamDestroy(c->stream);
  if (c->stream2) (void)hipStreamDestroy(c->stream2);
  delete c;
}

jxg_status jxg_encode_rgb8_device(jxg_ctx* ctx, const void* d_rgb, uint32_t w, uint32_t h,
                                  size_t stride, jxg_buffer* out) {
  if (!ctx || !d_rgb || !out || w == 0 || h == 0 || w > (1u << 18) || h > (1u << 18) ||
      stride < (size_t)w * 3)
    return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  const Clock::time_point t0 = Clock::now();
  out->data = nullptr;
  out->size = 0;
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  const jxg_status st = order_input(c, c);
  if (st) return st;
  return encode_device(c, static_cast<const uint8_t*>(d_rgb), w, h, stride, out, t0);
}

jxg_status jxg_encode_rgb8(jxg_ctx* ctx, const uint8_t* rgb, uint32_t w, uint32_t h, size_t stride,
                           jxg_buffer* out) {
  if (!ctx || !rgb || !out || w == 0 || h == 0 || w > (1u << 18) || h > (1u << 18) ||
      stride < (size_t)w * 3)
    return JXG_ERR_INVALID_ARG;
  const Clock::time_point t0 = Clock::now();
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;  // c->rgb may be an in-flight lane's input
  const size_t bytes = stride * (h - 1) + (size_t)w * 3;
  if (c->rgb.ensure(bytes) != hipSuccess) return JXG_ERR_OOM;
  if (hipMemcpyAsync(c->rgb.p, rgb, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return JXG_ERR_HIP;
  out->data = nullptr;
  out->size = 0;
  return encode_device(c, c->rgb.p, w, h, stride, out, t0);
}

// Batched encode (BASELINE config 3: 64 x 1080p) through the streaming
// pipeline (pipe_submit / pipe_receive): every frame is
// submitted in order and the codestreams already complete are collected after
// each submit, so the frames' transform kernels, rANS chains, host-side code
// construction (helper threads) and pinned H2D copies overlap over the
// pipeline's lanes.  Outputs are in frame order; the bytes of every frame equal
// jxg_encode_rgb8's.  The context must have no streamed frames pending.
static jxg_status batch_encode(Ctx* c, const uint8_t* const* frames, bool on_device, uint32_t n,
                               uint32_t w, uint32_t h, size_t stride, jxg_buffer* outs) {
  for (uint32_t i = 0; i < n; i++) outs[i] = jxg_buffer{nullptr, 0};
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;  // would interleave with the caller's stream
  uint32_t got = 0;
  jxg_status st = JXG_OK;
  for (uint32_t i = 0; i < n && !st; i++) {
    st = pipe_submit(c, frames[i], on_device, w, h, stride);
    // take completed frames whose codestream copy has landed (or when more
    // than two are waiting), without waiting on the newest one's
    while (!st && !c->pipe->done.empty() &&
           (c->pipe->done.size() > 2 || !c->pipe->done.front().ev ||
            hipEventQuery(c->pipe->done.front().ev) == hipSuccess))
      st = pipe_receive(c, &outs[got++]);
  }
  while (!st && got < n) st = pipe_receive(c, &outs[got++]);
  if (st) {  // the pipe is aborted by then; drop what it completed, and ours
    if (c->pipe) pipe_drop_done(*c->pipe);
    for (uint32_t i = 0; i < n; i++) jxg_buffer_free(&outs[i]);
  }
  return st;
}

jxg_status jxg_encode_batch_rgb8(jxg_ctx* ctx, const uint8_t* const* rgbs, uint32_t n, uint32_t w,
                                 uint32_t h, size_t stride, jxg_buffer* outs) {
  if (!ctx || !rgbs || !outs || w == 0 || h == 0 || w > (1u << 18) || h > (1u << 18) ||
      stride < (size_t)w * 3)
    return JXG_ERR_INVALID_ARG;
  for (uint32_t i = 0; i < n; i++)
    if (!rgbs[i]) return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  return batch_encode(c, rgbs, false, n, w, h, stride, outs);
}

jxg_status jxg_encode_batch_rgb8_device(jxg_ctx* ctx, const void* const* d_rgbs, uint32_t n,
                                        uint32_t w, uint32_t h, size_t stride,
                                        jxg_buffer* outs) {
  if (!ctx || !d_rgbs || !outs || w == 0 || h == 0 || w > (1u << 18) || h > (1u << 18) ||
      stride < (size_t)w * 3)
    return JXG_ERR_INVALID_ARG;
  for (uint32_t i = 0; i < n; i++)
    if (!d_rgbs[i]) return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  return batch_encode(c, reinterpret_cast<const uint8_t* const*>(d_rgbs), true, n, w, h, stride,
                      outs);
}

jxg_status jxg_submit_rgb8_device(jxg_ctx* ctx, const void* d_rgb, uint32_t w, uint32_t h,
                                  size_t stride) {
  if (!ctx || !d_rgb || w == 0 || h == 0 || w > (1u << 18) || h > (1u << 18) ||
      stride < (size_t)w * 3)
    return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  return pipe_submit(c, static_cast<const uint8_t*>(d_rgb), true, w, h, stride);
}

jxg_status jxg_submit_rgb8(jxg_ctx* ctx, const uint8_t* rgb, uint32_t w, uint32_t h, size_t stride) {
  if (!ctx || !rgb || w == 0 || h == 0 || w > (1u << 18) || h > (1u << 18) ||
      stride < (size_t)w * 3)
    return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  return pipe_submit(c, rgb, false, w, h, stride);
}

jxg_status jxg_receive(jxg_ctx* ctx, jxg_buffer* out) {
  if (!ctx || !out) return JXG_ERR_INVALID_ARG;
  out->data = nullptr;
  out->size = 0;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  return pipe_receive(c, out);
}

jxg_status jxg_pending(jxg_ctx* ctx, uint32_t* n) {
  if (!ctx || !n) return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  *n = c->pipe ? (uint32_t)(c->pipe->inflight.size() + c->pipe->done.size() +
                            c->pipe->ready.size())
               : 0u;
  return JXG_OK;
}

jxg_status jxg_get_stats(jxg_ctx* ctx, jxg_stats* stats) {
  if (!ctx || !stats) return JXG_ERR_INVALID_ARG;
  *stats = reinterpret_cast<Ctx*>(ctx)->stats;
  return JXG_OK;
}

void jxg_buffer_free(jxg_buffer* buf) {
  if (!buf) return;
  out_release(buf->data);
  buf->data = nullptr;
  buf->size = 0;
}

jxg_status jxg_shard_sizes(uint32_t xsize, uint32_t ysize, uint32_t world, size_t* hist_words,
                           size_t* slot_bytes) {
  if (!hist_words || !slot_bytes || xsize == 0 || ysize == 0 || world == 0)
    return JXG_ERR_INVALID_ARG;
  const Frame f = make_frame(xsize, ysize, 1.0f);
  *hist_words = (size_t)kMaxClusters * kAlpha + 4;  // + the varblocks per big kind
  // the largest send or receive buffer of any rank
  const Partition part = make_partition(f, world);
  size_t most = 1;
  for (uint32_t r = 0; r < world && world > 1; r++) {
    const Exchange X = make_exchange(f, part, r, world);
    most = std::max(most, std::max(X.send.size(), X.recv.size()));
  }
  *slot_bytes = most * kGroupRecordBytes;
  return JXG_OK;
}

jxg_status jxg_shard_exchange(uint32_t xsize, uint32_t ysize, uint32_t world, uint32_t rank,
                              size_t* send_bytes, size_t* recv_bytes) {
  if (!send_bytes || !recv_bytes || xsize == 0 || ysize == 0 || world == 0 || rank >= world)
    return JXG_ERR_INVALID_ARG;
  const Frame f = make_frame(xsize, ysize, 1.0f);
  const Exchange X = make_exchange(f, make_partition(f, world), rank, world);
  for (uint32_t p = 0; p < world; p++) {
    send_bytes[p] = (size_t)X.nsend[p] * kGroupRecordBytes;
    recv_bytes[p] = (size_t)X.nrecv[p] * kGroupRecordBytes;
  }
  return JXG_OK;
}

jxg_status jxg_shard_begin(jxg_ctx* ctx, const void* d_rgb, uint32_t w, uint32_t h, size_t stride,
                           uint32_t rank, uint32_t world, uint32_t* d_hist, void* d_xbuf) {
  if (!ctx || !d_rgb || !d_hist || !d_xbuf || w == 0 || h == 0 || w > (1u << 18) ||
      h > (1u << 18) || stride < (size_t)w * 3)
    return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  return shard_begin(c, static_cast<const uint8_t*>(d_rgb), w, h, stride, rank, world, d_hist,
                     static_cast<uint8_t*>(d_xbuf));
}

jxg_status jxg_shard_end(jxg_ctx* ctx, const uint32_t* d_hist, const void* d_xbuf,
                         size_t* payload_bytes) {
  if (!ctx || !d_hist || !d_xbuf || !payload_bytes) return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  *payload_bytes = 0;
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  return shard_end(c, d_hist, static_cast<const uint8_t*>(d_xbuf), payload_bytes);
}

jxg_status jxg_shard_payload(jxg_ctx* ctx, void* dst, int dst_on_device) {
  if (!ctx || !dst) return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  return shard_payload(c, dst, dst_on_device != 0);
}

jxg_status jxg_shard_assemble_device(jxg_ctx* ctx, const void* d_payloads, const size_t* offsets,
                                     const size_t* sizes, uint32_t n, jxg_buffer* out) {
  if (!ctx || !d_payloads || !offsets || !sizes || !out || n == 0) return JXG_ERR_INVALID_ARG;
  for (uint32_t i = 0; i < n; i++)
    if (offsets[i] % 4) return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  out->data = nullptr;
  out->size = 0;
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  return shard_assemble_device(c, static_cast<const uint8_t*>(d_payloads), offsets, sizes, n, out);
}

jxg_status jxg_shard_head(jxg_ctx* ctx, uint32_t* dst, size_t* nwords) {
  if (!ctx || !nwords) return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  const size_t n = c->payload_head.size();
  if (n == 0) return JXG_ERR_INVALID_ARG;
  if (dst) {
    if (*nwords < n) return JXG_ERR_INVALID_ARG;
    std::memcpy(dst, c->payload_head.data(), n * 4);
  }
  *nwords = n;
  return JXG_OK;
}

jxg_status jxg_shard_write_host(jxg_ctx* ctx, const uint32_t* const* heads, const size_t* head_words,
                                uint32_t n, void* dst, size_t dst_size, size_t* total) {
  if (!ctx || !heads || !head_words || !total || n == 0) return JXG_ERR_INVALID_ARG;
  *total = 0;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  return shard_write_host(c, heads, head_words, n, static_cast<uint8_t*>(dst), dst_size, total);
}

jxg_status jxg_host_register(void* ptr, size_t size) {
  if (!ptr || size == 0) return JXG_ERR_INVALID_ARG;
  return hipHostRegister(ptr, size, hipHostRegisterDefault) == hipSuccess ? JXG_OK : JXG_ERR_HIP;
}

jxg_status jxg_host_unregister(void* ptr) {
  if (!ptr) return JXG_ERR_INVALID_ARG;
  return hipHostUnregister(ptr) == hipSuccess ? JXG_OK : JXG_ERR_HIP;
}

jxg_status jxg_shard_assemble(const uint8_t* const* payloads, const size_t* sizes, uint32_t n,
                              jxg_buffer* out) {
  if (!out) return JXG_ERR_INVALID_ARG;
  out->data = nullptr;
  out->size = 0;
  return shard_assemble(payloads, sizes, n, out);
}

jxg_status jxg_shard_plan(uint32_t xsize, uint32_t ysize, uint32_t world, uint32_t* group_owner,
                          uint32_t* lf_owner, int* kind) {
  if (xsize == 0 || ysize == 0 || world == 0 || xsize > (1u << 18) || ysize > (1u << 18))
    return JXG_ERR_INVALID_ARG;
  const Frame f = make_frame(xsize, ysize, 1.0f);
  const Partition part = make_partition(f, world);
  if (group_owner) std::copy(part.group.begin(), part.group.end(), group_owner);
  if (lf_owner) std::copy(part.lf.begin(), part.lf.end(), lf_owner);
  if (kind) *kind = part.kind;
  return JXG_OK;
}

jxg_status jxg_set_input_stream(jxg_ctx* ctx, void* stream) {
  if (!ctx) return JXG_ERR_INVALID_ARG;
  reinterpret_cast<Ctx*>(ctx)->in_stream = static_cast<hipStream_t>(stream);
  return JXG_OK;
}

jxg_status jxg_pipeline_depth(jxg_ctx* ctx, uint32_t xsize, uint32_t ysize, uint32_t rank,
                              uint32_t world, uint32_t* depth) {
  if (!ctx || !depth || xsize == 0 || ysize == 0 || world == 0 || rank >= world)
    return JXG_ERR_INVALID_ARG;
  const Ctx* c = reinterpret_cast<Ctx*>(ctx);
  const Frame f = make_frame(xsize, ysize, c->params.distance);
  const Plan P = make_plan(f, rank, world);
  const uint32_t nt = P.tiles.empty() ? f.tiles_x * f.tiles_y : (uint32_t)P.tiles.size();
  *depth = pipe_shape(world > 1 ? P.ng() : f.ngroups, nt, c->lane_cap).pending();
  return JXG_OK;
}

jxg_status jxg_set_pipeline_lanes(jxg_ctx* ctx, uint32_t lanes) {
  if (!ctx || lanes > kPipeMaxLanes) return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  c->lane_cap = lanes;
  return JXG_OK;
}

jxg_status jxg_shard_submit_device(jxg_ctx* ctx, const void* d_rgb, uint32_t w, uint32_t h,
                                   size_t stride, uint32_t rank, uint32_t world) {
  if (!ctx || !d_rgb || w == 0 || h == 0 || w > (1u << 18) || h > (1u << 18) ||
      stride < (size_t)w * 3)
    return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  return pipe_submit(c, static_cast<const uint8_t*>(d_rgb), true, w, h, stride, rank, world, true);
}

jxg_status jxg_shard_next_head(jxg_ctx* ctx, uint32_t* dst, size_t* nwords) {
  if (!ctx || !nwords) return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  PipeFrame* fr = nullptr;
  const jxg_status st = pipe_shard_oldest(c, &fr);
  if (st) return st;
  const std::vector<uint32_t>& hw = fr->lane->payload_head;
  if (dst) {
    if (*nwords < hw.size()) return JXG_ERR_INVALID_ARG;
    std::memcpy(dst, hw.data(), hw.size() * 4);
  }
  *nwords = hw.size();
  c->stats = fr->lane->stats;
  return JXG_OK;
}

jxg_status jxg_shard_write_next(jxg_ctx* ctx, const uint32_t* const* heads, const size_t* head_words,
                                uint32_t n, void* dst, size_t dst_size, size_t* total) {
  if (!ctx || !heads || !head_words || !total || n == 0) return JXG_ERR_INVALID_ARG;
  *total = 0;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  PipeFrame* fr = nullptr;
  jxg_status st = pipe_shard_oldest(c, &fr);
  if (st) return st;
  Ctx* S = fr->lane;
  // the copies are enqueued, not waited for: this call returns once the
  // PREVIOUS frame's copies have landed (jxg_shard_write_flush: the last one's)
  st = shard_write_host(S, heads, head_words, n, static_cast<uint8_t*>(dst), dst_size, total, false);
  if (st) return st;  // (too small a buffer: the frame stays, *total tells the size)
  if (!S->ev_write && make_event(&S->ev_write, hipEventDisableTiming) != hipSuccess)
    return JXG_ERR_HIP;
  Pipe& p = *c->pipe;
  // this slot's event may still be queued for an older write of the slot:
  // wait for that write's copies before its record is replaced, so the
  // promise below never rests on an incidental earlier synchronisation
  for (auto it = p.writes.begin(); it != p.writes.end();) {
    if (*it == S->ev_write) {
      JXG_HIP(hipEventSynchronize(*it));
      it = p.writes.erase(it);
    } else {
      ++it;
    }
  }
  JXG_HIP(hipEventRecord(S->ev_write, S->stream));
  p.ready.erase(p.ready.begin());  // its slot is free again (later work queues behind the copies)
  // the copies of the write JXG_SHARD_WRITE_LAG calls back have landed on return
  // (copy kernels queue behind the other lanes' kernels: waiting for the
  // previous frame's held this thread ~0.27 ms per frame, profiles/r04l)
  p.writes.push_back(S->ev_write);
  while (p.writes.size() > JXG_SHARD_WRITE_LAG) {
    const hipEvent_t e = p.writes.front();
    p.writes.pop_front();
    if (e) JXG_HIP(hipEventSynchronize(e));
  }
  return JXG_OK;
}
jxg_status jxg_shard_write_flush(jxg_ctx* ctx) {
  if (!ctx) return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (c->pipe)
    while (!c->pipe->writes.empty()) {
      const hipEvent_t e = c->pipe->writes.front();
      c->pipe->writes.pop_front();
      if (e) JXG_HIP(hipEventSynchronize(e));
    }
  return JXG_OK;
}

jxg_status jxg_homogeneity_map(jxg_ctx* ctx, const float* xyb, uint32_t xsize, uint32_t ysize,
                               float distance, uint32_t flags, float* r3, uint8_t* type) {
  if (!ctx || !xyb || !r3 || !type || xsize == 0 || ysize == 0 || xsize % 8 || ysize % 8)
    return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  const size_t plane = (size_t)xsize * ysize, nb = plane / 64;
  JXG_HIP(c->xyb.ensure(plane * 3));
  JXG_HIP(c->r3.ensure(nb * 3));
  JXG_HIP(c->type.ensure(nb));
  hipStream_t s = c->stream;
  JXG_HIP(hipMemcpyAsync(c->xyb.p, xyb, plane * 12, hipMemcpyHostToDevice, s));
  HomogArgs a{c->xyb.p, xsize, ysize, xsize, plane, distance,
              (flags & JXG_FLAG_H1_INT_ABS) ? 1 : 0, c->r3.p, c->type.p};
  launch_homog(a, (xsize / 8 + 7) / 8, (ysize / 8 + 7) / 8, s);
  JXG_HIP(hipGetLastError());
  JXG_HIP(hipMemcpyAsync(r3, c->r3.p, nb * 12, hipMemcpyDeviceToHost, s));
  JXG_HIP(hipMemcpyAsync(type, c->type.p, nb, hipMemcpyDeviceToHost, s));
  JXG_HIP(hipStreamSynchronize(s));
  return JXG_OK;
}

// ---- decode-side quality (benchmark-jpegxl image_reader.rs:555-606) ----
// Gaussian window of the SSIM: exp(-(k-5)^2 / 4.5), normalized by the sum taken
// in k order (== oracle/metrics.py gaussian_window, libm exp on both sides)
static void gauss_window(double g[11]) {
  double sum = 0.0;
  for (int k = 0; k < 11; k++) {
    const double d = (double)(k - 5);
    g[k] = std::exp(-(d * d) / (2.0 * 1.5 * 1.5));
    sum += g[k];
  }
  for (int k = 0; k < 11; k++) g[k] /= sum;
}

static jxg_status compare_device(Ctx* c, const uint8_t* d_orig, size_t so, const uint8_t* d_comp,
                                 size_t sc, uint32_t w, uint32_t h, int want_ssim,
                                 jxg_quality* out) {
  hipStream_t s = c->stream;
  if (!c->gauss_ready) {
    std::lock_guard<std::mutex> lock(g_const_mu);
    double g[11];
    gauss_window(g);
    JXG_HIP(set_gauss_table(g, s));
    JXG_HIP(hipGetLastError());
    c->gauss_ready = true;
  }
  const uint32_t np = ssim_partials(w, h);
  const bool ssim = want_ssim && np > 0;
  JXG_HIP(c->q_sse.ensure(1));
  JXG_HIP(c->q_ssim.ensure(1));
  if (ssim) JXG_HIP(c->q_part.ensure(np));
  JXG_HIP(hipMemsetAsync(c->q_sse.p, 0, sizeof(uint64_t), s));
  MetricArgs a{d_orig, d_comp, so, sc, w, h, c->q_sse.p, ssim ? c->q_part.p : nullptr,
               ssim ? c->q_ssim.p : nullptr};
  launch_metrics(a, s);
  JXG_HIP(hipGetLastError());
  uint64_t sse = 0;
  double ssum = 0.0;
  JXG_HIP(hipMemcpyAsync(&sse, c->q_sse.p, sizeof(sse), hipMemcpyDeviceToHost, s));
  if (ssim) JXG_HIP(hipMemcpyAsync(&ssum, c->q_ssim.p, sizeof(ssum), hipMemcpyDeviceToHost, s));
  JXG_HIP(hipStreamSynchronize(s));
  out->sse = sse;
  out->samples = (uint64_t)w * h * 3;
  out->mse = (double)sse / (double)out->samples;
  out->psnr = 10.0 * std::log10((255.0 * 255.0) / out->mse);  // mse 0 -> +inf (as f64 in Rust)
  out->ssim = ssim ? ssum / (3.0 * (double)(w - 10) * (double)(h - 10)) : NAN;
  return JXG_OK;
}

jxg_status jxg_compare_rgb8_device(jxg_ctx* ctx, const void* d_orig, size_t orig_stride,
                                   const void* d_comp, size_t comp_stride, uint32_t xsize,
                                   uint32_t ysize, int want_ssim, jxg_quality* out) {
  if (!ctx || !d_orig || !d_comp || !out || xsize == 0 || ysize == 0 ||
      orig_stride < (size_t)xsize * 3 || comp_stride < (size_t)xsize * 3)
    return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  const jxg_status st = order_input(c, c);
  if (st) return st;
  return compare_device(c, static_cast<const uint8_t*>(d_orig), orig_stride,
                        static_cast<const uint8_t*>(d_comp), comp_stride, xsize, ysize, want_ssim,
                        out);
}

jxg_status jxg_compare_rgb8(jxg_ctx* ctx, const uint8_t* orig, size_t orig_stride,
                            const uint8_t* comp, size_t comp_stride, uint32_t xsize,
                            uint32_t ysize, int want_ssim, jxg_quality* out) {
  if (!ctx || !orig || !comp || !out || xsize == 0 || ysize == 0 ||
      orig_stride < (size_t)xsize * 3 || comp_stride < (size_t)xsize * 3)
    return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  const size_t row = (size_t)xsize * 3, n = row * ysize;
  JXG_HIP(c->q_orig.ensure(n));
  JXG_HIP(c->q_comp.ensure(n));
  hipStream_t s = c->stream;
  JXG_HIP(hipMemcpy2DAsync(c->q_orig.p, row, orig, orig_stride, row, ysize,
                           hipMemcpyHostToDevice, s));
  JXG_HIP(hipMemcpy2DAsync(c->q_comp.p, row, comp, comp_stride, row, ysize,
                           hipMemcpyHostToDevice, s));
  return compare_device(c, c->q_orig.p, row, c->q_comp.p, row, xsize, ysize, want_ssim, out);
}

// one synthetic frame of the caller's size through the one-at-a-time path:
// the context's buffers for that size are allocated and every kernel's code
// object is loaded before the caller's first frame (jxg_cjxl runs it beside
// the PNG decode: a new context's first 8K encode took 35 ms against 12 ms)
jxg_status jxg_warmup(jxg_ctx* ctx, uint32_t xsize, uint32_t ysize) {
  if (!ctx || xsize == 0 || ysize == 0 || xsize > (1u << 18) || ysize > (1u << 18))
    return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  if (pipe_busy(c)) return JXG_ERR_INVALID_ARG;
  const size_t stride = (size_t)xsize * 3;
  if (c->rgb.ensure(stride * ysize) != hipSuccess) return JXG_ERR_OOM;  // jxg_encode_rgb8's upload buffer
  JXG_HIP(launch_synth(c->rgb.p, xsize, ysize, stride, 0x5741524Dull, c->stream));
  jxg_buffer out{nullptr, 0};
  jxg_status st = order_input(c, c);
  if (!st) st = encode_device(c, c->rgb.p, xsize, ysize, stride, &out, Clock::now());
  jxg_buffer_free(&out);
  c->stats = jxg_stats{};
  return st;
}

jxg_status jxg_synth_rgb8_device(jxg_ctx* ctx, void* d_out, uint32_t xsize, uint32_t ysize,
                                 size_t row_stride, uint64_t seed) {
  if (!ctx || !d_out || xsize == 0 || ysize == 0 || row_stride < (size_t)xsize * 3)
    return JXG_ERR_INVALID_ARG;
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (hipSetDevice(c->params.device) != hipSuccess) return JXG_ERR_HIP;
  JXG_HIP(launch_synth(static_cast<uint8_t*>(d_out), xsize, ysize, row_stride, seed, c->stream));
  JXG_HIP(hipStreamSynchronize(c->stream));
  return JXG_OK;
}

}  // extern "C"
