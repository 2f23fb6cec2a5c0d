/*
 * jxg.h -- C ABI of the MI355X-native JPEG XL VarDCT encode path.
 *
 * Drop-in boundary: this library replaces what the benchmark harness reaches
 * through `docker exec ... /libjxl/build/tools/cjxl IN OUT --distance=D
 * --effort=E` (pscoro/JPEG-XL-Lossy-Image-Compression-Thesis,
 * benchmark-jpegxl/src/docker_manager.rs:100-137 DockerManager::execute_cjxl,
 * called from benchmark-jpegxl/src/benchmark.rs:654-677).  The encoder
 * internals it re-implements are libjxl's VarDCT heuristics with the thesis
 * hooks of proposals/combined.diff (HomogeneityPartition :213-235 hooked into
 * FindBest8x8Transform :270-274; EstimateEntropy factor :247-253).
 *
 * Conventions: status 0 = OK, negative on error (never aborts); one context
 * per host thread; device memory is owned by the context; output buffers are
 * allocated by the library and released with jxg_buffer_free.
 *
 * Device inputs (jxg_encode_rgb8_device, jxg_submit_rgb8_device,
 * jxg_shard_submit_device, jxg_shard_begin, jxg_compare_rgb8_device) are
 * read on the library's own HIP streams.  Either the caller's writes to them
 * are complete before the call (e.g. hipStreamSynchronize of the producing
 * stream), or the caller names its producing stream with
 * jxg_set_input_stream: every later device-input call then orders its reads
 * after all work submitted to that stream so far (an event recorded on it,
 * waited on by the library's stream -- no host synchronisation).
 *
 * A context with streamed frames pending (jxg_pending > 0) serves them as a
 * pipeline lane: the one-at-a-time, batch, sharded-begin/end, homogeneity
 * and compare entry points return JXG_ERR_INVALID_ARG until they are
 * received.
 */
#ifndef JXG_H_
#define JXG_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  JXG_OK = 0,
  JXG_ERR_INVALID_ARG = -1,
  JXG_ERR_NO_DEVICE = -2,
  JXG_ERR_HIP = -3,
  JXG_ERR_OOM = -4,
  JXG_ERR_UNSUPPORTED = -5,
  JXG_ERR_INTERNAL = -6
} jxg_status;

/* proposals bitmask: the thesis patches (proposals/ directory) */
#define JXG_PROPOSAL_P 1u /* homogeneity-partitioning.diff:272-276 */
#define JXG_PROPOSAL_F 2u /* homogeneity-factored-entropy.diff:247-253 */

/* flags */
#define JXG_FLAG_H1_INT_ABS 1u /* thesis SML with int abs(int) */
#define JXG_FLAG_KEEP_MAPS 2u  /* keep per-block maps for jxg_get_stats */
#define JXG_FLAG_ANS 4u        /* ANS (12-bit rANS) for the AC stream instead of prefix codes */
#define JXG_FLAG_FORCE_ONE_STREAM 8u /* testing: the split assembly takes its one-stream
                                      * fallback (as when its prefix bound is exceeded);
                                      * same bytes */
/* restoration filters (cjxl --gaborish / --epf), off by
 * default: GABORISH applies the encoder's inverse Gaborish to the XYB image
 * before every other stage and enables the decoder's 3x3 Gaborish; EPF enables
 * the decoder's edge-preserving filter (iterations from the distance: 1 below
 * d 1.5, 2 below d 4, else 3; constant sharpness 4 per block).  Both are
 * signalled in the frame header (LoopFilter) [ext, parity with libjxl
 * unpinned; DESIGN.md §3.8] */
#define JXG_FLAG_GABORISH 16u
#define JXG_FLAG_EPF 32u
/* libjxl-shaped adaptive quantization: the masking-based initial quant field
 * (InitialQuantField / AdaptiveQuantizationMap [ext]: gamma-weighted local
 * differences, fuzzy erosion, mask, HF and gamma modulation; restated as
 * recalled, parity with libjxl unpinned; oracle/aq.c) instead of the
 * activity heuristic; one extra kernel per frame (csrc/jxg_aq.hip) */
#define JXG_FLAG_AQ_MASKING 64u
/* What `cjxl IN OUT --distance=D --effort=E` with no other flag encodes (the
 * harness's argv, benchmark-jpegxl/src/docker_manager.rs:126-136): cjxl's
 * VarDCT defaults [ext] -- ANS, Gaborish, EPF iterations by distance, the
 * masking quant field.  jxg_cjxl starts from this set, INTEGRATION.md's
 * execute_cjxl over the C ABI passes it, and bench.py's headline value is
 * measured with it; the same (image, distance, effort, proposals) give the
 * same bytes through either route (tests/test_gpu_cli.py). */
#define JXG_FLAGS_CJXL_DEFAULTS (JXG_FLAG_ANS | JXG_FLAG_GABORISH | JXG_FLAG_EPF | JXG_FLAG_AQ_MASKING)

/* opaque encoder context (one HIP device, its streams and buffers) */
typedef struct jxg_ctx jxg_ctx;

typedef struct {
  float distance;      /* cjxl --distance (butteraugli target), (0, 25] */
  int effort;          /* cjxl --effort 1..9 (>=5: 8x8-class ACS search) */
  uint32_t proposals;  /* JXG_PROPOSAL_* */
  int num_devices;     /* informative; multi-GPU runs one context per rank */
  uint32_t flags;      /* JXG_FLAG_* */
  int device;          /* HIP device ordinal */
} jxg_params;

typedef struct {
  uint8_t* data;
  size_t size;
} jxg_buffer;

typedef struct {
  uint32_t xsize, ysize, xsize_blocks, ysize_blocks;
  uint32_t num_groups, num_lf_groups;
  uint32_t global_scale, quant_dc;
  size_t bytes;
  /* valid until the next encode on this context (JXG_FLAG_KEEP_MAPS) */
  const uint8_t* ac_strategy;  /* [ysize_blocks][xsize_blocks] raw strategy */
  const uint8_t* quant_field;  /* raw quant field - 1 */
  const int32_t* dc;           /* [3][blocks] quantized DC (X, Y, B) */
  const int32_t* ac;           /* [blocks][3][64] quantized AC, natural order */
  const uint32_t* ac_tokens;   /* [num_groups][3] AC token counts (X, Y, B) */
  const float* homogeneity;    /* [blocks][3] r_h r_v r_d (if P|F) */
  /* device time per stage, milliseconds (last encode) */
  float ms_front, ms_histogram, ms_emit, ms_assemble, ms_total;
  /* host wall clock of the whole call and of the host-side code/header work */
  float ms_host_call, ms_host_codes, ms_host_layout;
  /* device time of the fused front kernel alone (XYB + ACS + DCT + quant);
   * ms_front also covers the masking quant field and the merge stage */
  float ms_front_kernel;
  /* device time of the masking quant field kernel (JXG_FLAG_AQ_MASKING; 0 otherwise) */
  float ms_aq;
} jxg_stats;

const char* jxg_status_str(jxg_status s);
jxg_status jxg_create(const jxg_params* params, jxg_ctx** ctx);
void jxg_destroy(jxg_ctx* ctx);
/* the caller's stream (hipStream_t) that produces device inputs; NULL: none
 * (writes complete before each call) -- see the conventions above */
jxg_status jxg_set_input_stream(jxg_ctx* ctx, void* stream);

/* host RGB8 (interleaved, row_stride bytes per row) -> codestream */
jxg_status jxg_encode_rgb8(jxg_ctx* ctx, const uint8_t* rgb, uint32_t xsize, uint32_t ysize,
                           size_t row_stride, jxg_buffer* out);
/* device-resident RGB8 (same layout, device pointer) -> codestream */
jxg_status jxg_encode_rgb8_device(jxg_ctx* ctx, const void* d_rgb, uint32_t xsize,
                                  uint32_t ysize, size_t row_stride, jxg_buffer* out);
/* n frames of equal size (benchmark config 3: 64 x 1080p; the reference's
 * caller encodes every image at 10 distances x 5 efforts, benchmark.rs:
 * 637-642), through the streaming pipeline below (jxg_submit_rgb8 of every
 * frame, codestreams collected as they complete), so the frames' H2D copies,
 * kernels, rANS chains and host-side code construction overlap over the
 * pipeline's lanes.  outs[i] is frame i's codestream (byte-identical to
 * jxg_encode_rgb8 of that frame); on error every output is released.  The
 * context must have no streamed frames pending (JXG_ERR_INVALID_ARG
 * otherwise).  jxg_get_stats then describes the last frame. */
jxg_status jxg_encode_batch_rgb8(jxg_ctx* ctx, const uint8_t* const* rgbs, uint32_t n,
                                 uint32_t xsize, uint32_t ysize, size_t row_stride,
                                 jxg_buffer* outs);
/* the same with device-resident frames */
jxg_status jxg_encode_batch_rgb8_device(jxg_ctx* ctx, const void* const* d_rgbs, uint32_t n,
                                        uint32_t xsize, uint32_t ysize, size_t row_stride,
                                        jxg_buffer* outs);
/* Streaming encode, one host thread: frames are submitted in order and their
 * codestreams received in the same order (byte-identical to jxg_encode_rgb8
 * of each frame).  Internally a software pipeline over this context and up to
 * 11 lanes it creates on first use (same parameters; released by
 * jxg_destroy); the depth D follows the frame size (7 lanes at 8K, 12 at 4K
 * and below; jxg_pipeline_depth), never more than the process's hardware
 * queues - 1 (GPU_MAX_HW_QUEUES, HIP's default 4: raise it, at most 32,
 * before HIP initialises for the full depth -- two lanes on one queue
 * serialise their kernels): a submit finishes the frame submitted D calls earlier if it is
 * still in flight, launches the new frame's front end / merge stage /
 * statistics on a free lane, starts the previous frame's codes on a helper
 * thread and joins the codes of the frame `lag` submits back (1 at 8K, 3 for
 * small frames), whose helper launched its emission -- so the rANS chains
 * (JXG_FLAG_ANS) of earlier frames run under the transform kernels of the
 * next.  Each lane uses its own HIP stream: the process needs that many
 * hardware queues (GPU_MAX_HW_QUEUES=16 set before the HIP runtime starts).
 * jxg_receive blocks until the oldest frame is complete
 * (JXG_ERR_INVALID_ARG if none is pending); jxg_pending counts frames
 * submitted and not yet received.  A device frame must stay unchanged until
 * its codestream is received; a host frame is copied into pinned staging
 * before jxg_submit_rgb8 returns.  jxg_get_stats after jxg_receive describes
 * the received frame.  On an error every frame in flight is dropped. */
jxg_status jxg_submit_rgb8(jxg_ctx* ctx, const uint8_t* rgb, uint32_t xsize, uint32_t ysize,
                           size_t row_stride);
jxg_status jxg_submit_rgb8_device(jxg_ctx* ctx, const void* d_rgb, uint32_t xsize, uint32_t ysize,
                                  size_t row_stride);
jxg_status jxg_receive(jxg_ctx* ctx, jxg_buffer* out);
jxg_status jxg_pending(jxg_ctx* ctx, uint32_t* n);
/* frames the streaming pipeline keeps in flight for frames of this size
 * (world == 1) or for this rank's shard of them (jxg_shard_submit_device):
 * lanes x frames per lane (one batched launch per lane), less what keeps a
 * lane free for the next submit -- (lanes - 1) x batch + 1 */
jxg_status jxg_pipeline_depth(jxg_ctx* ctx, uint32_t xsize, uint32_t ysize, uint32_t rank,
                              uint32_t world, uint32_t* depth);
/* at most `lanes` pipeline lanes (1..12; 0: the default, GPU_MAX_HW_QUEUES - 1)
 * for this context's later streams -- for several contexts streaming on ONE
 * GPU (ranks rehearsed on a shared device), which would otherwise put up to
 * 12 lanes each on the same hardware queues.  JXG_ERR_INVALID_ARG while
 * frames are pending.  jxg_pipeline_depth reflects the cap. */
jxg_status jxg_set_pipeline_lanes(jxg_ctx* ctx, uint32_t lanes);
jxg_status jxg_get_stats(jxg_ctx* ctx, jxg_stats* stats);
void jxg_buffer_free(jxg_buffer* buf);

/* ---- multi-GPU group sharding (one context per rank) ----
 * A frame's 256x256 pass groups are split over `world` ranks (jxg_shard_plan):
 *   kind 0: balanced contiguous raster ranges (rank r: [n*r/world,
 *           n*(r+1)/world)), every LF group (2048x2048) owned by the rank of
 *           most of its pass groups, when that leaves no LF group split over
 *           ranks (16384^2 over 8);
 *   kind 1: else whole LF groups per rank (largest first to the least-loaded
 *           rank) when the largest load is within 5 % of the mean (8K over
 *           2 / 4 / 8): no per-block records move;
 *   kind 2: else the ranges of kind 0 with the record exchange below.
 * The owner of an LF group encodes its LF-group stream.  Per rank:
 *   1. jxg_shard_sizes: words of the AC histogram (132 x 128 counts, then
 *      the rank's varblock count per 128 / 256 px kind, whose sum decides
 *      which quant tables HfGlobal carries) and the byte capacity of the
 *      record send / receive buffers (the largest of any rank);
 *      jxg_shard_exchange: this rank's send and receive bytes per peer;
 *   2. jxg_shard_begin: front end + merge stage + AC token statistics of the
 *      rank's groups; writes the rank's AC histogram to d_hist (u32, device)
 *      and, into d_xbuf (device), the per-block records (strategy, quant
 *      field, quantized DC; 14 KB per pass group) of its groups whose LF group
 *      another rank owns, ordered by destination rank;
 *   -- caller: prefix codes only, all-reduce(sum) d_hist (ANS: nothing, see
 *      below); all_to_all of the records with the jxg_shard_exchange splits
 *      (RCCL over xGMI) into a receive buffer (kinds 0 / 1: all splits 0);
 *   3. jxg_shard_end(d_hist, receive buffer): LF-group streams of its LF
 *      groups, entropy codes, emission of the rank's sections into a payload
 *      kept in device memory (rank 0's also carries LfGlobal, and HfGlobal
 *      with prefix codes); jxg_shard_payload copies it (payload_bytes) to
 *      device or host memory;
 *   -- caller: gather the payloads on rank 0 (RCCL, device to device);
 *   4. jxg_shard_assemble_device (rank 0): payloads in device memory (word
 *      aligned offsets) -> codestream in host memory; or jxg_shard_assemble:
 *      the same from host payloads, host only (no device).
 * Prefix codes (one HF preset from the summed histogram): payload heads of
 * version 1, and the codestream is byte-identical to jxg_encode_rgb8 of the
 * whole frame.  ANS (JXG_FLAG_ANS) with world > 1: every rank clusters its
 * own histogram into its own HF preset, so d_hist needs NO all-reduce; the
 * payload head is version 2 and carries the preset, HfGlobal is written at
 * assembly with num_hf_presets = world, and every pass group selects its
 * rank's preset -- the codestream decodes to exactly the single-GPU image
 * (same coefficients, strategies, quant field, DC, CfL), but its bytes differ
 * from jxg_encode_rgb8's.  The frame needs at least max(2, world) pass groups.
 * Codestreams are released with jxg_buffer_free. */
jxg_status jxg_shard_sizes(uint32_t xsize, uint32_t ysize, uint32_t world, size_t* hist_words,
                           size_t* slot_bytes);
/* the partition: owner rank of every pass group ([num_groups]) and LF group
 * ([num_lf_groups]), and its kind (0 / 1 / 2 above); any pointer may be NULL */
jxg_status jxg_shard_plan(uint32_t xsize, uint32_t ysize, uint32_t world, uint32_t* group_owner,
                          uint32_t* lf_owner, int* kind);
jxg_status jxg_shard_exchange(uint32_t xsize, uint32_t ysize, uint32_t world, uint32_t rank,
                              size_t* send_bytes /* [world] */, size_t* recv_bytes /* [world] */);
jxg_status jxg_shard_begin(jxg_ctx* ctx, const void* d_rgb, uint32_t xsize, uint32_t ysize,
                           size_t row_stride, uint32_t rank, uint32_t world, uint32_t* d_hist,
                           void* d_xbuf);
jxg_status jxg_shard_end(jxg_ctx* ctx, const uint32_t* d_hist, const void* d_xbuf,
                         size_t* payload_bytes);
jxg_status jxg_shard_payload(jxg_ctx* ctx, void* dst, int dst_on_device);
jxg_status jxg_shard_assemble_device(jxg_ctx* ctx, const void* d_payloads, const size_t* offsets,
                                     const size_t* sizes, uint32_t n, jxg_buffer* out);
jxg_status jxg_shard_assemble(const uint8_t* const* payloads, const size_t* sizes, uint32_t n,
                              jxg_buffer* out);

/* Distributed host assembly (instead of the payload gather + rank-0
 * assembly): after jxg_shard_end every rank exports its payload head
 * (jxg_shard_head: a few hundred u32; dst NULL -> *nwords = size), the heads
 * are all-gathered (any collective), and every rank calls
 * jxg_shard_write_host with all heads in rank order: it writes its own
 * sections D2H into `dst` -- one host buffer shared by all ranks (e.g. a
 * /dev/shm mapping, registered with jxg_host_register for DMA) -- at their
 * codestream offsets; rank 0 also writes headers + TOC.  *total = codestream
 * bytes (also returned with JXG_ERR_INVALID_ARG when dst_size is too small).
 * Once every rank has returned (a barrier), dst[0, total) holds the
 * codestream, byte-identical to jxg_shard_assemble_device. */
jxg_status jxg_shard_head(jxg_ctx* ctx, uint32_t* dst, size_t* nwords);
jxg_status jxg_shard_write_host(jxg_ctx* ctx, const uint32_t* const* heads, const size_t* head_words,
                                uint32_t n, void* dst, size_t dst_size, size_t* total);
/* Streaming sharded encode (the multi-GPU pipeline; kinds 0 / 1 with ANS, or
 * world == 1): every rank submits its shard of consecutive frames, in the
 * same order, through the same lanes as jxg_submit_rgb8_device -- front end,
 * merge stage, statistics, codes and rANS chains of several frames overlap,
 * with no collective inside a frame.  For each frame, in submission order:
 *   jxg_shard_next_head: waits until the oldest pending frame's sections are
 *     emitted and exports its payload head (dst NULL -> *nwords = size; the
 *     frame stays pending);
 *   -- caller: all-gather the heads (any collective);
 *   jxg_shard_write_next: as jxg_shard_write_host for that frame (its
 *     sections D2H into the shared host buffer at their codestream offsets,
 *     rank 0 adds headers + TOC), then releases its slot.  The copies are
 *     enqueued and NOT waited for: the call returns once the copies of the
 *     write JXG_SHARD_WRITE_LAG calls back have landed (this rank's part of
 *     frame k is in place when write_next of frame k + JXG_SHARD_WRITE_LAG
 *     returns, or after jxg_shard_write_flush);
 *   jxg_shard_write_flush: waits for every write's copies.
 * A frame's codestream is complete once every rank's part is in place.  At
 * most jxg_pipeline_depth frames may be pending (submit returns
 * JXG_ERR_INVALID_ARG when full; JXG_ERR_UNSUPPORTED for a plan needing the
 * record exchange or, with world > 1, for prefix codes).  The frame's device
 * RGB8 must stay unchanged until its write. */
jxg_status jxg_shard_submit_device(jxg_ctx* ctx, const void* d_rgb, uint32_t xsize, uint32_t ysize,
                                   size_t row_stride, uint32_t rank, uint32_t world);
jxg_status jxg_shard_next_head(jxg_ctx* ctx, uint32_t* dst, size_t* nwords);
jxg_status jxg_shard_write_next(jxg_ctx* ctx, const uint32_t* const* heads, const size_t* head_words,
                                uint32_t n, void* dst, size_t dst_size, size_t* total);
#define JXG_SHARD_WRITE_LAG 2
jxg_status jxg_shard_write_flush(jxg_ctx* ctx);
/* page-lock a host range (e.g. the node-shared /dev/shm codestream buffer of
 * jxg_shard_write_host / jxg_shard_write_next) so the ranks' D2H copies are DMA */
jxg_status jxg_host_register(void* ptr, size_t size);
jxg_status jxg_host_unregister(void* ptr);

/* thesis selector alone over a host XYB frame [3][ysize][xsize] (xsize, ysize
 * multiples of 8): r3 = (r_h, r_v, r_d) per block, type = raw strategy
 * (combined.diff:183-235) */
jxg_status jxg_homogeneity_map(jxg_ctx* ctx, const float* xyb, uint32_t xsize, uint32_t ysize,
                               float distance, uint32_t flags, float* r3, uint8_t* type);

/* ---- decode-side quality: the harness's metrics on the GPU ----
 * Replaces ImageReader::calculate_mse / calculate_psnr
 * (benchmark-jpegxl/src/image_reader.rs:555-606, via metrics.rs:28-53) and
 * calculate_ssim (metrics.rs:55-84, ImageMagick `compare -metric SSIM`).
 * orig / comp: RGB8 interleaved rows (comp = the decoded image).  mse is
 * bit-identical to the reference's sequential f64 sum; ssim is the mean
 * Gaussian-window (11x11, sigma 1.5, K1 0.01, K2 0.03) SSIM over all window
 * positions inside the image and the three channels -- ImageMagick's exact
 * variant is not in the reference (parity unpinned). */
typedef struct {
  uint64_t sse;     /* sum of squared sample differences (exact) */
  uint64_t samples; /* 3 * xsize * ysize */
  double mse;       /* sse / samples */
  double psnr;      /* 10 log10(255^2 / mse); +inf when mse == 0 */
  double ssim;      /* NaN when not requested or the image is under 11x11 */
} jxg_quality;

jxg_status jxg_compare_rgb8(jxg_ctx* ctx, const uint8_t* orig, size_t orig_stride,
                            const uint8_t* comp, size_t comp_stride, uint32_t xsize,
                            uint32_t ysize, int want_ssim, jxg_quality* out);
jxg_status jxg_compare_rgb8_device(jxg_ctx* ctx, const void* d_orig, size_t orig_stride,
                                   const void* d_comp, size_t comp_stride, uint32_t xsize,
                                   uint32_t ysize, int want_ssim, jxg_quality* out);

/* Prepares the context for frames of xsize x ysize before the first one
 * arrives: encodes one synthetic frame of that size (device-generated, result
 * discarded), which allocates the size's device buffers and loads every
 * kernel.  Optional -- a caller that creates a context per image (the
 * harness's execute_cjxl pattern, docker_manager.rs:126-136) runs it beside
 * its image decode; jxg_cjxl does.  Not while streamed frames are pending. */
jxg_status jxg_warmup(jxg_ctx* ctx, uint32_t xsize, uint32_t ysize);
/* ---- benchmark input ----
 * The deterministic synthetic RGB8 frame of SURVEY.md §8(d) (64x64 tiles of
 * flat / gradient / stripe / checker / edge / noise content, splitmix64
 * hashes, seed 0x4A584C00 + config index), written into device memory
 * d_out (row_stride bytes per row) on the context's stream; returns when it
 * is complete.  Same bytes as jxg/synth.py synth_rgb8. */
jxg_status jxg_synth_rgb8_device(jxg_ctx* ctx, void* d_out, uint32_t xsize, uint32_t ysize,
                                 size_t row_stride, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif
