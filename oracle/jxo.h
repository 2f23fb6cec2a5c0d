/*
 * jxo.h -- CPU ORACLE (test infrastructure only; never shipped, never measured
 * as the product).  Plain-C restatement of the JPEG XL VarDCT encode path the
 * MI355X build accelerates, used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker.
 *
 * Provenance of each part:
 *  - homog.c : thesis homogeneity selector, restated from
 *              /root/reference/proposals/combined.diff:17-235 (+ hook F :247-253,
 *              hook P :270-274).  Parity vs the reference is pinned by
 *              hand-derived known-answer vectors from the diff text
 *              (tests/golden/homog_kat.json); the verbatim patch cannot be
 *              compiled here (it needs libjxl's ACSConfig/AcStrategy headers,
 *              which are absent; stand-ins are not allowed) -- see DESIGN.md.
 *  - the libjxl stages (XYB, AQ, ACS, DCT, quant, tokens, prefix/ANS coding,
 *    headers) are [ext]: libjxl is not in /root/reference (it is cloned
 *    unpinned at benchmark-jpegxl/Dockerfile:40).  They are restated from the
 *    JPEG XL format as documented in DESIGN.md; "parity unpinned" against
 *    libjxl.  The GPU path must match THIS oracle bit-for-bit.
 */
#ifndef JXO_H_
#define JXO_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* raw AcStrategy ids (combined.diff:227-233 returns DCT=0, DCT4X4=3,
 * DCT4X8=12, DCT8X4=13) */
enum { JXO_DCT8 = 0, JXO_IDENTITY = 1, JXO_DCT2X2 = 2, JXO_DCT4X4 = 3,
       JXO_DCT4X8 = 12, JXO_DCT8X4 = 13 };

/* XYB plane view.  Samples outside [0,xsize)x[0,ysize) read as 0.0f
 * (SURVEY H2 convention: the reference reads row padding / before-plane memory
 * there).  xsize/ysize are the block-padded frame dimensions. */
typedef struct {
  const float* plane[3]; /* X, Y, B */
  size_t xsize, ysize, stride;
} jxo_xyb;

/* flags for the H1 'abs' ambiguity */
#define JXO_H1_FLOAT_ABS 0 /* canonical: fabs on float */
#define JXO_H1_INT_ABS 1   /* int abs(int) overload resolution */

float jxo_homogeneity(const jxo_xyb* img, size_t x, size_t y, size_t xs,
                      size_t ys, size_t bx, size_t by, float distance,
                      int h1_mode);
void jxo_homog_indices(const jxo_xyb* img, size_t x, size_t y, float distance,
                       int h1_mode, float* r_h, float* r_v, float* r_d);
uint8_t jxo_homog_partition(const jxo_xyb* img, size_t x, size_t y,
                            float distance, int h1_mode);
/* hook F: ret * 0.8 * avg_r evaluated in double, stored to float */
float jxo_hook_f(float ret, float r_h, float r_v, float r_d);
/* whole-frame map: r3[3*block] = (r_h, r_v, r_d), type[block] */
void jxo_homog_map(const jxo_xyb* img, float distance, int h1_mode, float* r3,
                   uint8_t* type);

/* ---------------- full encoder oracle (encode.c) ---------------- */
typedef struct {
  float distance;
  int effort;
  uint32_t proposals; /* bit0 = P (homogeneity-partitioning), bit1 = F */
  int coder;          /* 0 = prefix codes, 1 = ANS */
  uint32_t filters;   /* JXO_FILTER_*: restoration filters the frame signals */
} jxo_params;

/* restoration filters [ext: libjxl LoopFilter, cjxl
 * --gaborish / --epf]: GAB = the encoder's inverse Gaborish on XYB and the
 * decoder's 3x3 Gaborish; EPF = the decoder's edge-preserving filter,
 * jxo_epf_iters(distance) iterations, constant sharpness JXO_EPF_SHARPNESS */
#define JXO_FILTER_GAB 1u
#define JXO_FILTER_EPF 2u
/* encoder option in the same mask (not a filter): the libjxl-shaped masking
 * quant field (aq.c) instead of the activity heuristic */
#define JXO_OPT_AQ_MASKING 4u
#define JXO_EPF_SHARPNESS 4
int jxo_epf_iters(float distance);
/* loop-filter code of the frame header: bit 0 gab, bits 1-2 epf_iters */
uint32_t jxo_lf_code(uint32_t filters, float distance);
/* in place on a [3][yp][xp] XYB frame (edge replication at its borders) */
void jxo_gab_inverse(float* xyb, uint32_t xp, uint32_t yp);

typedef struct {
  uint32_t xsize, ysize;   /* image */
  uint32_t bxs, bys;       /* blocks */
  uint8_t* acs;            /* [bys*bxs] raw strategy */
  uint8_t* qf;             /* [bys*bxs] quant field raw-1 (0..255) */
  int32_t* dc;             /* [3][bys*bxs] quantized DC, channel order X,Y,B */
  int32_t* ac;             /* [bys*bxs][3][64] quantized coeffs (X,Y,B) */
  uint32_t* ac_tokens;     /* [ngroups][3] number of AC tokens per channel */
  float* homog;            /* [bys*bxs][3] r_h r_v r_d (only if P|F) */
  int8_t* cmap;            /* [2][tiles_y*tiles_x] chroma from luma: ytox, ytob per 64x64 tile */
  uint32_t tiles_x, tiles_y;
  uint32_t global_scale, quant_dc;
  uint8_t* bytes;          /* encoded codestream */
  size_t nbytes;
} jxo_result;

int jxo_encode_rgb8(const uint8_t* rgb, uint32_t w, uint32_t h,
                    size_t row_stride, const jxo_params* p, jxo_result* out);
void jxo_result_free(jxo_result* r);
/* synthetic RGB8 frame (jxg/synth.py synth_rgb8), out: h*w*3 bytes */
void jxo_synth_rgb8(uint32_t w, uint32_t h, uint64_t seed, uint8_t* out);
/* OpenMP threads of the encode's parallel loops (n <= 0: query only) */
int jxo_set_threads(int n);

/* stage-level entry points (used by tests) */
void jxo_srgb8_to_xyb(const uint8_t* rgb, uint32_t w, uint32_t h,
                      size_t row_stride, uint32_t xsize_pad, uint32_t ysize_pad,
                      float* xyb /* [3][ysize_pad][xsize_pad] */);
float jxo_cbrtf(float x);

#ifdef __cplusplus
}
#endif
#endif
