/*
 * jxo_internal.h -- ORACLE internals (test infrastructure only).
 * Constant tables of the JPEG XL VarDCT format [ext: ISO/IEC 18181-1 / libjxl,
 * not in /root/reference; restated, parity unpinned against libjxl].
 */
#ifndef JXO_INTERNAL_H_
#define JXO_INTERNAL_H_
#include <stddef.h>
#include <stdint.h>

#include "jxo.h"

/* opsin absorbance matrix and bias [ext libjxl opsin_params.h] */
#define JXO_M00 0.30f
#define JXO_M01 0.622f
#define JXO_M02 0.078f
#define JXO_M10 0.23f
#define JXO_M11 0.692f
#define JXO_M12 0.078f
#define JXO_M20 0.24342268924547819f
#define JXO_M21 0.20476744424496821f
#define JXO_M22 0.55180986650955360f
#define JXO_BIAS 0.0037930732552754493f

void jxo_srgb_lut(float lut[256]);
void jxo_pixel_xyb(const float lut[256], const float cb, uint8_t r, uint8_t g,
                   uint8_t b, float* X, float* Y, float* B);

/* ---- frame geometry / quantizer scalars (all computed on the host) ---- */
typedef struct {
  uint32_t w, h, bxs, bys, xp, yp;
  uint32_t gxs, gys, ngroups, lfxs, lfys, nlf;
  float distance;
  int effort;
  uint32_t proposals;
  float qf_base, inv_g;
  uint32_t G, qdc;
  float dc_mul[3], dc_step[3];
  float wts[5][3][64]; /* [quant kind][channel X,Y,B][coef] */
  float sdw[6][3][64];  /* [8x8-class strategy index][channel][coef] distortion weights */
} jxo_frame;

/* estimate multipliers of the two Haar-type 8x8 candidates (the search's
 * (bits + 8 dist) * tmul; DCT8 1.0, DCT4X4 1.05, DCT4X8 / DCT8X4 1.02) */
#ifndef JXO_TMUL_DCT2
#define JXO_TMUL_DCT2 1.05f
#endif
#ifndef JXO_TMUL_ID
#define JXO_TMUL_ID 1.08f
#endif
enum { JXO_QK_DCT8 = 0, JXO_QK_DCT4 = 1, JXO_QK_DCT4X8 = 2, JXO_QK_ID = 3, JXO_QK_DCT2 = 4 };

void jxo_frame_init(jxo_frame* f, uint32_t w, uint32_t h, const jxo_params* p);
void jxo_quant_weights(int kind, float out[3][64]);
/* distortion weight of a coefficient (see front.c jxo_dist_weight) */
float jxo_dist_weight(int c, int area, float w);
extern const float jxo_w0[3];
void jxo_natural_order8(uint8_t order[64]);
void jxo_quant_dc(const jxo_frame* f, const float dc[3], int32_t dcq[3]);

/* AC context model constants [ext libjxl ac_context.h] */
#define JXO_NUM_ORDERS 13
#define JXO_NZ_BUCKETS 37
#define JXO_ZD_CTX 458
#define JXO_BLOCK_CTX 15
#define JXO_AC_CTX (JXO_BLOCK_CTX * (JXO_NZ_BUCKETS + JXO_ZD_CTX)) /* 7425 */
extern const uint8_t jxo_strategy_order[27];
extern const uint8_t jxo_default_ctx_map[39];
extern const uint8_t jxo_freq_ctx[64];
extern const uint16_t jxo_nnz_ctx[64];

/* merged varblocks (merge.c) [ext AcStrategy / quant_weights / coeff_order] */
enum { JXO_VK_16X8 = 0, JXO_VK_16, JXO_VK_32X16, JXO_VK_32, JXO_VK_64X32, JXO_VK_64,
       JXO_VK_128X64, JXO_VK_128, JXO_VK_256X128, JXO_VK_256, JXO_NVKINDS };
typedef struct {
  uint8_t type, cy, cx, kind; /* raw id, blocks down, blocks across, weight kind */
  float tmul;                 /* cost multiplier of the search */
} jxo_shape;
/* shapes by level L (16, 32, 64, 128, 256 px): tall 3L, wide 3L + 1, full
 * 3L + 2; levels 128 / 256 (raw ids 21-26) are searched at effort >= 8 */
#define JXO_NSHAPES 15
#define JXO_NTILE_SHAPES 9 /* levels <= 64: inside one 64x64 tile */
#define JXO_LLF_DIM 32     /* LLF buffers: [3][32][32] (a 256x256 varblock's) */
extern const jxo_shape jxo_shapes[JXO_NSHAPES];
typedef struct {
  int rows, cols; /* stored orientation: rows = 8 min(cy,cx), cols = 8 max(cy,cx) */
  float* w[3];    /* weights per channel X, Y, B, stored raster */
  float* sd[3];   /* distortion weights jxo_dist_weight(c, rows*cols, w) */
  uint16_t* nat;  /* stored raster index -> natural order position */
} jxo_vkind;
const jxo_vkind* jxo_vkinds(void);
/* weight parameters of a kind as the stream carries them (merge.c): kinds
 * 128X64 ... 256X256 rounded through binary16 (written explicitly into
 * DequantMatrices), the others the library defaults */
double jxo_kind_param(int kind, int c, int i);
int jxo_kind_num_bands(int kind);
double jxo_f16_round(double v);
uint32_t jxo_f16_bits(double v);
int jxo_shape_of(int type); /* shape index of a merged raw id, -1 otherwise */
float jxo_varblock(const jxo_frame* f, const jxo_shape* s, const float* xyb, int px0, int py0,
                   int raw, int32_t* q /* [3][R*C] natural order */, float* llf /* [3][32][32] */,
                   int* nz /* [3] */, const float cfl[2] /* chroma-from-luma kx, kb */);
float jxo_llf_dc(const jxo_shape* s, const float* llf_c, int by, int bx);
void jxo_merge_tile(const jxo_frame* f, const float* xyb, const float* homog, int tx, int ty,
                    int max_s, float* ent, const int* raw, uint8_t* acs, const float cfl[2]);
/* levels 128 / 256 px (s = 16 / 32 blocks) over the whole frame, after every
 * tile's merge (regions span tiles; a candidate's chroma-from-luma factors
 * are those of its top-left block's tile, as the decoder applies them) */
void jxo_merge_big(const jxo_frame* f, const float* xyb, const float* homog, int s, float* ent,
                   const int* raw, uint8_t* acs, const int8_t* cmap, uint32_t tiles_x,
                   size_t ntiles);
/* chroma from luma (front.c): the tile's int8 factors, and kx, kb from them */
void jxo_cfl_tile(const jxo_frame* f, const float* xyb, int tx, int ty, int8_t* ytox,
                  int8_t* ytob);
void jxo_cfl_factors(int8_t ytox, int8_t ytob, float cfl[2]);
void jxo_transform(int t, const float* px, float* co);
/* covered 8x8 blocks of a raw strategy id (1 for the 8x8 class) */
static inline int jxo_covered(int type) {
  const int s = jxo_shape_of(type);
  return s < 0 ? 1 : jxo_shapes[s].cy * jxo_shapes[s].cx;
}

#define JXO_MAX_CLUSTERS 132
#define JXO_ALPHA 128
int jxo_ac_cluster(int ctx);

/* bit writer */
typedef struct {
  uint8_t* buf;
  size_t cap;   /* bytes */
  size_t nbits;
} jxo_bw;
void jxo_bw_init(jxo_bw* w);
void jxo_bw_put(jxo_bw* w, uint32_t nbits, uint64_t v);
void jxo_bw_pad(jxo_bw* w);
void jxo_bw_append(jxo_bw* dst, const jxo_bw* src); /* bit-concat */
void jxo_bw_free(jxo_bw* w);

/* hybrid uint */
typedef struct {
  uint32_t split_exp, msb, lsb;
} jxo_uintcfg;
void jxo_hybrid(uint32_t v, const jxo_uintcfg* c, uint32_t* tok, uint32_t* nb,
                uint32_t* bits);

/* prefix codes */
typedef struct {
  uint32_t alphabet; /* written alphabet size */
  uint8_t len[JXO_ALPHA > 256 ? JXO_ALPHA : 256];
  uint16_t code[256]; /* bit-reversed canonical code */
  int nsym;           /* used symbols */
  int simple;         /* simple code NSYM (1..4), 0 = complex */
  int tree_select;
  uint16_t ssyms[4];
} jxo_prefix;
void jxo_build_prefix(const uint32_t* counts, int n, jxo_prefix* p);
void jxo_write_prefix(jxo_bw* w, const jxo_prefix* p);

/* ANS (ans.c): normalized 12-bit frequencies, alias inverse */
typedef struct {
  uint16_t freq[128];
  uint16_t cum[128];
  uint16_t inv[4096]; /* [cum[s] + off] -> alias table position */
  int nused, omit, omit_code;
} jxo_ans;
void jxo_ans_normalize(const uint32_t* counts /* [128] */, jxo_ans* a);
void jxo_ans_write_hist(jxo_bw* w, const jxo_ans* a);
/* at most 8 clustered histograms: their alias inverses (64 KB) share a CU's
 * LDS with the GPU's other kernels, so the rANS chains of one frame overlap the
 * transform stages of the next (16 would be 128 KB for +1.2% smaller output on
 * the synthetic 8K frame, +0.2% on natural content); a new centre needs >= 64
 * bits of merge cost (Q16) */
#ifndef JXO_ANS_MAX_HISTS
#define JXO_ANS_MAX_HISTS 8
#endif
#define JXO_ANS_MIN_DIST (64ll << 16)
/* hist[nh][128] -> assign[nh] (centre id, -1 for empty); returns #centres */
int jxo_ans_cluster(const uint32_t (*hist)[JXO_ALPHA], int nh, int* assign);
void jxo_ans_write_stream(jxo_bw* w, const jxo_ans* hists, size_t n, const uint8_t* hist,
                          const uint8_t* sym, const uint8_t* nbits, const uint32_t* bits);

/* libjxl-shaped masking quant field (aq.c): raw - 1 of every block [bys][bxs],
 * on the block-padded XYB frame before the inverse Gaborish */
void jxo_aq_masking(const jxo_frame* f, const float* xyb, uint8_t* raw);
/* its stages (the GPU kernel jxg_aq.hip follows them op for op) */
float jxo_aq_diff(const float* Y, uint32_t xp, uint32_t yp, int x, int y);
float jxo_aq_cell(const float* Y, uint32_t xp, uint32_t yp, int cx, int cy);
void jxo_aq_erosion_weights(float distance, float w[4]);
float jxo_aq_erode(const float* cells, int ncx, int ncy, int cx, int cy, const float w[4]);
float jxo_aq_mask(float v);
float jxo_aq_modulate(const float* X, const float* Y, uint32_t xp, int bx, int by, float v);

#endif
