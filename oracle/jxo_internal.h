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
  float wts[3][3][64]; /* [quant kind][channel X,Y,B][coef] */
} jxo_frame;

enum { JXO_QK_DCT8 = 0, JXO_QK_DCT4 = 1, JXO_QK_DCT4X8 = 2 };

void jxo_frame_init(jxo_frame* f, uint32_t w, uint32_t h, const jxo_params* p);
void jxo_quant_weights(int kind, float out[3][64]);
void jxo_natural_order8(uint8_t order[64]);

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

#endif
