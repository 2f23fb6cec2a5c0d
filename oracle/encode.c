/*
 * encode.c -- ORACLE (test infrastructure).  Whole-frame VarDCT encode:
 * front end per block, AC tokenization per 256x256 pass group, LF-group
 * modular streams (quantized DC + AC metadata), prefix-coded entropy streams,
 * headers, TOC and section assembly.
 *
 * [ext] JPEG XL codestream layout (ISO/IEC 18181-1; libjxl dec_frame.cc,
 * dec_group.cc, dec_modular.cc, frame_header.h, headers.h).  None of it is in
 * /root/reference; restated per DESIGN.md §3, parity unpinned against libjxl.
 * The harness contract it serves is benchmark-jpegxl/src/docker_manager.rs:
 * 100-137 (execute_cjxl) -- a .jxl decodable to 8-bit RGB.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "jxo_internal.h"

int jxo_front_block(const jxo_frame* f, const float px[3][64], const float* homog,
                    int32_t q[3][64], int32_t dcq[3], int* qf_raw, float* ent_out,
                    const float cfl[2], int aq_raw);

static const jxo_uintcfg kCfg = {4, 2, 0};

uint32_t* jxo_debug_group_bins = NULL; /* tests: see the AC token loop */
void jxo_set_debug_group_bins(uint32_t* p) { jxo_debug_group_bins = p; }
static const jxo_uintcfg kCfgMap = {8, 0, 0};

static uint32_t ceil_log2(uint32_t x) { /* CeilLog2Nonzero */
  uint32_t n = 0;
  while ((1u << n) < x) n++;
  return n;
}
static uint32_t pack_signed(int32_t v) {
  return v >= 0 ? (uint32_t)v * 2u : (uint32_t)(-(int64_t)v) * 2u - 1u;
}

/* ------------------------- field writers ------------------------- */
static void put_u32_sel(jxo_bw* w, uint32_t sel, uint32_t nbits, uint32_t v) {
  jxo_bw_put(w, 2, sel);
  jxo_bw_put(w, nbits, v);
}
static void put_varlen16(jxo_bw* w, uint32_t v) {
  if (v == 0) {
    jxo_bw_put(w, 1, 0);
    return;
  }
  uint32_t n = 0;
  while ((v >> (n + 1)) != 0) n++;
  jxo_bw_put(w, 1, 1);
  jxo_bw_put(w, 4, n);
  jxo_bw_put(w, n, v - (1u << n));
}
static void put_uintcfg(jxo_bw* w, const jxo_uintcfg* c) { /* log_alpha = 15 */
  jxo_bw_put(w, 4, c->split_exp);
  if (c->split_exp != 15) {
    jxo_bw_put(w, ceil_log2(c->split_exp + 1), c->msb);
    jxo_bw_put(w, ceil_log2(c->split_exp - c->msb + 1), c->lsb);
  }
}
static void put_token(jxo_bw* w, const jxo_prefix* p, const jxo_uintcfg* c,
                      uint32_t v) {
  uint32_t tok, nb, bits;
  jxo_hybrid(v, c, &tok, &nb, &bits);
  jxo_bw_put(w, p->len[tok], p->code[tok]);
  jxo_bw_put(w, nb, bits);
}

/* DequantMatrices [ext quant_weights.cc DequantMatrices::Decode]: all_default,
 * else one encoding per quant table in the format's table order (DCT,
 * IDENTITY, DCT2X2, DCT4X4, DCT16X16, DCT32X32, DCT16X8, DCT32X8, DCT32X16,
 * DCT64X64, DCT64X32, DCT4X8, AFV0, DCT128X128, DCT128X64, DCT256X256,
 * DCT256X128): 3-bit mode, 0 = Library (the decoder's defaults), 6 = DCT
 * (4-bit band count - 1, then per channel the bands as binary16, the first one
 * divided by 64).  The tables of the 128 / 256 px kinds a frame uses (effort
 * >= 8) are written (merge.c jxo_kind_param) -- the stream then does not
 * depend on the decoder's defaults for them; a frame without such a
 * varblock keeps all_default. */
static const int kQuantTableKind[17] = {-1, -1, -1, -1, JXO_VK_16, JXO_VK_32, JXO_VK_16X8, -1,
                                        JXO_VK_32X16, JXO_VK_64, JXO_VK_64X32, -1, -1,
                                        JXO_VK_128, JXO_VK_128X64, JXO_VK_256, JXO_VK_256X128};
/* mask: bit k - JXO_VK_128X64 set when the frame holds a varblock of kind k */
static uint32_t big_kind_mask(const uint8_t* acs, size_t nb) {
  uint32_t m = 0;
  for (size_t i = 0; i < nb; i++) {
    const int t = acs[i];
    if (t >= 21 && t <= 26) m |= 1u << (jxo_shapes[jxo_shape_of(t)].kind - JXO_VK_128X64);
  }
  return m;
}
static void put_dequant_matrices(jxo_bw* w, uint32_t mask) {
  if (!mask) {
    jxo_bw_put(w, 1, 1); /* all_default */
    return;
  }
  jxo_bw_put(w, 1, 0);
  for (int t = 0; t < 17; t++) {
    const int k = kQuantTableKind[t];
    if (k < JXO_VK_128X64 || !(mask >> (k - JXO_VK_128X64) & 1)) {
      jxo_bw_put(w, 3, 0); /* Library */
      continue;
    }
    const int nb = jxo_kind_num_bands(k);
    jxo_bw_put(w, 3, 6); /* DCT */
    jxo_bw_put(w, 4, (uint32_t)(nb - 1));
    for (int c = 0; c < 3; c++)
      for (int i = 0; i < nb; i++) {
        const double v = jxo_kind_param(k, c, i);
        jxo_bw_put(w, 16, jxo_f16_bits(i ? v : v / 64.0));
      }
  }
}

/* Entropy-code header (DecodeHistograms): lz77 off, context map, prefix
 * codes.  ctxmap[nctx] holds dense histogram ids. */
static void put_histograms(jxo_bw* w, int nctx, const uint8_t* ctxmap, int nhist,
                           const jxo_prefix* codes, const jxo_uintcfg* cfg);

static void put_context_map(jxo_bw* w, int nctx, const uint8_t* map, int nhist) {
  if (nhist == 1) {
    jxo_bw_put(w, 1, 1);
    jxo_bw_put(w, 2, 0);
    return;
  }
  if (nhist <= 8 && nctx <= 16) {
    uint32_t bits = ceil_log2((uint32_t)nhist);
    jxo_bw_put(w, 1, 1);
    jxo_bw_put(w, 2, bits);
    for (int i = 0; i < nctx; i++) jxo_bw_put(w, bits, map[i]);
    return;
  }
  jxo_bw_put(w, 1, 0); /* is_simple */
  jxo_bw_put(w, 1, 0); /* use_mtf */
  uint32_t counts[256] = {0};
  for (int i = 0; i < nctx; i++) counts[map[i]]++;
  jxo_prefix p;
  jxo_build_prefix(counts, 256, &p);
  uint8_t one = 0;
  put_histograms(w, 1, &one, 1, &p, &kCfgMap);
  for (int i = 0; i < nctx; i++) put_token(w, &p, &kCfgMap, map[i]);
}

static void put_histograms(jxo_bw* w, int nctx, const uint8_t* ctxmap, int nhist,
                           const jxo_prefix* codes, const jxo_uintcfg* cfg) {
  jxo_bw_put(w, 1, 0); /* lz77.enabled */
  if (nctx > 1) put_context_map(w, nctx, ctxmap, nhist);
  jxo_bw_put(w, 1, 1); /* use_prefix_code */
  for (int h = 0; h < nhist; h++) put_uintcfg(w, cfg);
  for (int h = 0; h < nhist; h++) put_varlen16(w, codes[h].alphabet - 1);
  for (int h = 0; h < nhist; h++) jxo_write_prefix(w, &codes[h]);
}

/* --------------------- modular streams (LF group) --------------------- */
typedef struct {
  int prop, splitval, lchild, rchild, predictor, leaf; /* prop<0 => leaf */
  int offset;                                         /* leaf: value offset */
} tnode;
/* DC tree: split on channel -> 3 leaves (Y, B, X), clamped gradient */
static const tnode kDcTree[5] = {{0, 0, 1, 2, 0, -1},  {0, 1, 3, 4, 0, -1},
                                 {-1, 0, 0, 0, 5, 0}, {-1, 0, 0, 0, 5, 1},
                                 {-1, 0, 0, 0, 5, 2}};
/* AC-metadata tree: cmap | epf | acs row (zero) | qf row (west) */
static const tnode kMetaTree[7] = {{0, 1, 1, 2, 0, -1}, {0, 2, 3, 4, 0, -1},
                                   {-1, 0, 0, 0, 0, 0}, {-1, 0, 0, 0, 0, 1},
                                   {2, 0, 5, 6, 0, -1}, {-1, 0, 0, 0, 1, 2},
                                   {-1, 0, 0, 0, 0, 3}};

static void put_tree(jxo_bw* w, const tnode* t, int n) {
  /* tokens: (ctx, value) in BFS order; one histogram for the 6 contexts */
  uint32_t tv[64][2];
  int nt = 0;
  for (int i = 0; i < n; i++) {
    if (t[i].prop < 0) {
      tv[nt][0] = 1; tv[nt++][1] = 0;
      tv[nt][0] = 2; tv[nt++][1] = (uint32_t)t[i].predictor;
      tv[nt][0] = 3; tv[nt++][1] = pack_signed(t[i].offset);
      tv[nt][0] = 4; tv[nt++][1] = 0;
      tv[nt][0] = 5; tv[nt++][1] = 0;
    } else {
      tv[nt][0] = 1; tv[nt++][1] = (uint32_t)t[i].prop + 1;
      tv[nt][0] = 0; tv[nt++][1] = pack_signed(t[i].splitval);
    }
  }
  uint32_t counts[JXO_ALPHA] = {0};
  for (int i = 0; i < nt; i++) {
    uint32_t tok, nb, bits;
    jxo_hybrid(tv[i][1], &kCfg, &tok, &nb, &bits);
    counts[tok]++;
  }
  jxo_prefix p;
  jxo_build_prefix(counts, JXO_ALPHA, &p);
  uint8_t map6[6] = {0};
  put_histograms(w, 6, map6, 1, &p, &kCfg);
  for (int i = 0; i < nt; i++) put_token(w, &p, &kCfg, tv[i][1]);
}

static int32_t predict(int pred, const int32_t* img, int wdt, int x, int y) {
  if (pred == 0) return 0;
  int32_t W = x > 0 ? img[y * wdt + x - 1] : (y > 0 ? img[(y - 1) * wdt + x] : 0);
  if (pred == 1) return W;
  int32_t N = y > 0 ? img[(y - 1) * wdt + x] : W;
  int32_t NW = (x > 0 && y > 0) ? img[(y - 1) * wdt + x - 1] : W;
  /* 5: clamped gradient */
  int32_t g = W + N - NW;
  int32_t lo = W < N ? W : N, hi = W < N ? N : W;
  return g < lo ? lo : (g > hi ? hi : g);
}

typedef struct {
  int32_t* data;
  int w, h;
} mchan;

static int tree_leaf(const tnode* t, int chan, int y) {
  int i = 0;
  while (t[i].prop >= 0) {
    int v = t[i].prop == 0 ? chan : y;
    i = v > t[i].splitval ? t[i].lchild : t[i].rchild;
  }
  return i;
}

/* GroupHeader + local tree + histograms + residual tokens */
static void put_modular(jxo_bw* w, const tnode* t, int nnodes, int nleaves,
                        const mchan* ch, int nch) {
  jxo_bw_put(w, 1, 0);  /* use_global_tree */
  jxo_bw_put(w, 1, 1);  /* wp_header.all_default */
  jxo_bw_put(w, 2, 0);  /* nb_transforms = 0 */
  put_tree(w, t, nnodes);
  uint32_t counts[8][JXO_ALPHA];
  memset(counts, 0, sizeof(counts));
  for (int pass = 0; pass < 2; pass++) {
    static _Thread_local jxo_prefix codes[8];
    if (pass == 1) {
      for (int l = 0; l < nleaves; l++) jxo_build_prefix(counts[l], JXO_ALPHA, &codes[l]);
      uint8_t map[8];
      for (int l = 0; l < nleaves; l++) map[l] = (uint8_t)l;
      put_histograms(w, nleaves, map, nleaves, codes, &kCfg);
    }
    for (int c = 0; c < nch; c++) {
      if (ch[c].w == 0 || ch[c].h == 0) continue;
      for (int y = 0; y < ch[c].h; y++) {
        const int node = tree_leaf(t, c, y);
        const int leaf = t[node].leaf;
        for (int x = 0; x < ch[c].w; x++) {
          int32_t r = ch[c].data[y * ch[c].w + x] - t[node].offset -
                      predict(t[node].predictor, ch[c].data, ch[c].w, x, y);
          uint32_t u = pack_signed(r);
          if (pass == 0) {
            uint32_t tok, nb, bits;
            jxo_hybrid(u, &kCfg, &tok, &nb, &bits);
            counts[leaf][tok]++;
          } else {
            put_token(w, &codes[leaf], &kCfg, u);
          }
        }
      }
    }
  }
}

static void lf_group_section(const jxo_frame* f, const jxo_result* r, int lg,
                             uint32_t filters, jxo_bw* w) {
  const uint32_t lgx = lg % f->lfxs, lgy = lg / f->lfxs;
  const uint32_t bx0 = lgx * 256, by0 = lgy * 256;
  const uint32_t bw = (f->bxs - bx0) < 256 ? f->bxs - bx0 : 256;
  const uint32_t bh = (f->bys - by0) < 256 ? f->bys - by0 : 256;
  const size_t nb = (size_t)f->bxs * f->bys;
  /* VarDCT DC: extra_precision, modular image (Y, X, B) */
  jxo_bw_put(w, 2, 0);
  mchan ch[4];
  static const int mc[3] = {1, 0, 2};
  for (int i = 0; i < 3; i++) {
    ch[i].w = (int)bw;
    ch[i].h = (int)bh;
    ch[i].data = (int32_t*)malloc(sizeof(int32_t) * bw * bh);
    for (uint32_t y = 0; y < bh; y++)
      for (uint32_t x = 0; x < bw; x++)
        ch[i].data[y * bw + x] = r->dc[mc[i] * nb + (size_t)(by0 + y) * f->bxs + bx0 + x];
  }
  put_modular(w, kDcTree, 5, 3, ch, 3);
  for (int i = 0; i < 3; i++) free(ch[i].data);
  /* AC metadata: count, then [ytox, ytob, acs+qf, epf]; one entry per
   * varblock, in raster order of the varblocks' top-left blocks */
  uint32_t count = 0;
  for (uint32_t y = 0; y < bh; y++)
    for (uint32_t x = 0; x < bw; x++)
      count += !(r->acs[(size_t)(by0 + y) * f->bxs + bx0 + x] & 0x80);
  jxo_bw_put(w, ceil_log2(bw * bh), count - 1);
  const int cw = (int)((bw + 7) / 8), chh = (int)((bh + 7) / 8);
  const size_t ntiles = (size_t)r->tiles_x * r->tiles_y;
  for (int i = 0; i < 2; i++) { /* the LF group's colour tiles: ytox, ytob */
    ch[i].w = cw;
    ch[i].h = chh;
    ch[i].data = (int32_t*)calloc((size_t)cw * chh, sizeof(int32_t));
    for (int ty = 0; ty < chh; ty++)
      for (int tx = 0; tx < cw; tx++)
        ch[i].data[ty * cw + tx] =
            r->cmap[i * ntiles + (size_t)(by0 / 8 + ty) * r->tiles_x + bx0 / 8 + tx];
  }
  ch[2].w = (int)count;
  ch[2].h = 2;
  ch[2].data = (int32_t*)malloc(sizeof(int32_t) * count * 2);
  uint32_t k = 0;
  for (uint32_t y = 0; y < bh; y++)
    for (uint32_t x = 0; x < bw; x++) {
      size_t b = (size_t)(by0 + y) * f->bxs + bx0 + x;
      if (r->acs[b] & 0x80) continue;
      ch[2].data[k] = r->acs[b];
      ch[2].data[count + k] = r->qf[b];
      k++;
    }
  ch[3].w = (int)bw;
  ch[3].h = (int)bh;
  ch[3].data = (int32_t*)calloc((size_t)bw * bh, sizeof(int32_t));
  /* EPF sharpness per block: a constant [ext: libjxl's encoder default,
   * unpinned], carried by the EPF leaf's offset (every residual 0) */
  tnode meta[7];
  memcpy(meta, kMetaTree, sizeof(meta));
  if ((filters & JXO_FILTER_EPF) && jxo_epf_iters(f->distance) > 0) {
    meta[3].offset = JXO_EPF_SHARPNESS;
    for (size_t i = 0; i < (size_t)bw * bh; i++) ch[3].data[i] = JXO_EPF_SHARPNESS;
  }
  put_modular(w, meta, 7, 4, ch, 4);
  for (int i = 0; i < 4; i++) free(ch[i].data);
}

/* ------------------------- AC tokenization ------------------------- */
typedef struct {
  uint16_t ctx;
  uint32_t v;
} actok;

static int nz_bucket(int n) {
  if (n >= 64) n = 64;
  return n < 8 ? n : 4 + n / 2;
}

/* tokens of one pass group in bitstream order: varblocks in raster order of
 * their top-left blocks, channels Y, X, B [ext dec_group DecodeACVarBlock].
 * A varblock covering cb = 2^lcb blocks codes cb*64 - cb coefficients
 * (natural order after the LLF); its non-zero count is predicted at its
 * top-left block and (nz + cb - 1) >> lcb is stored for every covered block;
 * the zero-density context scales nz_left and k down by cb. */
static size_t group_tokens(const jxo_frame* f, const jxo_result* r, int g,
                           actok* out, uint32_t* ntok_c) {
  const uint32_t gx = g % f->gxs, gy = g / f->gxs;
  const uint32_t bx0 = gx * 32, by0 = gy * 32;
  const uint32_t gw = (f->bxs - bx0) < 32 ? f->bxs - bx0 : 32;
  const uint32_t gh = (f->bys - by0) < 32 ? f->bys - by0 : 32;
  int32_t nzs[3][32 * 32];
  size_t n = 0;
  for (uint32_t by = 0; by < gh; by++)
    for (uint32_t bx = 0; bx < gw; bx++) {
      const size_t b = (size_t)(by0 + by) * f->bxs + bx0 + bx;
      const int type = r->acs[b];
      if (type & 0x80) continue;
      const int si = jxo_shape_of(type);
      const int cyb = si < 0 ? 1 : jxo_shapes[si].cy, cxb = si < 0 ? 1 : jxo_shapes[si].cx;
      const int cb = cyb * cxb;
      int lcb = 0;
      while ((1 << lcb) < cb) lcb++;
      const int size = cb * 64;
      const int ord = jxo_strategy_order[type];
      static const int corder[3] = {1, 0, 2};
      for (int ci = 0; ci < 3; ci++) {
        const int c = corder[ci];
#define QAT(k) r->ac[(((size_t)(by0 + by + ((k) >> 6) / cxb) * f->bxs + bx0 + bx + \
                       ((k) >> 6) % cxb) * 3 + c) * 64 + ((k) & 63)]
        int nz = 0;
        for (int k = cb; k < size; k++) nz += QAT(k) != 0;
        int pred;
        if (bx == 0)
          pred = by == 0 ? 32 : nzs[c][(by - 1) * 32 + bx];
        else if (by == 0)
          pred = nzs[c][by * 32 + bx - 1];
        else
          pred = (nzs[c][(by - 1) * 32 + bx] + nzs[c][by * 32 + bx - 1] + 1) / 2;
        for (int iy = 0; iy < cyb; iy++)
          for (int ix = 0; ix < cxb; ix++)
            nzs[c][(by + iy) * 32 + bx + ix] = (nz + cb - 1) >> lcb;
        const int bctx = jxo_default_ctx_map[(c < 2 ? c ^ 1 : 2) * JXO_NUM_ORDERS + ord];
        size_t n0 = n;
        out[n].ctx = (uint16_t)(nz_bucket(pred) * JXO_BLOCK_CTX + bctx);
        out[n++].v = (uint32_t)nz;
        const int zoff = JXO_BLOCK_CTX * JXO_NZ_BUCKETS + JXO_ZD_CTX * bctx;
        int prev = nz > size / 16 ? 0 : 1;
        int left = nz;
        for (int k = cb; k < size && left > 0; k++) {
          const int32_t v = QAT(k);
          out[n].ctx = (uint16_t)(zoff + (jxo_nnz_ctx[(left + cb - 1) >> lcb] +
                                          jxo_freq_ctx[k >> lcb]) * 2 + prev);
          out[n++].v = pack_signed(v);
          prev = v != 0;
          left -= prev;
        }
#undef QAT
        if (ntok_c) ntok_c[c] += (uint32_t)(n - n0);
      }
    }
  return n;
}

/* ------------------------- frame header ------------------------- */
static void put_size(jxo_bw* w, uint32_t v) { /* U32(BitsOffset(9,1),13,18,30) */
  uint32_t m = v - 1;
  if (m < (1u << 9)) put_u32_sel(w, 0, 9, m);
  else if (m < (1u << 13)) put_u32_sel(w, 1, 13, m);
  else if (m < (1u << 18)) put_u32_sel(w, 2, 18, m);
  else put_u32_sel(w, 3, 30, m);
}

static void put_headers(jxo_bw* w, uint32_t xs, uint32_t ys, uint32_t lf) {
  jxo_bw_put(w, 8, 0xFF);
  jxo_bw_put(w, 8, 0x0A);
  /* SizeHeader */
  if (xs % 8 == 0 && ys % 8 == 0 && xs <= 256 && ys <= 256) {
    jxo_bw_put(w, 1, 1);
    jxo_bw_put(w, 5, ys / 8 - 1);
    jxo_bw_put(w, 3, 0);
    jxo_bw_put(w, 5, xs / 8 - 1);
  } else {
    jxo_bw_put(w, 1, 0);
    put_size(w, ys);
    jxo_bw_put(w, 3, 0);
    put_size(w, xs);
  }
  jxo_bw_put(w, 1, 1); /* ImageMetadata.all_default: 8-bit sRGB, xyb_encoded */
  jxo_bw_pad(w);
  /* FrameHeader */
  jxo_bw_put(w, 1, 0);   /* all_default */
  jxo_bw_put(w, 2, 0);   /* frame_type regular */
  jxo_bw_put(w, 1, 0);   /* encoding VarDCT */
  put_u32_sel(w, 2, 8, 128 - 17); /* flags U64 = kSkipAdaptiveDCSmoothing */
  jxo_bw_put(w, 2, 0);   /* upsampling = 1 */
  jxo_bw_put(w, 3, 2);   /* x_qm_scale */
  jxo_bw_put(w, 3, 2);   /* b_qm_scale */
  jxo_bw_put(w, 2, 0);   /* num_passes = 1 */
  jxo_bw_put(w, 1, 0);   /* have_crop */
  jxo_bw_put(w, 2, 0);   /* blending mode replace */
  jxo_bw_put(w, 1, 1);   /* is_last */
  jxo_bw_put(w, 2, 0);   /* name length 0 */
  /* LoopFilter [ext loop_filter.h]: all_default = gab on + one EPF iteration */
  const uint32_t gab = lf & 1u, epf = (lf >> 1) & 3u;
  if (gab && epf == 1) {
    jxo_bw_put(w, 1, 1); /* loop_filter.all_default */
  } else {
    jxo_bw_put(w, 1, 0); /* loop_filter.all_default */
    jxo_bw_put(w, 1, gab);
    if (gab) jxo_bw_put(w, 1, 0); /* gab_custom */
    jxo_bw_put(w, 2, epf); /* epf_iters */
    if (epf) {
      jxo_bw_put(w, 1, 0); /* epf_sharp_custom (VarDCT) */
      jxo_bw_put(w, 1, 0); /* epf_weight_custom */
      jxo_bw_put(w, 1, 0); /* epf_sigma_custom */
    }
    jxo_bw_put(w, 2, 0); /* extensions */
  }
  jxo_bw_put(w, 2, 0);   /* extensions */
}

static void put_toc_entry(jxo_bw* w, uint32_t s) {
  if (s < 1024) put_u32_sel(w, 0, 10, s);
  else if (s < 17408) put_u32_sel(w, 1, 14, s - 1024);
  else if (s < 4211712) put_u32_sel(w, 2, 22, s - 17408);
  else put_u32_sel(w, 3, 30, s - 4211712);
}

/* ------------------------------ encode ------------------------------ */
int jxo_encode_rgb8(const uint8_t* rgb, uint32_t w, uint32_t h, size_t row_stride,
                    const jxo_params* p, jxo_result* out) {
  memset(out, 0, sizeof(*out));
  if (!rgb || w == 0 || h == 0 || w > (1u << 18) || h > (1u << 18)) return -1;
  if (!(p->distance > 0.0f) || p->distance > 25.0f) return -2;
  if (p->coder != 0 && p->coder != 1) return -3;
  if (p->filters & ~(JXO_FILTER_GAB | JXO_FILTER_EPF | JXO_OPT_AQ_MASKING)) return -4;
  jxo_frame f;
  jxo_frame_init(&f, w, h, p);
  const size_t plane = (size_t)f.xp * f.yp, nb = (size_t)f.bxs * f.bys;
  float* xyb = (float*)malloc(sizeof(float) * plane * 3);
  jxo_srgb8_to_xyb(rgb, w, h, row_stride, f.xp, f.yp, xyb);
  /* the masking quant field on the XYB image before the inverse Gaborish
   * (libjxl's order [ext]) */
  uint8_t* aqraw = NULL;
  if (p->filters & JXO_OPT_AQ_MASKING) {
    aqraw = (uint8_t*)malloc(nb);
    jxo_aq_masking(&f, xyb, aqraw);
  }
  if (p->filters & JXO_FILTER_GAB) jxo_gab_inverse(xyb, f.xp, f.yp);
  out->xsize = w;
  out->ysize = h;
  out->bxs = f.bxs;
  out->bys = f.bys;
  out->global_scale = f.G;
  out->quant_dc = f.qdc;
  out->acs = (uint8_t*)malloc(nb);
  out->qf = (uint8_t*)malloc(nb);
  out->dc = (int32_t*)malloc(sizeof(int32_t) * nb * 3);
  out->ac = (int32_t*)malloc(sizeof(int32_t) * nb * 192);
  out->ac_tokens = (uint32_t*)calloc((size_t)f.ngroups * 3, sizeof(uint32_t));
  if (p->proposals & 3) {
    out->homog = (float*)malloc(sizeof(float) * nb * 3);
    jxo_xyb img = {{xyb, xyb + plane, xyb + 2 * plane}, f.xp, f.yp, f.xp};
    jxo_homog_map(&img, p->distance, JXO_H1_FLOAT_ABS, out->homog, NULL);
  }
  uint8_t order[64];
  jxo_natural_order8(order);
  /* chroma from luma: one (ytox, ytob) pair per 64x64 tile, before the
   * AC-strategy search (front.c jxo_cfl_tile) */
  const uint32_t tiles_x = (f.bxs + 7) / 8, tiles_y = (f.bys + 7) / 8;
  const size_t ntiles = (size_t)tiles_x * tiles_y;
  out->tiles_x = tiles_x;
  out->tiles_y = tiles_y;
  out->cmap = (int8_t*)malloc(2 * ntiles);
#pragma omp parallel for schedule(dynamic)
  for (size_t t = 0; t < ntiles; t++)
    jxo_cfl_tile(&f, xyb, (int)(t % tiles_x), (int)(t / tiles_x), &out->cmap[t],
                 &out->cmap[ntiles + t]);
  float* ent = (float*)malloc(sizeof(float) * nb);
  int* raws = (int*)malloc(sizeof(int) * nb);
  (void)jxo_vkinds(); /* build the merge tables before any parallel region */
  /* Parallel loops (OpenMP, test/baseline speed only): every iteration
   * writes disjoint outputs, and every reduction is an integer sum, so the
   * bytes do not depend on the thread count. */
#pragma omp parallel for schedule(dynamic)
  for (uint32_t by = 0; by < f.bys; by++)
    for (uint32_t bx = 0; bx < f.bxs; bx++) {
      float px[3][64];
      for (int c = 0; c < 3; c++)
        for (int y = 0; y < 8; y++)
          for (int x = 0; x < 8; x++)
            px[c][y * 8 + x] = xyb[c * plane + (size_t)(by * 8 + y) * f.xp + bx * 8 + x];
      const size_t b = (size_t)by * f.bxs + bx;
      int32_t q[3][64], dcq[3];
      int raw;
      const size_t ti = (size_t)(by / 8) * tiles_x + bx / 8;
      float cfl[2];
      jxo_cfl_factors(out->cmap[ti], out->cmap[ntiles + ti], cfl);
      int t = jxo_front_block(&f, px, out->homog ? out->homog + 3 * b : NULL, q,
                              dcq, &raw, &ent[b], cfl, aqraw ? (int)aqraw[b] + 1 : 0);
      out->acs[b] = (uint8_t)t;
      out->qf[b] = (uint8_t)(raw - 1);
      raws[b] = raw;
      for (int c = 0; c < 3; c++) {
        out->dc[c * nb + b] = dcq[c];
        /* coefficients are kept in natural (zigzag) order */
        for (int k = 0; k < 64; k++) out->ac[(b * 3 + c) * 64 + k] = q[c][order[k]];
      }
    }
  /* ---- merge stage: 16x8 ... 64x64 varblocks (effort >= 5) ---- */
  if (p->effort >= 5) {
    const int max_s = p->effort >= 6 ? 8 : 4;
    /* effort >= 8: also levels 128 / 256 px (raw ids 21-26) */
    const uint32_t tx_n = (f.bxs + 7) / 8, ty_n = (f.bys + 7) / 8;
#pragma omp parallel for schedule(dynamic) collapse(2)
    for (uint32_t ty = 0; ty < ty_n; ty++)
      for (uint32_t tx = 0; tx < tx_n; tx++) {
        const size_t ti = (size_t)ty * tiles_x + tx;
        float cfl[2];
        jxo_cfl_factors(out->cmap[ti], out->cmap[ntiles + ti], cfl);
        jxo_merge_tile(&f, xyb, out->homog, (int)tx, (int)ty, max_s, ent, raws, out->acs, cfl);
      }
    if (p->effort >= 8)
      for (int s = 16; s <= 32; s *= 2)
        jxo_merge_big(&f, xyb, out->homog, s, ent, raws, out->acs, out->cmap, tiles_x, ntiles);
#pragma omp parallel for schedule(dynamic)
    for (uint32_t by = 0; by < f.bys; by++)
      for (uint32_t bx = 0; bx < f.bxs; bx++) {
        static _Thread_local int32_t vq[3 * 65536];
        static _Thread_local float llf[3 * JXO_LLF_DIM * JXO_LLF_DIM];
        const size_t b = (size_t)by * f.bxs + bx;
        const int si = jxo_shape_of(out->acs[b]);
        if (si < 0) continue; /* 8x8 class or covered */
        const jxo_shape* sh = &jxo_shapes[si];
        int rmax = 0;
        for (int iy = 0; iy < sh->cy; iy++)
          for (int ix = 0; ix < sh->cx; ix++) {
            const int v = raws[(by + iy) * f.bxs + bx + ix];
            rmax = v > rmax ? v : rmax;
          }
        const size_t ti = (size_t)(by / 8) * tiles_x + bx / 8;
        float cfl[2];
        jxo_cfl_factors(out->cmap[ti], out->cmap[ntiles + ti], cfl);
        jxo_varblock(&f, sh, xyb, (int)bx * 8, (int)by * 8, rmax, vq, llf, NULL, cfl);
        const int RC = 64 * sh->cy * sh->cx;
        for (int iy = 0; iy < sh->cy; iy++)
          for (int ix = 0; ix < sh->cx; ix++) {
            const size_t bi = (size_t)(by + iy) * f.bxs + bx + ix;
            const int slice = iy * sh->cx + ix;
            float dcv[3];
            int32_t dcq[3];
            for (int c = 0; c < 3; c++) {
              memcpy(out->ac + (bi * 3 + c) * 64, vq + c * RC + slice * 64, sizeof(int32_t) * 64);
              dcv[c] = jxo_llf_dc(sh, llf + c * JXO_LLF_DIM * JXO_LLF_DIM, iy, ix);
            }
            jxo_quant_dc(&f, dcv, dcq);
            for (int c = 0; c < 3; c++) out->dc[c * nb + bi] = dcq[c];
            out->qf[bi] = (uint8_t)(rmax - 1);
          }
      }
  }
  free(ent);
  free(raws);
  free(xyb);
  free(aqraw);

  /* ---- AC tokens and clustered histograms ---- */
  /* (debug: the largest count of one (static cluster, token) bin inside one
   * pass group -- what a group's LDS histogram on the GPU must hold) */
  uint32_t dbg_max_bin = 0;
  actok** gt = (actok**)malloc(sizeof(actok*) * f.ngroups);
  size_t* gn = (size_t*)malloc(sizeof(size_t) * f.ngroups);
  static uint32_t hist[JXO_MAX_CLUSTERS][JXO_ALPHA];
  memset(hist, 0, sizeof(hist));
#pragma omp parallel
  {
    static _Thread_local uint32_t lh[JXO_MAX_CLUSTERS][JXO_ALPHA];
    memset(lh, 0, sizeof(lh));
    /* one worst-case token buffer per thread, reused by its groups; each
     * group keeps an exact-size copy (510 concurrent 1.5 MB allocations per
     * 8K frame used to serialise the threads on page faults) */
    actok* scratch = (actok*)malloc(sizeof(actok) * 32 * 32 * 3 * 64);
#pragma omp for schedule(dynamic)
    for (uint32_t g = 0; g < f.ngroups; g++) {
      gn[g] = group_tokens(&f, out, (int)g, scratch, out->ac_tokens + g * 3);
      gt[g] = (actok*)malloc(sizeof(actok) * (gn[g] ? gn[g] : 1));
      memcpy(gt[g], scratch, sizeof(actok) * gn[g]);
      for (size_t i = 0; i < gn[g]; i++) {
        uint32_t tok, nbt, bits;
        jxo_hybrid(gt[g][i].v, &kCfg, &tok, &nbt, &bits);
        lh[jxo_ac_cluster(gt[g][i].ctx)][tok]++;
      }
      if (jxo_debug_group_bins) {
        uint32_t* gh = (uint32_t*)calloc(JXO_MAX_CLUSTERS * JXO_ALPHA, 4);
        uint32_t mx = 0;
        for (size_t i = 0; i < gn[g]; i++) {
          uint32_t tok, nbt, bits;
          jxo_hybrid(gt[g][i].v, &kCfg, &tok, &nbt, &bits);
          const uint32_t v = ++gh[jxo_ac_cluster(gt[g][i].ctx) * JXO_ALPHA + tok];
          mx = v > mx ? v : mx;
        }
        free(gh);
#pragma omp critical
        dbg_max_bin = mx > dbg_max_bin ? mx : dbg_max_bin;
      }
    }
    free(scratch);
#pragma omp critical
    for (int cl = 0; cl < JXO_MAX_CLUSTERS; cl++)
      for (int s = 0; s < JXO_ALPHA; s++) hist[cl][s] += lh[cl][s];
  }
  if (jxo_debug_group_bins) *jxo_debug_group_bins = dbg_max_bin;
  /* prefix codes: one histogram per static cluster.  ANS: the static
   * clusters are clustered again into <= JXO_ANS_MAX_HISTS centres
   * (jxo_ans_cluster).  Dense ids in order of first appearance over contexts. */
  int group[JXO_MAX_CLUSTERS]; /* static cluster -> histogram group (-1: empty) */
  int ngrp = 0;
  if (p->coder == 1) {
    ngrp = jxo_ans_cluster((const uint32_t(*)[JXO_ALPHA])hist, JXO_MAX_CLUSTERS, group);
  } else {
    for (int cl = 0; cl < JXO_MAX_CLUSTERS; cl++) {
      uint64_t tot = 0;
      for (int s = 0; s < JXO_ALPHA; s++) tot += hist[cl][s];
      group[cl] = tot ? ngrp++ : -1;
    }
  }
  int dense[JXO_MAX_CLUSTERS];
  for (int i = 0; i < JXO_MAX_CLUSTERS; i++) dense[i] = -1;
  int nhist = 0;
  uint8_t* ctxmap = (uint8_t*)malloc(JXO_AC_CTX);
  for (int ctx = 0; ctx < JXO_AC_CTX; ctx++) {
    const int gr = group[jxo_ac_cluster(ctx)];
    if (gr >= 0 && dense[gr] < 0) dense[gr] = nhist++;
    ctxmap[ctx] = (uint8_t)(gr < 0 ? 0 : dense[gr]);
  }
  static uint32_t dhist[JXO_MAX_CLUSTERS][JXO_ALPHA];
  memset(dhist, 0, sizeof(dhist));
  for (int cl = 0; cl < JXO_MAX_CLUSTERS; cl++)
    if (group[cl] >= 0 && dense[group[cl]] >= 0)
      for (int s = 0; s < JXO_ALPHA; s++) dhist[dense[group[cl]]][s] += hist[cl][s];
  jxo_prefix* codes = (jxo_prefix*)malloc(sizeof(jxo_prefix) * (nhist ? nhist : 1));
  jxo_ans* ans = p->coder == 1 ? (jxo_ans*)malloc(sizeof(jxo_ans) * (nhist ? nhist : 1)) : NULL;
  for (int h = 0; h < nhist; h++) {
    if (ans)
      jxo_ans_normalize(dhist[h], &ans[h]);
    else
      jxo_build_prefix(dhist[h], JXO_ALPHA, &codes[h]);
  }

  /* ---- sections ---- */
  const int nsec = (f.ngroups == 1) ? 1 : (int)(2 + f.nlf + f.ngroups);
  jxo_bw* sec = (jxo_bw*)malloc(sizeof(jxo_bw) * (2 + f.nlf + f.ngroups));
  const int nparts = (int)(2 + f.nlf + f.ngroups);
  for (int i = 0; i < nparts; i++) jxo_bw_init(&sec[i]);
  /* LfGlobal */
  {
    jxo_bw* s = &sec[0];
    jxo_bw_put(s, 1, 1); /* LfChannelDequantization.all_default */
    if (f.G <= 2048) put_u32_sel(s, 0, 11, f.G - 1);
    else if (f.G <= 4096) put_u32_sel(s, 1, 11, f.G - 2049);
    else if (f.G <= 8192) put_u32_sel(s, 2, 12, f.G - 4097);
    else put_u32_sel(s, 3, 16, f.G - 8193);
    if (f.qdc == 16) jxo_bw_put(s, 2, 0);
    else if (f.qdc <= 32) put_u32_sel(s, 1, 5, f.qdc - 1);
    else if (f.qdc <= 256) put_u32_sel(s, 2, 8, f.qdc - 1);
    else put_u32_sel(s, 3, 16, f.qdc - 1);
    jxo_bw_put(s, 1, 1); /* BlockCtxMap default */
    jxo_bw_put(s, 1, 1); /* ColorCorrelation DC all_default */
    jxo_bw_put(s, 1, 0); /* GlobalModular: no global tree; 0 channels */
  }
#pragma omp parallel for schedule(dynamic)
  for (uint32_t lg = 0; lg < f.nlf; lg++) lf_group_section(&f, out, (int)lg, p->filters, &sec[1 + lg]);
  {
    jxo_bw* s = &sec[1 + f.nlf];
    put_dequant_matrices(s, big_kind_mask(out->acs, (size_t)f.bxs * f.bys));
    jxo_bw_put(s, ceil_log2(f.ngroups), 0); /* num_hf_presets - 1 */
    put_u32_sel(s, 2, 0, 0);                /* used_orders = 0 */
    if (!ans) {
      put_histograms(s, JXO_AC_CTX, ctxmap, nhist, codes, &kCfg);
    } else {
      /* ANS: lz77 off, context map, use_prefix_code = 0, log_alpha 7 */
      jxo_bw_put(s, 1, 0);
      put_context_map(s, JXO_AC_CTX, ctxmap, nhist);
      jxo_bw_put(s, 1, 0);
      jxo_bw_put(s, 2, 7 - 5);
      for (int h = 0; h < nhist; h++) { /* uint config at log_alpha 7 */
        jxo_bw_put(s, 3, kCfg.split_exp);
        if (kCfg.split_exp != 7) {
          jxo_bw_put(s, ceil_log2(kCfg.split_exp + 1), kCfg.msb);
          jxo_bw_put(s, ceil_log2(kCfg.split_exp - kCfg.msb + 1), kCfg.lsb);
        }
      }
      for (int h = 0; h < nhist; h++) jxo_ans_write_hist(s, &ans[h]);
    }
  }
#pragma omp parallel for schedule(dynamic)
  for (uint32_t g = 0; g < f.ngroups; g++) {
    jxo_bw* s = &sec[2 + f.nlf + g];
    if (!ans) {
      for (size_t i = 0; i < gn[g]; i++)
        put_token(s, &codes[ctxmap[gt[g][i].ctx]], &kCfg, gt[g][i].v);
    } else {
      const size_t n = gn[g];
      uint8_t* th = (uint8_t*)malloc(n + 1);
      uint8_t* ts = (uint8_t*)malloc(n + 1);
      uint8_t* tn = (uint8_t*)malloc(n + 1);
      uint32_t* tb = (uint32_t*)malloc(sizeof(uint32_t) * (n + 1));
      for (size_t i = 0; i < n; i++) {
        uint32_t tok, nb, bits;
        jxo_hybrid(gt[g][i].v, &kCfg, &tok, &nb, &bits);
        th[i] = ctxmap[gt[g][i].ctx];
        ts[i] = (uint8_t)tok;
        tn[i] = (uint8_t)nb;
        tb[i] = bits;
      }
      jxo_ans_write_stream(s, ans, n, th, ts, tn, tb);
      free(th);
      free(ts);
      free(tn);
      free(tb);
    }
  }
  free(ans);

  /* ---- assemble ---- */
  jxo_bw o;
  jxo_bw_init(&o);
  put_headers(&o, w, h, jxo_lf_code(p->filters, p->distance));
  jxo_bw_put(&o, 1, 0); /* TOC not permuted */
  jxo_bw_pad(&o);
  if (nsec == 1) {
    jxo_bw all;
    jxo_bw_init(&all);
    for (int i = 0; i < nparts; i++) jxo_bw_append(&all, &sec[i]);
    put_toc_entry(&o, (uint32_t)((all.nbits + 7) / 8));
    jxo_bw_pad(&o);
    jxo_bw_pad(&all);
    jxo_bw_append(&o, &all);
    jxo_bw_free(&all);
  } else {
    for (int i = 0; i < nparts; i++) put_toc_entry(&o, (uint32_t)((sec[i].nbits + 7) / 8));
    jxo_bw_pad(&o);
    for (int i = 0; i < nparts; i++) {
      jxo_bw_pad(&sec[i]);
      jxo_bw_append(&o, &sec[i]);
    }
  }
  out->nbytes = (o.nbits + 7) / 8;
  out->bytes = (uint8_t*)malloc(out->nbytes);
  memcpy(out->bytes, o.buf, out->nbytes);
  jxo_bw_free(&o);
  for (int i = 0; i < nparts; i++) jxo_bw_free(&sec[i]);
  free(sec);
  for (uint32_t g = 0; g < f.ngroups; g++) free(gt[g]);
  free(gt);
  free(gn);
  free(ctxmap);
  free(codes);
  return 0;
}

#ifdef _OPENMP
#include <omp.h>
#endif
/* threads of the parallel loops (bench.py's cpu_baseline states the count);
 * returns the count in effect */
int jxo_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
  return omp_get_max_threads();
#else
  (void)n;
  return 1;
#endif
}

void jxo_result_free(jxo_result* r) {
  free(r->acs);
  free(r->qf);
  free(r->dc);
  free(r->ac);
  free(r->ac_tokens);
  free(r->homog);
  free(r->cmap);
  free(r->bytes);
  memset(r, 0, sizeof(*r));
}
