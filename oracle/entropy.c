/*
 * entropy.c -- ORACLE (test infrastructure).  Bit writer, hybrid-uint
 * tokens, Brotli-style prefix codes as used by JPEG XL entropy-coded streams
 * with use_prefix_code=1, and the AC context tables.
 * [ext] JPEG XL entropy coding (libjxl dec_ans.cc / huffman_decode.cc /
 * ac_context.h; RFC 7932 §3.4-3.5 for the prefix-code wire format); not in
 * /root/reference, parity unpinned against libjxl.
 */
#include <stdlib.h>
#include <string.h>

#include "jxo_internal.h"

/* [ext] kStrategyOrder: raw AcStrategy -> coefficient-order bucket */
const uint8_t jxo_strategy_order[27] = {0, 1, 1, 1, 2, 3, 4, 4, 5,  5,  6,  6,  1, 1,
                                        1, 1, 1, 1, 7, 8, 8, 9, 10, 10, 11, 12, 12};
/* [ext] default HF block-context map (Y row, X row, B row) */
const uint8_t jxo_default_ctx_map[39] = {
    0, 1, 2, 2, 3,  3,  4,  5,  6,  6,  6,  6,  6,   //
    7, 8, 9, 9, 10, 11, 12, 13, 14, 14, 14, 14, 14,  //
    7, 8, 9, 9, 10, 11, 12, 13, 14, 14, 14, 14, 14};
const uint8_t jxo_freq_ctx[64] = {
    0,  0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14,
    15, 15, 16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 21, 21, 22, 22,
    23, 23, 23, 23, 24, 24, 24, 24, 25, 25, 25, 25, 26, 26, 26, 26,
    27, 27, 27, 27, 28, 28, 28, 28, 29, 29, 29, 29, 30, 30, 30, 30};
const uint16_t jxo_nnz_ctx[64] = {
    0,   0,   31,  62,  62,  93,  93,  93,  93,  123, 123, 123, 123,
    152, 152, 152, 152, 152, 152, 152, 152, 180, 180, 180, 180, 180,
    180, 180, 180, 180, 180, 180, 180, 206, 206, 206, 206, 206, 206,
    206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206,
    206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206, 206};

/* Static context clustering of the 7425 AC contexts (an encoder choice; the
 * map is transmitted).  bclass: Y {DCT8, small, large}, XB {DCT8, small,
 * large}. */
static int bclass(int bctx) {
  if (bctx < 7) return bctx == 0 ? 0 : (bctx == 1 ? 1 : 2);
  return bctx == 7 ? 3 : (bctx == 8 ? 4 : 5);
}
int jxo_ac_cluster(int ctx) {
  if (ctx < JXO_BLOCK_CTX * JXO_NZ_BUCKETS) {
    int bucket = ctx / JXO_BLOCK_CTX, bctx = ctx % JXO_BLOCK_CTX;
    int nb = bucket == 0 ? 0 : (bucket <= 2 ? 1 : (bucket <= 8 ? 2 : 3));
    return bclass(bctx) * 4 + nb;
  }
  int z = ctx - JXO_BLOCK_CTX * JXO_NZ_BUCKETS;
  int bctx = z / JXO_ZD_CTX, zz = z % JXO_ZD_CTX;
  int prev = zz & 1, base = zz >> 1;
  static const int nzb_base[8] = {0, 31, 62, 93, 123, 152, 180, 206};
  int bi = 7;
  while (nzb_base[bi] > base) bi--;
  int fc = base - nzb_base[bi];
  int nzg = bi < 2 ? 0 : (bi < 4 ? 1 : 2);
  int fg = fc < 4 ? 0 : (fc < 12 ? 1 : 2);
  return 24 + ((bclass(bctx) * 3 + nzg) * 3 + fg) * 2 + prev;
}

/* ---------------- bit writer (LSB-first) ---------------- */
void jxo_bw_init(jxo_bw* w) {
  w->cap = 1024;
  w->buf = (uint8_t*)calloc(w->cap, 1);
  w->nbits = 0;
}
static void bw_reserve(jxo_bw* w, size_t bits) {
  size_t need = (w->nbits + bits + 64) / 8 + 8;
  if (need > w->cap) {
    size_t nc = w->cap * 2;
    while (nc < need) nc *= 2;
    w->buf = (uint8_t*)realloc(w->buf, nc);
    memset(w->buf + w->cap, 0, nc - w->cap);
    w->cap = nc;
  }
}
void jxo_bw_put(jxo_bw* w, uint32_t nbits, uint64_t v) {
  if (nbits == 0) return;
  bw_reserve(w, nbits);
  for (uint32_t i = 0; i < nbits; i++) {
    if ((v >> i) & 1) w->buf[(w->nbits + i) >> 3] |= (uint8_t)(1u << ((w->nbits + i) & 7));
  }
  w->nbits += nbits;
}
void jxo_bw_pad(jxo_bw* w) { w->nbits = (w->nbits + 7) & ~(size_t)7; bw_reserve(w, 0); }
void jxo_bw_append(jxo_bw* dst, const jxo_bw* src) {
  for (size_t i = 0; i < src->nbits; i += 32) {
    uint32_t n = (uint32_t)(src->nbits - i < 32 ? src->nbits - i : 32);
    uint64_t v = 0;
    for (uint32_t b = 0; b < n; b++)
      v |= (uint64_t)((src->buf[(i + b) >> 3] >> ((i + b) & 7)) & 1) << b;
    jxo_bw_put(dst, n, v);
  }
}
void jxo_bw_free(jxo_bw* w) {
  free(w->buf);
  w->buf = NULL;
  w->cap = w->nbits = 0;
}

/* ---------------- hybrid uint ---------------- */
static uint32_t floor_log2(uint32_t v) {
  uint32_t n = 0;
  while (v >> (n + 1)) n++;
  return n;
}
void jxo_hybrid(uint32_t v, const jxo_uintcfg* c, uint32_t* tok, uint32_t* nb,
                uint32_t* bits) {
  uint32_t split = 1u << c->split_exp;
  if (v < split) {
    *tok = v;
    *nb = 0;
    *bits = 0;
    return;
  }
  uint32_t n = floor_log2(v);
  uint32_t m = v - (1u << n);
  *tok = split + ((n - c->split_exp) << (c->msb + c->lsb)) +
         ((m >> (n - c->msb)) << c->lsb) + (v & ((1u << c->lsb) - 1));
  *nb = n - c->msb - c->lsb;
  *bits = (v >> c->lsb) & ((*nb >= 32) ? 0xffffffffu : ((1u << *nb) - 1));
}

/* ---------------- Huffman code lengths ----------------
 * Deterministic: leaves sorted by (count asc, symbol asc); two-queue merge,
 * ties prefer the leaf queue; if the depth exceeds maxlen, counts become
 * (c>>1)|1 and the build repeats. */
static void huff_lengths(const uint32_t* counts_in, int n, int maxlen,
                         uint8_t* len) {
  uint32_t counts[256];
  memcpy(counts, counts_in, sizeof(uint32_t) * n);
  for (;;) {
    int sym[256], k = 0;
    for (int i = 0; i < n; i++) {
      len[i] = 0;
      if (counts[i]) sym[k++] = i;
    }
    if (k == 0) return;
    if (k == 1) {
      len[sym[0]] = 1;
      return;
    }
    /* insertion sort by (count, symbol) */
    for (int i = 1; i < k; i++) {
      int s = sym[i], j = i - 1;
      while (j >= 0 && (counts[sym[j]] > counts[s] ||
                        (counts[sym[j]] == counts[s] && sym[j] > s))) {
        sym[j + 1] = sym[j];
        j--;
      }
      sym[j + 1] = s;
    }
    uint64_t w[512];
    int parent[512];
    for (int i = 0; i < k; i++) w[i] = counts[sym[i]];
    int li = 0, ii = k, in_end = k; /* leaves [li,k), internals [ii,in_end) */
    while ((k - li) + (in_end - ii) > 1) {
      int pick[2];
      for (int t = 0; t < 2; t++) {
        if (li < k && (ii >= in_end || w[li] <= w[ii]))
          pick[t] = li++;
        else
          pick[t] = ii++;
      }
      w[in_end] = w[pick[0]] + w[pick[1]];
      parent[pick[0]] = parent[pick[1]] = in_end;
      in_end++;
    }
    int root = in_end - 1;
    int depth[512];
    depth[root] = 0;
    for (int i = root - 1; i >= 0; i--) depth[i] = depth[parent[i]] + 1;
    int maxd = 0;
    for (int i = 0; i < k; i++) {
      len[sym[i]] = (uint8_t)depth[i];
      if (depth[i] > maxd) maxd = depth[i];
    }
    if (maxd <= maxlen) return;
    for (int i = 0; i < n; i++)
      if (counts[i]) counts[i] = (counts[i] >> 1) | 1u;
  }
}

static void canonical_codes(const uint8_t* len, int n, uint16_t* code) {
  int bl_count[16] = {0};
  for (int i = 0; i < n; i++) bl_count[len[i]]++;
  bl_count[0] = 0;
  int next[16];
  int c = 0;
  for (int b = 1; b < 16; b++) {
    c = (c + bl_count[b - 1]) << 1;
    next[b] = c;
  }
  for (int i = 0; i < n; i++) {
    if (!len[i]) {
      code[i] = 0;
      continue;
    }
    int v = next[len[i]]++;
    int r = 0;
    for (int b = 0; b < len[i]; b++) r |= ((v >> b) & 1) << (len[i] - 1 - b);
    code[i] = (uint16_t)r;
  }
}

void jxo_build_prefix(const uint32_t* counts, int n, jxo_prefix* p) {
  memset(p, 0, sizeof(*p));
  int last = -1, nsym = 0;
  for (int i = 0; i < n; i++)
    if (counts[i]) {
      last = i;
      nsym++;
    }
  p->nsym = nsym;
  if (last <= 0) { /* nothing or only symbol 0: alphabet 1, zero bits */
    p->alphabet = 1;
    return;
  }
  p->alphabet = (uint32_t)last + 1;
  huff_lengths(counts, last + 1, 15, p->len);
  if (nsym == 1) {
    p->len[last] = 0; /* 0-bit simple code */
    p->simple = 1;
    p->ssyms[0] = (uint16_t)last;
    return;
  }
  if (nsym <= 4) {
    int s[4], k = 0;
    for (int i = 0; i <= last; i++)
      if (counts[i]) s[k++] = i;
    /* order listed symbols: by length, then symbol (simple-code layout) */
    for (int i = 1; i < k; i++) {
      int v = s[i], j = i - 1;
      while (j >= 0 && (p->len[s[j]] > p->len[v] ||
                        (p->len[s[j]] == p->len[v] && s[j] > v))) {
        s[j + 1] = s[j];
        j--;
      }
      s[j + 1] = v;
    }
    p->simple = nsym;
    for (int i = 0; i < k; i++) p->ssyms[i] = (uint16_t)s[i];
    if (nsym == 4 && p->len[s[0]] == 1) p->tree_select = 1;
  }
  canonical_codes(p->len, last + 1, p->code);
}

/* [ext] code-length code order and the static code for code-length code
 * lengths (Brotli; LSB-first values): 0->00,1->0111,2->011,3->10,4->01,5->1111 */
static const uint8_t kCLOrder[18] = {1, 2, 3, 4, 0, 5, 17, 6, 16,
                                     7, 8, 9, 10, 11, 12, 13, 14, 15};
static const uint8_t kCLCLcode[6] = {0, 7, 3, 2, 1, 15};
static const uint8_t kCLCLlen[6] = {2, 4, 3, 2, 2, 4};

void jxo_write_prefix(jxo_bw* w, const jxo_prefix* p) {
  if (p->alphabet <= 1) return;
  if (p->simple) {
    uint32_t max_bits = 0;
    while ((1u << max_bits) < p->alphabet) max_bits++;
    /* max_bits = FloorLog2(alphabet-1)+1 */
    jxo_bw_put(w, 2, 1);
    jxo_bw_put(w, 2, (uint32_t)p->simple - 1);
    for (int i = 0; i < p->simple; i++) jxo_bw_put(w, max_bits, p->ssyms[i]);
    if (p->simple == 4) jxo_bw_put(w, 1, (uint32_t)p->tree_select);
    return;
  }
  const int n = (int)p->alphabet;
  uint32_t clc[18] = {0};
  for (int i = 0; i < n; i++) clc[p->len[i]]++;
  uint8_t cll[18];
  huff_lengths(clc, 18, 5, cll);
  int num_codes = 0;
  for (int i = 0; i < 18; i++) num_codes += cll[i] != 0;
  uint16_t clcode[18];
  canonical_codes(cll, 18, clcode);
  jxo_bw_put(w, 2, 0); /* HSKIP = 0 */
  int space = 32;
  for (int i = 0; i < 18 && space > 0; i++) {
    int v = cll[kCLOrder[i]];
    jxo_bw_put(w, kCLCLlen[v], kCLCLcode[v]);
    if (v) space -= 32 >> v;
  }
  if (num_codes == 1) {
    /* single code-length symbol: the decoder reads all 18 entries (done
     * above since space stays > 0) and every length costs 0 bits */
    return;
  }
  for (int i = 0; i < n; i++) jxo_bw_put(w, cll[p->len[i]], clcode[p->len[i]]);
}
