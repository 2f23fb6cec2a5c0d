/*
 * ans.c -- ORACLE (test infrastructure).  ANS entropy coding of the AC (HF)
 * stream: 12-bit rANS with the alias mapping of the JPEG XL decoder [ext
 * ISO/IEC 18181-1 Annex C / libjxl enc_ans.cc, dec_ans.cc; not in
 * /root/reference, restated, parity unpinned against libjxl; the test decoder
 * oracle/jxl_decode.py read_ans_histogram / alias_table is the reader].
 *
 * Restated encoder choices (deterministic; the HIP path mirrors them):
 *  - alphabet 128 (log_alpha 7); frequencies sum to 4096 and are sent at full
 *    precision (shift 12);
 *  - normalization: f = max(1, count * 4096 / total) (floor) for every used
 *    symbol; the omitted symbol is the first one with the largest log-count
 *    and takes 4096 - (sum of the others); while that is < 1 the largest
 *    other frequency (first on ties) is lowered by one;
 *  - 1 used symbol: simple histogram with one symbol; 2: simple with two
 *    (12-bit count of the first); else the general form without RLE;
 *  - state: starts at 0x130000 (the decoder's final-state check), tokens are
 *    encoded last to first; a 16-bit chunk is emitted before a token when
 *    (x >> 20) >= f; the final state is the stream's first 32 bits, then per
 *    token [chunk][hybrid-uint raw bits].
 */
#include <stdlib.h>
#include <string.h>

#include "jxo_internal.h"

#define LOG_TAB 12
#define TAB_SIZE 4096
#define ALPHA 128
#define LOG_ALPHA 7

/* log-count prefix code (symbol -> (bits, code)), == jxl_decode.LOGCOUNT_CODE */
static const uint8_t kLcBits[14] = {5, 4, 4, 4, 4, 4, 3, 3, 3, 3, 3, 6, 7, 7};
static const uint8_t kLcCode[14] = {17, 11, 15, 3, 9, 7, 4, 2, 5, 6, 0, 33, 1, 65};

static int logcount(uint32_t f) {
  int n = 0;
  while (f) {
    n++;
    f >>= 1;
  }
  return n; /* floor(log2 f) + 1, 0 for f = 0 */
}

void jxo_ans_normalize(const uint32_t* counts, jxo_ans* a) {
  memset(a, 0, sizeof(*a));
  uint64_t total = 0;
  int nused = 0, last = 0;
  for (int s = 0; s < ALPHA; s++) {
    total += counts[s];
    if (counts[s]) {
      nused++;
      last = s;
    }
  }
  a->nused = nused;
  if (nused <= 1) {
    a->freq[nused ? last : 0] = TAB_SIZE;
    a->omit = nused ? last : 0;
  } else {
    for (int s = 0; s < ALPHA; s++) {
      if (!counts[s]) continue;
      uint64_t f = counts[s] * (uint64_t)TAB_SIZE / total;
      a->freq[s] = (uint16_t)(f < 1 ? 1 : f);
    }
    int omit = -1, best = -1;
    for (int s = 0; s < ALPHA; s++)
      if (a->freq[s] && logcount(a->freq[s]) > best) {
        best = logcount(a->freq[s]);
        omit = s;
      }
    a->omit = omit;
    a->omit_code = best;
    int rem = TAB_SIZE;
    for (int s = 0; s < ALPHA; s++)
      if (s != omit) rem -= a->freq[s];
    while (rem < 1) {
      int t = -1;
      for (int s = 0; s < ALPHA; s++)
        if (s != omit && a->freq[s] > 1 && (t < 0 || a->freq[s] > a->freq[t])) t = s;
      a->freq[t]--;
      rem++;
    }
    a->freq[omit] = (uint16_t)rem;
  }
  /* alias table (== jxl_decode.alias_table), then its inverse */
  const int entry = TAB_SIZE >> LOG_ALPHA;
  int cutoff[ALPHA], right[ALPHA], offset[ALPHA], cut[ALPHA];
  int nz = 0, only = 0;
  for (int i = 0; i < ALPHA; i++)
    if (a->freq[i]) {
      nz++;
      only = i;
    }
  if (nz == 1) {
    for (int i = 0; i < ALPHA; i++) {
      right[i] = only;
      offset[i] = i * entry;
      cutoff[i] = 0;
    }
  } else {
    int under[ALPHA], over[ALPHA], nu = 0, no = 0;
    for (int i = 0; i < ALPHA; i++) {
      cut[i] = a->freq[i];
      right[i] = 0;
      offset[i] = 0;
      if (cut[i] > entry)
        over[no++] = i;
      else if (cut[i] < entry)
        under[nu++] = i;
    }
    while (no) {
      const int o = over[no - 1];
      const int u = under[--nu];
      const int by = entry - cut[u];
      cut[o] -= by;
      right[u] = o;
      offset[u] = cut[o];
      if (cut[o] < entry) {
        no--;
        under[nu++] = o;
      } else if (cut[o] == entry) {
        no--;
      }
    }
    for (int i = 0; i < ALPHA; i++) {
      if (cut[i] == entry) {
        right[i] = i;
        offset[i] = 0;
        cutoff[i] = 0;
      } else {
        offset[i] -= cut[i];
        cutoff[i] = cut[i];
      }
    }
  }
  int c = 0;
  for (int s = 0; s < ALPHA; s++) {
    a->cum[s] = (uint16_t)c;
    c += a->freq[s];
  }
  for (int res = 0; res < TAB_SIZE; res++) {
    const int i = res / entry, pos = res % entry;
    int sym, off;
    if (pos >= cutoff[i]) {
      sym = right[i];
      off = offset[i] + pos;
    } else {
      sym = i;
      off = pos;
    }
    a->inv[a->cum[sym] + off] = (uint16_t)res;
  }
}

static void put_varlen_u8(jxo_bw* w, uint32_t v) {
  if (v == 0) {
    jxo_bw_put(w, 1, 0);
    return;
  }
  uint32_t n = 0;
  while ((v >> (n + 1)) != 0) n++;
  jxo_bw_put(w, 1, 1);
  jxo_bw_put(w, 3, n);
  jxo_bw_put(w, n, v - (1u << n));
}

void jxo_ans_write_hist(jxo_bw* w, const jxo_ans* a) {
  if (a->nused <= 2) {
    int syms[2], n = 0;
    for (int s = 0; s < ALPHA && n < 2; s++)
      if (a->freq[s]) syms[n++] = s;
    if (n == 0) syms[n++] = 0;
    jxo_bw_put(w, 1, 1); /* simple */
    jxo_bw_put(w, 1, (uint32_t)(n - 1));
    for (int i = 0; i < n; i++) put_varlen_u8(w, (uint32_t)syms[i]);
    if (n == 2) jxo_bw_put(w, LOG_TAB, a->freq[syms[0]]);
    return;
  }
  jxo_bw_put(w, 1, 0); /* not simple */
  jxo_bw_put(w, 1, 0); /* not flat */
  /* shift 12: (shift + 1) = 13 = 0b1101 -> log 3 (three 1s, = upper), 3 bits of 5 */
  jxo_bw_put(w, 3, 7);
  jxo_bw_put(w, 3, 5);
  int length = 0;
  for (int s = 0; s < ALPHA; s++)
    if (a->freq[s]) length = s + 1;
  put_varlen_u8(w, (uint32_t)(length - 3));
  for (int s = 0; s < length; s++) {
    const int code = s == a->omit ? a->omit_code : logcount(a->freq[s]);
    jxo_bw_put(w, kLcBits[code], kLcCode[code]);
  }
  for (int s = 0; s < length; s++) {
    if (s == a->omit || a->freq[s] == 0) continue;
    const int L = logcount(a->freq[s]) - 1; /* full precision: bc = L */
    if (L > 0) jxo_bw_put(w, (uint32_t)L, a->freq[s] & ((1u << L) - 1));
  }
}

/* tokens (histogram, symbol, raw bits) of one stream -> w */
void jxo_ans_write_stream(jxo_bw* w, const jxo_ans* hists, size_t n, const uint8_t* hist,
                          const uint8_t* sym, const uint8_t* nbits, const uint32_t* bits) {
  uint16_t* chunk = (uint16_t*)malloc(sizeof(uint16_t) * (n ? n : 1));
  uint8_t* has = (uint8_t*)calloc(n ? n : 1, 1);
  uint32_t x = 0x130000u;
  for (size_t k = n; k-- > 0;) {
    const jxo_ans* a = &hists[hist[k]];
    const uint32_t f = a->freq[sym[k]];
    if ((x >> 20) >= f) {
      chunk[k] = (uint16_t)(x & 0xFFFF);
      has[k] = 1;
      x >>= 16;
    }
    x = ((x / f) << LOG_TAB) + a->inv[a->cum[sym[k]] + x % f];
  }
  jxo_bw_put(w, 32, x);
  for (size_t k = 0; k < n; k++) {
    if (has[k]) jxo_bw_put(w, 16, chunk[k]);
    jxo_bw_put(w, nbits[k], bits[k]);
  }
  free(chunk);
  free(has);
}

/* ------------------------------------------------------------------ */
/* Histogram clustering for the ANS-coded AC stream [ext libjxl
 * enc_cluster.cc FastClusterHistograms, restated]: farthest-point choice of
 * at most JXO_ANS_MAX_HISTS centres, then every histogram joins its nearest
 * centre.  Costs are integer Q16 bit counts (fixed-point log2 below) so the
 * HIP path's host code (jxg_bitstream.cpp cluster_histograms) reproduces the
 * choice bit for bit. */
static const uint16_t kLog2Frac[256] = {
    0, 369, 736, 1102, 1466, 1829, 2190, 2551, 2909, 3267, 3623, 3978, 4331, 4683, 5034, 5384, 5732,
    6079, 6425, 6769, 7112, 7454, 7795, 8134, 8473, 8810, 9146, 9480, 9814, 10146, 10477, 10807, 11136,
    11464, 11791, 12116, 12440, 12764, 13086, 13407, 13727, 14046, 14363, 14680, 14996, 15310, 15624,
    15937, 16248, 16559, 16868, 17177, 17484, 17791, 18096, 18401, 18704, 19007, 19308, 19609, 19909,
    20207, 20505, 20802, 21098, 21393, 21687, 21980, 22272, 22564, 22854, 23144, 23433, 23720, 24007,
    24293, 24579, 24863, 25146, 25429, 25711, 25992, 26272, 26551, 26830, 27108, 27384, 27660, 27936,
    28210, 28484, 28757, 29029, 29300, 29571, 29840, 30109, 30378, 30645, 30912, 31178, 31443, 31707,
    31971, 32234, 32496, 32758, 33019, 33279, 33538, 33797, 34055, 34312, 34569, 34825, 35080, 35334,
    35588, 35841, 36094, 36346, 36597, 36847, 37097, 37346, 37595, 37842, 38090, 38336, 38582, 38827,
    39072, 39316, 39559, 39802, 40044, 40286, 40527, 40767, 41006, 41246, 41484, 41722, 41959, 42196,
    42432, 42667, 42902, 43137, 43370, 43603, 43836, 44068, 44300, 44530, 44761, 44990, 45220, 45448,
    45676, 45904, 46131, 46357, 46583, 46809, 47034, 47258, 47482, 47705, 47928, 48150, 48372, 48593,
    48813, 49034, 49253, 49472, 49691, 49909, 50127, 50344, 50560, 50776, 50992, 51207, 51422, 51636,
    51850, 52063, 52276, 52488, 52700, 52911, 53122, 53332, 53542, 53751, 53960, 54169, 54377, 54584,
    54791, 54998, 55204, 55410, 55615, 55820, 56025, 56229, 56432, 56635, 56838, 57040, 57242, 57443,
    57644, 57845, 58045, 58245, 58444, 58643, 58841, 59039, 59237, 59434, 59631, 59827, 60023, 60219,
    60414, 60609, 60803, 60997, 61190, 61384, 61576, 61769, 61961, 62152, 62343, 62534, 62725, 62915,
    63104, 63294, 63483, 63671, 63859, 64047, 64234, 64421, 64608, 64794, 64980, 65166, 65351};

static inline int64_t log2_q16(uint32_t v) { /* v >= 1 */
  const int e = 31 - __builtin_clz(v);
  const uint32_t m = e >= 8 ? (v >> (e - 8)) & 255u : (v << (8 - e)) & 255u;
  return ((int64_t)e << 16) + kLog2Frac[m];
}

/* Q16 bits of coding h (total t) with its own ideal code */
static int64_t hist_cost(const uint32_t* h, uint64_t t) {
  if (!t) return 0;
  const int64_t lt = log2_q16((uint32_t)(t > 0xFFFFFFFFull ? 0xFFFFFFFFull : t));
  int64_t c = 0;
  for (int s = 0; s < ALPHA; s++)
    if (h[s]) c += (int64_t)h[s] * (lt - log2_q16(h[s]));
  return c;
}

static int64_t merge_cost(const uint32_t* a, uint64_t ta, int64_t ca, const uint32_t* b,
                          uint64_t tb, int64_t cb) {
  uint32_t m[ALPHA];
  for (int s = 0; s < ALPHA; s++) m[s] = a[s] + b[s];
  return hist_cost(m, ta + tb) - ca - cb;
}

int jxo_ans_cluster(const uint32_t (*hist)[ALPHA], int nh, int* assign) {
  int64_t cost[256], dist[256];
  uint64_t tot[256];
  uint8_t isc[256] = {0};
  int ncl = 0, first = -1;
  for (int i = 0; i < nh; i++) {
    tot[i] = 0;
    for (int s = 0; s < ALPHA; s++) tot[i] += hist[i][s];
    cost[i] = hist_cost(hist[i], tot[i]);
    assign[i] = -1;
    if (tot[i] && (first < 0 || tot[i] > tot[first])) first = i;
  }
  if (first < 0) return 0;
  ncl = 1;
  for (int i = 0; i < nh; i++) {
    if (!tot[i]) continue;
    if (i == first) {
      assign[i] = 0;
      isc[i] = 1;
      continue;
    }
    dist[i] = merge_cost(hist[i], tot[i], cost[i], hist[first], tot[first], cost[first]);
    assign[i] = 0;
  }
  while (ncl < JXO_ANS_MAX_HISTS) {
    int pick = -1;
    for (int i = 0; i < nh; i++)
      if (tot[i] && !isc[i] && (pick < 0 || dist[i] > dist[pick])) pick = i;
    if (pick < 0 || dist[pick] < JXO_ANS_MIN_DIST) break;
    const int c = ncl++;
    assign[pick] = c;
    isc[pick] = 1;
    for (int i = 0; i < nh; i++) {
      if (!tot[i] || isc[i]) continue;
      const int64_t d = merge_cost(hist[i], tot[i], cost[i], hist[pick], tot[pick], cost[pick]);
      if (d < dist[i]) {
        dist[i] = d;
        assign[i] = c;
      }
    }
  }
  return ncl;
}
