// jxg_bitstream.cpp -- see jxg_bitstream.h.
#include "jxg_bitstream.h"

#include "../../include/jxg.h"

#include <algorithm>
#include <cstring>

namespace jxg {

void hybrid_encode(uint32_t v, const UintCfg& c, uint32_t* tok, uint32_t* nb, uint32_t* bits) {
  const uint32_t split = 1u << c.split_exp;
  if (v < split) {
    *tok = v;
    *nb = 0;
    *bits = 0;
    return;
  }
  const uint32_t n = 31u - (uint32_t)__builtin_clz(v);
  const uint32_t m = v - (1u << n);
  *tok = split + ((n - c.split_exp) << (c.msb + c.lsb)) + ((m >> (n - c.msb)) << c.lsb) +
         (v & ((1u << c.lsb) - 1));
  *nb = n - c.msb - c.lsb;
  *bits = (v >> c.lsb) & (*nb >= 32 ? 0xFFFFFFFFu : ((1u << *nb) - 1));
}

namespace {

// Huffman code lengths.  Leaves ordered by (count, symbol); two-queue merge
// that prefers the leaf queue on ties; if the deepest leaf exceeds maxlen the
// counts become (c >> 1) | 1 and the construction repeats.  Allocation-free
// (n <= 256): the leaf order is a sort of unique (count, symbol) keys.
void huffman_lengths(const uint32_t* counts_in, int n, int maxlen, uint8_t* len) {
  uint32_t counts[256];
  uint64_t key[256];
  uint64_t weight[512];
  int16_t parent[512];
  uint8_t depth[512];
  for (int i = 0; i < n; i++) counts[i] = counts_in[i];
  for (;;) {
    int k = 0;
    for (int i = 0; i < n; i++) {
      len[i] = 0;
      if (counts[i]) key[k++] = ((uint64_t)counts[i] << 16) | (uint64_t)i;
    }
    if (k == 0) return;
    if (k == 1) {
      len[key[0] & 0xFFFF] = 1;
      return;
    }
    std::sort(key, key + k);
    for (int i = 0; i < k; i++) {
      weight[i] = key[i] >> 16;
      parent[i] = -1;
    }
    int next_leaf = 0, next_node = k, end = k;
    while ((k - next_leaf) + (end - next_node) > 1) {
      int pick[2];
      for (int& p : pick) {
        if (next_leaf < k && (next_node >= end || weight[next_leaf] <= weight[next_node]))
          p = next_leaf++;
        else
          p = next_node++;
      }
      weight[end] = weight[pick[0]] + weight[pick[1]];
      parent[pick[0]] = parent[pick[1]] = (int16_t)end;
      parent[end] = -1;
      end++;
    }
    depth[end - 1] = 0;
    for (int i = end - 2; i >= 0; i--) depth[i] = (uint8_t)(depth[parent[i]] + 1);
    int deepest = 0;
    for (int i = 0; i < k; i++) {
      len[key[i] & 0xFFFF] = depth[i];
      deepest = std::max<int>(deepest, depth[i]);
    }
    if (deepest <= maxlen) return;
    for (int i = 0; i < n; i++)
      if (counts[i]) counts[i] = (counts[i] >> 1) | 1u;
  }
}

// canonical codes (shorter first, then by symbol), bit-reversed for LSB-first
void canonical(const uint8_t* len, int n, uint16_t* code) {
  int count[16] = {0};
  for (int i = 0; i < n; i++)
    if (len[i]) count[len[i]]++;
  int next[16] = {0};
  int c = 0;
  for (int b = 1; b < 16; b++) {
    c = (c + count[b - 1]) << 1;
    next[b] = c;
  }
  for (int i = 0; i < n; i++) {
    code[i] = 0;
    if (!len[i]) continue;
    const int v = next[len[i]]++;
    int r = 0;
    for (int b = 0; b < len[i]; b++) r |= ((v >> b) & 1) << (len[i] - 1 - b);
    code[i] = (uint16_t)r;
  }
}

}  // namespace

PrefixCode build_prefix_code(const uint32_t* counts, int n) {
  PrefixCode p;
  int last = -1;
  for (int i = 0; i < n; i++)
    if (counts[i]) {
      last = i;
      p.nsym++;
    }
  if (last <= 0) return p;  // alphabet 1: every symbol costs 0 bits
  p.alphabet = (uint32_t)last + 1;
  huffman_lengths(counts, last + 1, 15, p.len.data());
  if (p.nsym == 1) {
    p.len[last] = 0;
    p.simple = 1;
    p.ssyms[0] = (uint16_t)last;
    return p;
  }
  if (p.nsym <= 4) {
    std::vector<int> s;
    for (int i = 0; i <= last; i++)
      if (counts[i]) s.push_back(i);
    std::stable_sort(s.begin(), s.end(), [&](int a, int b) {
      return p.len[a] != p.len[b] ? p.len[a] < p.len[b] : a < b;
    });
    p.simple = p.nsym;
    for (int i = 0; i < p.nsym; i++) p.ssyms[i] = (uint16_t)s[i];
    if (p.nsym == 4 && p.len[s[0]] == 1) p.tree_select = 1;
  }
  canonical(p.len.data(), last + 1, p.code.data());
  return p;
}

void write_prefix_code(BitWriter& w, const PrefixCode& p) {
  if (p.alphabet <= 1) return;
  if (p.simple) {
    uint32_t max_bits = 0;
    while ((1u << max_bits) < p.alphabet) max_bits++;
    w.put(2, 1);
    w.put(2, (uint32_t)p.simple - 1);
    for (int i = 0; i < p.simple; i++) w.put(max_bits, p.ssyms[i]);
    if (p.simple == 4) w.put(1, (uint32_t)p.tree_select);
    return;
  }
  // code-length code (RFC 7932 §3.5) over the used length values 0..15
  static const uint8_t kOrder[18] = {1, 2, 3, 4, 0, 5, 17, 6, 16, 7, 8, 9, 10, 11, 12, 13, 14, 15};
  static const uint8_t kStaticCode[6] = {0, 7, 3, 2, 1, 15};
  static const uint8_t kStaticLen[6] = {2, 4, 3, 2, 2, 4};
  const int n = (int)p.alphabet;
  uint32_t hist[18] = {0};
  for (int i = 0; i < n; i++) hist[p.len[i]]++;
  uint8_t cl_len[18];
  uint16_t cl_code[18];
  huffman_lengths(hist, 18, 5, cl_len);
  canonical(cl_len, 18, cl_code);
  int used = 0;
  for (int i = 0; i < 18; i++) used += cl_len[i] != 0;
  w.put(2, 0);  // HSKIP
  int space = 32;
  for (int i = 0; i < 18 && space > 0; i++) {
    const int v = cl_len[kOrder[i]];
    w.put(kStaticLen[v], kStaticCode[v]);
    if (v) space -= 32 >> v;
  }
  if (used == 1) return;  // one code-length symbol: every length costs 0 bits
  for (int i = 0; i < n; i++) w.put(cl_len[p.len[i]], cl_code[p.len[i]]);
}

void write_token(BitWriter& w, const PrefixCode& p, const UintCfg& c, uint32_t v) {
  uint32_t tok, nb, bits;
  hybrid_encode(v, c, &tok, &nb, &bits);
  w.put(p.len[tok], p.code[tok]);
  w.put(nb, bits);
}

void write_u32_sel(BitWriter& w, uint32_t sel, uint32_t nbits, uint32_t v) {
  w.put(2, sel);
  w.put(nbits, v);
}

namespace {
void write_varlen16(BitWriter& w, uint32_t v) {
  if (v == 0) {
    w.put(1, 0);
    return;
  }
  const uint32_t n = 31u - (uint32_t)__builtin_clz(v);
  w.put(1, 1);
  w.put(4, n);
  w.put(n, v - (1u << n));
}
void write_uint_config(BitWriter& w, const UintCfg& c) {  // log_alpha_size 15
  w.put(4, c.split_exp);
  if (c.split_exp != 15) {
    w.put(ceil_log2(c.split_exp + 1), c.msb);
    w.put(ceil_log2(c.split_exp - c.msb + 1), c.lsb);
  }
}
}  // namespace

void write_context_map(BitWriter& w, const std::vector<uint8_t>& map, int nhist) {
  const int n = (int)map.size();
  if (nhist == 1) {
    w.put(1, 1);
    w.put(2, 0);
    return;
  }
  if (nhist <= 8 && n <= 16) {
    const uint32_t bits = ceil_log2((uint32_t)nhist);
    w.put(1, 1);
    w.put(2, bits);
    for (uint8_t v : map) w.put(bits, v);
    return;
  }
  w.put(1, 0);  // entropy coded
  w.put(1, 0);  // no move-to-front
  uint32_t counts[256] = {0};
  for (uint8_t v : map) counts[v]++;
  std::vector<PrefixCode> code{build_prefix_code(counts, 256)};
  write_histograms(w, std::vector<uint8_t>{0}, 1, code, kCfgMap);
  // every entry's token code + raw bits as one put (a per-rank-preset map of a
  // sharded frame has ranks x 7425 entries, written by every rank each frame)
  uint32_t len[256];
  uint64_t val[256];
  for (int v = 0; v < 256; v++) {
    if (!counts[v]) continue;
    uint32_t tok, nb, bits;
    hybrid_encode((uint32_t)v, kCfgMap, &tok, &nb, &bits);
    len[v] = code[0].len[tok] + nb;
    val[v] = (uint64_t)code[0].code[tok] | ((uint64_t)bits << code[0].len[tok]);
  }
  if (w.count_only()) {
    uint64_t nbits = 0;
    for (int v = 0; v < 256; v++)
      if (counts[v]) nbits += (uint64_t)counts[v] * len[v];
    w.skip(nbits);
    return;
  }
  uint64_t acc = 0;  // (entries gathered 64 bits at a time)
  uint32_t na = 0;
  for (uint8_t v : map) {
    const uint32_t l = len[v];
    acc |= val[v] << na;
    if (na + l >= 64) {
      w.put(64, acc);
      const uint32_t used = 64 - na;  // bits of this entry that went out
      acc = used < 64 ? val[v] >> used : 0;
      na = na + l - 64;
    } else {
      na += l;
    }
  }
  w.put(na, acc);
}

void write_histograms(BitWriter& w, const std::vector<uint8_t>& ctxmap, int nhist,
                      const std::vector<PrefixCode>& codes, const UintCfg& cfg,
                      const BitWriter* ctxmap_bits) {
  w.put(1, 0);  // lz77.enabled
  if (ctxmap.size() > 1) {
    if (ctxmap_bits)
      w.append(*ctxmap_bits);
    else
      write_context_map(w, ctxmap, nhist);
  }
  w.put(1, 1);  // use_prefix_code
  for (int h = 0; h < nhist; h++) write_uint_config(w, cfg);
  for (int h = 0; h < nhist; h++) write_varlen16(w, codes[h].alphabet - 1);
  for (int h = 0; h < nhist; h++) write_prefix_code(w, codes[h]);
}

// ---------------------------------------------------------------------------
// ANS tables [ext spec Annex C]: same algorithm as oracle/ans.c
// ---------------------------------------------------------------------------
static int logcount(uint32_t f) {
  int n = 0;
  while (f) {
    n++;
    f >>= 1;
  }
  return n;
}

// ---------------------------------------------------------------------------
// Histogram clustering for ANS [ext libjxl enc_cluster.cc
// FastClusterHistograms, restated in oracle/ans.c jxo_ans_cluster]: at most
// kAnsMaxHists farthest-point centres, every histogram joins its nearest one.
// Integer Q16 bit costs, so the choice is reproducible bit for bit.
// ---------------------------------------------------------------------------
namespace {
constexpr uint16_t kLog2Frac[256] = {
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

inline int64_t log2_q16(uint32_t v) {
  const int e = 31 - __builtin_clz(v);
  const uint32_t m = e >= 8 ? (v >> (e - 8)) & 255u : (v << (8 - e)) & 255u;
  return ((int64_t)e << 16) + kLog2Frac[m];
}

// bins [0, n) hold every non-zero count (n = 1 + last non-zero bin)
int64_t hist_cost(const uint32_t* h, uint64_t t, int n = 128) {
  if (!t) return 0;
  const int64_t lt = log2_q16((uint32_t)std::min<uint64_t>(t, 0xFFFFFFFFull));
  int64_t c = 0;
  for (int s = 0; s < n; s++)
    if (h[s]) c += (int64_t)h[s] * (lt - log2_q16(h[s]));
  return c;
}

int64_t merge_cost(const uint32_t* a, uint64_t ta, int64_t ca, int na, const uint32_t* b,
                   uint64_t tb, int64_t cb, int nb) {
  uint32_t m[128];
  const int n = std::max(na, nb);
  for (int s = 0; s < n; s++) m[s] = a[s] + b[s];
  return hist_cost(m, ta + tb, n) - ca - cb;
}
}  // namespace

int cluster_ans_histograms(const uint32_t* hist, int nh, int* assign) {
  std::vector<int64_t> cost(nh), dist(nh, 0);
  std::vector<uint64_t> tot(nh, 0);
  std::vector<uint8_t> centre(nh, 0);
  std::vector<int> len(nh, 0);  // 1 + last non-zero bin (AC tokens stay below 64)
  int first = -1;
  for (int i = 0; i < nh; i++) {
    for (int s = 0; s < 128; s++) {
      tot[i] += hist[i * 128 + s];
      if (hist[i * 128 + s]) len[i] = s + 1;
    }
    cost[i] = hist_cost(hist + i * 128, tot[i], len[i]);
    assign[i] = -1;
    if (tot[i] && (first < 0 || tot[i] > tot[first])) first = i;
  }
  if (first < 0) return 0;
  int ncl = 1;
  for (int i = 0; i < nh; i++) {
    if (!tot[i]) continue;
    assign[i] = 0;
    if (i == first)
      centre[i] = 1;
    else
      dist[i] = merge_cost(hist + i * 128, tot[i], cost[i], len[i], hist + first * 128, tot[first],
                           cost[first], len[first]);
  }
  while (ncl < kAnsMaxHists) {
    int pick = -1;
    for (int i = 0; i < nh; i++)
      if (tot[i] && !centre[i] && (pick < 0 || dist[i] > dist[pick])) pick = i;
    if (pick < 0 || dist[pick] < kAnsMinDist) break;
    const int c = ncl++;
    assign[pick] = c;
    centre[pick] = 1;
    for (int i = 0; i < nh; i++) {
      if (!tot[i] || centre[i]) continue;
      const int64_t d = merge_cost(hist + i * 128, tot[i], cost[i], len[i], hist + pick * 128,
                                   tot[pick], cost[pick], len[pick]);
      if (d < dist[i]) {
        dist[i] = d;
        assign[i] = c;
      }
    }
  }
  return ncl;
}

AnsTable build_ans_table(const uint32_t* counts, bool with_inverse) {
  constexpr int kAlpha = 128, kTab = 4096, kEntry = kTab / kAlpha;
  AnsTable t;
  uint64_t total = 0;
  int last = 0;
  for (int s = 0; s < kAlpha; s++) {
    total += counts[s];
    if (counts[s]) {
      t.nused++;
      last = s;
    }
  }
  if (t.nused <= 1) {
    t.freq[t.nused ? last : 0] = kTab;
    t.omit = t.nused ? last : 0;
  } else {
    for (int s = 0; s < kAlpha; s++) {
      if (!counts[s]) continue;
      const uint64_t f = counts[s] * (uint64_t)kTab / total;
      t.freq[s] = (uint16_t)(f < 1 ? 1 : f);
    }
    int omit = -1, best = -1;
    for (int s = 0; s < kAlpha; s++)
      if (t.freq[s] && logcount(t.freq[s]) > best) {
        best = logcount(t.freq[s]);
        omit = s;
      }
    t.omit = omit;
    t.omit_code = best;
    int rem = kTab;
    for (int s = 0; s < kAlpha; s++)
      if (s != omit) rem -= t.freq[s];
    while (rem < 1) {
      int m = -1;
      for (int s = 0; s < kAlpha; s++)
        if (s != omit && t.freq[s] > 1 && (m < 0 || t.freq[s] > t.freq[m])) m = s;
      t.freq[m]--;
      rem++;
    }
    t.freq[omit] = (uint16_t)rem;
  }
  if (!with_inverse) return t;  // (the histogram writers need the frequencies only)
  // alias table of the decoder, then its inverse
  int cutoff[kAlpha], right[kAlpha], offset[kAlpha], cut[kAlpha];
  int nz = 0, only = 0;
  for (int i = 0; i < kAlpha; i++)
    if (t.freq[i]) {
      nz++;
      only = i;
    }
  if (nz == 1) {
    for (int i = 0; i < kAlpha; i++) {
      right[i] = only;
      offset[i] = i * kEntry;
      cutoff[i] = 0;
    }
  } else {
    int under[kAlpha], over[kAlpha], nu = 0, no = 0;
    for (int i = 0; i < kAlpha; i++) {
      cut[i] = t.freq[i];
      right[i] = 0;
      offset[i] = 0;
      if (cut[i] > kEntry)
        over[no++] = i;
      else if (cut[i] < kEntry)
        under[nu++] = i;
    }
    while (no) {
      const int o = over[no - 1];
      const int u = under[--nu];
      const int by = kEntry - cut[u];
      cut[o] -= by;
      right[u] = o;
      offset[u] = cut[o];
      if (cut[o] < kEntry) {
        no--;
        under[nu++] = o;
      } else if (cut[o] == kEntry) {
        no--;
      }
    }
    for (int i = 0; i < kAlpha; i++) {
      if (cut[i] == kEntry) {
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
  for (int s = 0; s < kAlpha; s++) {
    t.cum[s] = (uint16_t)c;
    c += t.freq[s];
  }
  t.inv.assign(kTab, 0);
  for (int res = 0; res < kTab; res++) {
    const int i = res / kEntry, pos = res % kEntry;
    int sym, off;
    if (pos >= cutoff[i]) {
      sym = right[i];
      off = offset[i] + pos;
    } else {
      sym = i;
      off = pos;
    }
    t.inv[t.cum[sym] + off] = (uint16_t)res;
  }
  return t;
}

static void write_varlen8(BitWriter& w, uint32_t v) {
  if (v == 0) {
    w.put(1, 0);
    return;
  }
  uint32_t n = 0;
  while ((v >> (n + 1)) != 0) n++;
  w.put(1, 1);
  w.put(3, n);
  w.put(n, v - (1u << n));
}

void write_ans_histogram(BitWriter& w, const AnsTable& t) {
  static const uint8_t kLcBits[14] = {5, 4, 4, 4, 4, 4, 3, 3, 3, 3, 3, 6, 7, 7};
  static const uint8_t kLcCode[14] = {17, 11, 15, 3, 9, 7, 4, 2, 5, 6, 0, 33, 1, 65};
  if (t.nused <= 2) {
    int syms[2], n = 0;
    for (int s = 0; s < 128 && n < 2; s++)
      if (t.freq[s]) syms[n++] = s;
    if (n == 0) syms[n++] = 0;
    w.put(1, 1);
    w.put(1, (uint32_t)(n - 1));
    for (int i = 0; i < n; i++) write_varlen8(w, (uint32_t)syms[i]);
    if (n == 2) w.put(12, t.freq[syms[0]]);
    return;
  }
  w.put(1, 0);
  w.put(1, 0);
  w.put(3, 7);  // shift 12
  w.put(3, 5);
  int length = 0;
  for (int s = 0; s < 128; s++)
    if (t.freq[s]) length = s + 1;
  write_varlen8(w, (uint32_t)(length - 3));
  for (int s = 0; s < length; s++) {
    const int code = s == t.omit ? t.omit_code : logcount(t.freq[s]);
    w.put(kLcBits[code], kLcCode[code]);
  }
  for (int s = 0; s < length; s++) {
    if (s == t.omit || t.freq[s] == 0) continue;
    const int L = logcount(t.freq[s]) - 1;
    if (L > 0) w.put((uint32_t)L, t.freq[s] & ((1u << L) - 1));
  }
}

void write_ans_histograms(BitWriter& w, const std::vector<uint8_t>& ctxmap, int nhist,
                          const std::vector<AnsTable>& tables, const UintCfg& cfg,
                          const BitWriter* ctxmap_bits) {
  w.put(1, 0);  // lz77.enabled
  if (ctxmap.size() > 1) {
    if (ctxmap_bits)
      w.append(*ctxmap_bits);
    else
      write_context_map(w, ctxmap, nhist);
  }
  w.put(1, 0);      // use_prefix_code = 0
  w.put(2, 7 - 5);  // log_alpha 7
  for (int h = 0; h < nhist; h++) {  // uint config at log_alpha 7
    w.put(3, cfg.split_exp);
    if (cfg.split_exp != 7) {
      w.put(ceil_log2(cfg.split_exp + 1), cfg.msb);
      w.put(ceil_log2(cfg.split_exp - cfg.msb + 1), cfg.lsb);
    }
  }
  for (int h = 0; h < nhist; h++) write_ans_histogram(w, tables[h]);
}

// DC: split on channel -> leaves (Y), (B), (X); clamped gradient predictor
const TreeNode kDcTree[5] = {{0, 0, 1, 2, 0, -1},
                             {0, 1, 3, 4, 0, -1},
                             {-1, 0, 0, 0, 5, 0},
                             {-1, 0, 0, 0, 5, 1},
                             {-1, 0, 0, 0, 5, 2}};
// AC metadata: cmap (zero) | epf (zero) | qf row (west) | acs row (zero)
const TreeNode kMetaTree[7] = {{0, 1, 1, 2, 0, -1},  {0, 2, 3, 4, 0, -1},
                               {-1, 0, 0, 0, 0, 0},  {-1, 0, 0, 0, 0, 1},
                               {2, 0, 5, 6, 0, -1},  {-1, 0, 0, 0, 1, 2},
                               {-1, 0, 0, 0, 0, 3}};
// with EPF: every block's sharpness is kEpfSharpness, carried by the EPF
// leaf's offset (the residuals the GPU emits stay 0; oracle encode.c)
const TreeNode kMetaTreeEpf[7] = {{0, 1, 1, 2, 0, -1},  {0, 2, 3, 4, 0, -1},
                                  {-1, 0, 0, 0, 0, 0},  {-1, 0, 0, 0, 0, 1, kEpfSharpness},
                                  {2, 0, 5, 6, 0, -1},  {-1, 0, 0, 0, 1, 2},
                                  {-1, 0, 0, 0, 0, 3}};

void write_modular_prelude(BitWriter& w, const TreeNode* tree, int nnodes, int nleaves,
                           const std::vector<PrefixCode>& leaf_codes) {
  w.put(1, 0);  // use_global_tree
  w.put(1, 1);  // wp_header.all_default
  w.put(2, 0);  // nb_transforms = 0
  // tree tokens (context, value) breadth-first; one histogram for 6 contexts
  std::vector<std::pair<int, uint32_t>> toks;
  for (int i = 0; i < nnodes; i++) {
    const TreeNode& t = tree[i];
    if (t.prop < 0) {
      toks.push_back({1, 0});
      toks.push_back({2, (uint32_t)t.predictor});
      toks.push_back({3, t.offset >= 0 ? (uint32_t)t.offset * 2u : (uint32_t)(-t.offset) * 2u - 1u});
      toks.push_back({4, 0});
      toks.push_back({5, 0});
    } else {
      toks.push_back({1, (uint32_t)t.prop + 1});
      const int32_t sv = t.splitval;
      toks.push_back({0, sv >= 0 ? (uint32_t)sv * 2u : (uint32_t)(-sv) * 2u - 1u});
    }
  }
  uint32_t counts[128] = {0};
  for (auto& t : toks) {
    uint32_t tok, nb, bits;
    hybrid_encode(t.second, kCfg420, &tok, &nb, &bits);
    counts[tok]++;
  }
  std::vector<PrefixCode> tc{build_prefix_code(counts, 128)};
  write_histograms(w, std::vector<uint8_t>(6, 0), 1, tc, kCfg420);
  for (auto& t : toks) write_token(w, tc[0], kCfg420, t.second);
  std::vector<uint8_t> map(nleaves);
  for (int l = 0; l < nleaves; l++) map[l] = (uint8_t)l;
  write_histograms(w, map, nleaves, leaf_codes, kCfg420);
}

namespace {
void write_size(BitWriter& w, uint32_t v) {
  const uint32_t m = v - 1;
  if (m < (1u << 9))
    write_u32_sel(w, 0, 9, m);
  else if (m < (1u << 13))
    write_u32_sel(w, 1, 13, m);
  else if (m < (1u << 18))
    write_u32_sel(w, 2, 18, m);
  else
    write_u32_sel(w, 3, 30, m);
}
}  // namespace

uint32_t lf_code(uint32_t flags, float distance) {
  uint32_t c = (flags & JXG_FLAG_GABORISH) ? 1u : 0u;
  // EPF iterations by distance (cjxl --epf=-1, libjxl's thresholds 0.7 / 1.5 /
  // 4.0 as recalled [ext, unpinned]): none below d 0.7, then 1 / 2 / 3
  if (flags & JXG_FLAG_EPF)
    c |= (distance < 0.7f ? 0u : (distance < 1.5f ? 1u : (distance < 4.0f ? 2u : 3u))) << 1;
  return c;
}

void write_headers(BitWriter& w, uint32_t xs, uint32_t ys, uint32_t lf) {
  w.put(8, 0xFF);
  w.put(8, 0x0A);
  if (xs % 8 == 0 && ys % 8 == 0 && xs <= 256 && ys <= 256) {
    w.put(1, 1);
    w.put(5, ys / 8 - 1);
    w.put(3, 0);
    w.put(5, xs / 8 - 1);
  } else {
    w.put(1, 0);
    write_size(w, ys);
    w.put(3, 0);
    write_size(w, xs);
  }
  w.put(1, 1);  // ImageMetadata.all_default (8-bit sRGB, xyb_encoded)
  w.pad_to_byte();
  // FrameHeader
  w.put(1, 0);                      // all_default
  w.put(2, 0);                      // frame_type: regular
  w.put(1, 0);                      // encoding: VarDCT
  write_u32_sel(w, 2, 8, 128 - 17); // flags = kSkipAdaptiveDCSmoothing
  w.put(2, 0);                      // upsampling 1
  w.put(3, 2);                      // x_qm_scale
  w.put(3, 2);                      // b_qm_scale
  w.put(2, 0);                      // num_passes 1
  w.put(1, 0);                      // no crop
  w.put(2, 0);                      // blending: replace
  w.put(1, 1);                      // is_last
  w.put(2, 0);                      // name length 0
  // LoopFilter [ext loop_filter.h]: all_default = Gaborish + one EPF iteration
  const uint32_t gab = lf & 1u, epf = (lf >> 1) & 3u;
  if (gab && epf == 1) {
    w.put(1, 1);                    // loop filter all_default
  } else {
    w.put(1, 0);                    // loop filter not all_default
    w.put(1, gab);                  //   gab
    if (gab) w.put(1, 0);           //   gab_custom
    w.put(2, epf);                  //   epf_iters
    if (epf) {
      w.put(1, 0);                  //   epf_sharp_custom
      w.put(1, 0);                  //   epf_weight_custom
      w.put(1, 0);                  //   epf_sigma_custom
    }
    w.put(2, 0);                    //   loop filter extensions
  }
  w.put(2, 0);                      // frame extensions
}

void write_toc(BitWriter& w, const std::vector<uint32_t>& sizes) {
  w.put(1, 0);  // not permuted
  w.pad_to_byte();
  for (uint32_t s : sizes) {
    if (s < 1024)
      write_u32_sel(w, 0, 10, s);
    else if (s < 17408)
      write_u32_sel(w, 1, 14, s - 1024);
    else if (s < 4211712)
      write_u32_sel(w, 2, 22, s - 17408);
    else
      write_u32_sel(w, 3, 30, s - 4211712);
  }
  w.pad_to_byte();
}

}  // namespace jxg
