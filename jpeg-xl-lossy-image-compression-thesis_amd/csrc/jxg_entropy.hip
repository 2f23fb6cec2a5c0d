// jxg_entropy.hip -- token statistics and bit emission on gfx950.
//
// (pass-group AC kernels: jxg_ac.hip)
// LF groups (modular streams of quantized DC and AC metadata) are processed
// in chunks of <= 4096 samples of one stream per workgroup, 16 consecutive
// samples per thread: lf_hist -> (host codes) -> lf_code.
// concat  : bit-exact assembly of all sections (device scratch + host chunks)
//           into the final codestream, one word per lane.
// Token order, contexts and hybrid-uint split are those of oracle/encode.c
// (group_tokens, put_modular) -- [ext] JPEG XL AC/modular coding.
#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

// ----------------------------- LF groups -----------------------------------
struct LfGeom {
  uint32_t bx0, by0, bw, bh;
};
__device__ __forceinline__ LfGeom lf_geom(const LfArgs& a, uint32_t lg) {
  LfGeom r;
  r.bx0 = (lg % a.lfxs) * 256;
  r.by0 = (lg / a.lfxs) * 256;
  r.bw = min(256u, a.bxs - r.bx0);
  r.bh = min(256u, a.bys - r.by0);
  return r;
}

__device__ __forceinline__ int32_t lf_value(const LfArgs& a, const LfRow& r, const LfGeom& L,
                                            int x, int y) {
  const size_t nb = (size_t)a.bxs * a.bys;
  if (r.stream == 0) {
    const int c = r.chan == 0 ? 1 : (r.chan == 1 ? 0 : 2);
    return a.dc[c * nb + (size_t)(L.by0 + y) * a.bxs + L.bx0 + x];
  }
  if (r.chan < 2)  // colour tile (x, y) of the LF group
    return a.cmap[(size_t)r.chan * a.ntiles_all + (size_t)(L.by0 / 8 + y) * a.tiles_x +
                  L.bx0 / 8 + x];
  if (r.chan != 2) return 0;
  // varblock x of the LF group (raster order of first blocks)
  const size_t b = a.vb[(size_t)r.lg * 65536 + (uint32_t)x];
  return y == 0 ? (int32_t)a.acs[b] : (int32_t)a.qf[b];
}

// residual and leaf of sample (x, row.y)
__device__ __forceinline__ void lf_residual(const LfArgs& a, const LfRow& r, const LfGeom& L,
                                            int x, uint32_t& u, int& leaf) {
  const int y = (int)r.y;
  const int32_t v = lf_value(a, r, L, x, y);
  int32_t pred = 0;
  if (r.stream == 0) {
    leaf = r.chan == 0 ? 0 : (r.chan == 2 ? 1 : 2);
    const int32_t W = x > 0 ? lf_value(a, r, L, x - 1, y) : (y > 0 ? lf_value(a, r, L, x, y - 1) : 0);
    const int32_t N = y > 0 ? lf_value(a, r, L, x, y - 1) : W;
    const int32_t NW = (x > 0 && y > 0) ? lf_value(a, r, L, x - 1, y - 1) : W;
    const int32_t gr = W + N - NW;
    const int32_t lo = W < N ? W : N, hi = W < N ? N : W;
    pred = gr < lo ? lo : (gr > hi ? hi : gr);
  } else {
    if (r.chan <= 1) {
      leaf = 0;
    } else if (r.chan == 3) {
      leaf = 1;
    } else if (y > 0) {
      leaf = 2;
      pred = x > 0 ? lf_value(a, r, L, x - 1, y) : lf_value(a, r, L, x, y - 1);
    } else {
      leaf = 3;
    }
  }
  u = pack_signed(v - pred);
}

// Chunk bookkeeping in LDS: segment starts (sample index within the chunk)
struct LfChunkLds {
  LfRow row[kLfChunkRows];
  uint32_t start[kLfChunkRows + 1];
};

__device__ __forceinline__ LfChunk load_chunk(const LfArgs& a, LfChunkLds& S) {
  const LfChunk ch = a.chunks[blockIdx.x];
  if (threadIdx.x < ch.nrows) S.row[threadIdx.x] = a.rows[ch.row0 + threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < ch.nrows; i++) {
      S.start[i] = acc;
      acc += S.row[i].width;
    }
    S.start[ch.nrows] = acc;
  }
  __syncthreads();
  return ch;
}

// Visit this thread's samples [t*kLfPer, ...) of the chunk in stream order:
// f(j, u, leaf) for j = 0..cnt-1.
template <class F>
__device__ __forceinline__ void for_my_samples(const LfArgs& a, const LfChunk& ch,
                                               const LfChunkLds& S, F&& f) {
  const uint32_t first = threadIdx.x * kLfPer;
  if (first >= ch.nsamp) return;
  uint32_t seg = 0;
  while (S.start[seg + 1] <= first) seg++;
  uint32_t pos = first;
  // the row's geometry (two integer divisions) and varblock count only when
  // the thread's samples cross into the next row
  LfGeom L = lf_geom(a, S.row[seg].lg);
  uint32_t nvb = a.vcount[S.row[seg].lg];
#pragma unroll
  for (uint32_t j = 0; j < kLfPer; j++) {
    if (pos < ch.nsamp) {
      if (S.start[seg + 1] <= pos) {
        while (S.start[seg + 1] <= pos) seg++;
        L = lf_geom(a, S.row[seg].lg);
        nvb = a.vcount[S.row[seg].lg];
      }
      const LfRow& r = S.row[seg];
      const uint32_t x = r.x0 + pos - S.start[seg];
      // the strategy/quant-field channel is laid out for bw*bh entries; only
      // the first count (= varblocks) exist
      if (!(r.stream == 1 && r.chan == 2) || x < nvb) {
        uint32_t u;
        int leaf;
        lf_residual(a, r, L, (int)x, u, leaf);
        f(j, u, leaf);
      }
    }
    pos++;
  }
}

__global__ __launch_bounds__(256) void lf_hist_kernel(Batch<LfArgs> bt_) {
  const LfArgs& a = bt_.a[blockIdx.z];
  __shared__ uint32_t sHist[4 * kAlpha];
  __shared__ uint32_t sBound;
  __shared__ LfChunkLds S;
  for (int i = threadIdx.x; i < 4 * kAlpha; i += blockDim.x) sHist[i] = 0;
  if (threadIdx.x == 0) {
    sBound = 0;
    a.status[blockIdx.x] = 0;  // lf_code's look-back word of this chunk
  }
  const LfChunk ch = load_chunk(a, S);
  uint32_t bound = 0;
  for_my_samples(a, ch, S, [&](uint32_t, uint32_t u, int leaf) {
    uint32_t tok, nb, bits;
    hybrid420(u, tok, nb, bits);
    atomicAdd(&sHist[leaf * kAlpha + tok], 1u);
    bound += 15u + nb;
  });
  atomicAdd(&sBound, bound);
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * kAlpha; i += blockDim.x)
    if (sHist[i]) atomicAdd(&a.hist[(size_t)ch.sid * 4 * kAlpha + i], sHist[i]);
  if (threadIdx.x == 0) atomicAdd(&a.sbound[ch.sid], sBound);
}

// workgroup exclusive scan of one value per thread (256 threads); sWave
// holds the four wave totals afterwards
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* sWave) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d);
    if (lane >= d) incl += t;
  }
  if (lane == 63) sWave[wv] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (int i = 0; i < wv; i++) before += sWave[i];
  return before + incl - v;
}

// One launch codes the LF streams (chunk = workgroup; a stream's chunks are
// consecutive workgroups in stream order): every thread codes its samples,
// a workgroup scan places them in the chunk, a decoupled look-back over the
// stream's earlier chunks gives the chunk's offset (status word per chunk:
// aggregate, then inclusive prefix; a chunk only waits on lower-indexed,
// already dispatched workgroups, and the stream's first chunk publishes its
// prefix at once), the chunk's bits are assembled in LDS at the word
// alignment of that offset and stored as whole words.  The two words a chunk
// shares with its neighbours are merged with an AND then an OR over the
// chunk's own bits only (disjoint masks commute), so the arena needs no zero
// fill; the concat kernel masks the bits past a stream's end.  Replaces the
// lf_bits -> lf_scan -> lf_emit launches (the samples were coded twice).
constexpr uint64_t kLfAgg = 1ull << 62, kLfPre = 2ull << 62, kLfVal = (1ull << 62) - 1;
constexpr uint32_t kLfImgWords = (kLfPer * 256 * 31 + 31) / 32 + 2;  // 31 bits per sample at most
__device__ __forceinline__ uint64_t lf_status_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lf_status_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ __launch_bounds__(256) void lf_code_kernel(Batch<LfArgs> bt_) {
  const LfArgs& a = bt_.a[blockIdx.z];
  __shared__ LfChunkLds S;
  __shared__ uint32_t sWave[4];
  __shared__ uint32_t sImg[kLfImgWords];
  __shared__ uint64_t sExcl;
  for (uint32_t i = threadIdx.x; i < kLfImgWords; i += 256) sImg[i] = 0;
  const LfChunk ch = load_chunk(a, S);  // (barriers: sImg is clear after it)
  uint32_t val[kLfPer], len[kLfPer];
  uint32_t tot = 0;
#pragma unroll
  for (uint32_t j = 0; j < kLfPer; j++) len[j] = 0;
  for_my_samples(a, ch, S, [&](uint32_t j, uint32_t u, int leaf) {
    uint32_t tok, nb, bits;
    hybrid420(u, tok, nb, bits);
    const uint32_t cl = a.codes[((size_t)ch.sid * 4 + leaf) * kAlpha + tok];
    // prefix code (<= 15 bits) then raw bits (<= 16): at most 31 bits
    val[j] = (cl & 0xFFFFu) | (bits << (cl >> 16));
    len[j] = (cl >> 16) + nb;
    tot += len[j];
  });
  const uint32_t off = block_excl_scan256(tot, sWave);
  const uint32_t total = sWave[0] + sWave[1] + sWave[2] + sWave[3];
  if (threadIdx.x == 0) {
    const uint32_t r = blockIdx.x, c0 = a.stream_chunks[ch.sid];
    uint64_t excl = 0;
    if (r == c0) {
      lf_status_store(&a.status[r], kLfPre | total);
    } else {
      lf_status_store(&a.status[r], kLfAgg | total);
      for (uint32_t q = r - 1;;) {
        const uint64_t v = lf_status_load(&a.status[q]);
        if (!(v >> 62)) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        excl += v & kLfVal;
        if ((v & kLfPre) || q == c0) break;
        q--;
      }
      lf_status_store(&a.status[r], kLfPre | (excl + total));
    }
    sExcl = excl;
    if (r + 1 == a.stream_chunks[ch.sid + 1]) a.stream_bits[ch.sid] = (uint32_t)(excl + total);
  }
  __syncthreads();
  const uint64_t start = a.stream_base[ch.sid] + sExcl;  // absolute bit of the chunk
  const uint32_t sh = (uint32_t)(start & 31);
  // this thread's codes into the LDS image (bit 0 = the start word's bit 0)
  uint32_t pos = sh + off;
#pragma unroll
  for (uint32_t j = 0; j < kLfPer; j++) {
    if (len[j]) {
      const uint32_t w = pos >> 5, b = pos & 31;
      atomicOr(&sImg[w], val[j] << b);
      if (b + len[j] > 32) atomicOr(&sImg[w + 1], val[j] >> (32 - b));
      pos += len[j];
    }
  }
  __syncthreads();
  const uint64_t w0 = start >> 5;
  const uint32_t end = sh + total, nw = (end + 31) >> 5;
  for (uint32_t i = threadIdx.x; i < nw; i += 256) {
    const uint32_t lo = i == 0 ? sh : 0, hi = min(32u, end - 32 * i);
    const uint32_t word = sImg[i];
    if (lo == 0 && hi == 32) {
      a.scratch[w0 + i] = word;
    } else {  // shared with a neighbouring chunk: only this chunk's bits
      const uint32_t m = (hi == 32 ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
      atomicAnd(&a.scratch[w0 + i], ~m);
      atomicOr(&a.scratch[w0 + i], word & m);
    }
  }
}

// ------------------------------- concat ------------------------------------
__device__ __forceinline__ uint32_t read_bits32(const uint32_t* src, uint64_t bit) {
  const uint64_t w = bit >> 5;
  const int sh = (int)(bit & 31);
  uint32_t lo = src[w] >> sh;
  if (sh) lo |= src[w + 1] << (32 - sh);
  return lo;
}

// One thread per output word: the word's bits from the pieces that overlap
// it (pieces are sorted by destination and disjoint), one plain store -- so
// the output needs no zero fill.  The workgroup's first piece is found once
// (binary search by thread 0); each thread walks on from it.
constexpr int kConcatThreads = 256;
__global__ __launch_bounds__(kConcatThreads) void concat_kernel(const ConcatPiece* pieces,
                                                                uint32_t npieces,
                                                                const uint32_t* scratch,
                                                                const uint32_t* chunks,
                                                                const uint32_t* scratch2,
                                                                uint32_t* out, uint64_t out_words) {
  __shared__ uint32_t sFirst;
  const uint64_t w0 = (uint64_t)blockIdx.x * kConcatThreads;
  if (threadIdx.x == 0) {
    // first piece ending after the workgroup's first bit
    uint32_t lo = 0, hi = npieces;
    const uint64_t bit0 = w0 * 32;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pieces[mid].dst_bit + pieces[mid].nbits <= bit0) lo = mid + 1;
      else hi = mid;
    }
    sFirst = lo;
  }
  __syncthreads();
  const uint64_t w = w0 + threadIdx.x;
  if (w >= out_words) return;
  const uint64_t b0 = w * 32, b1 = b0 + 32;
  uint32_t v = 0;
  for (uint32_t i = sFirst; i < npieces; i++) {
    const ConcatPiece p = pieces[i];
    if (p.dst_bit >= b1) break;
    if (p.dst_bit + p.nbits <= b0) continue;
    const uint64_t s0 = p.dst_bit > b0 ? p.dst_bit : b0;
    const uint64_t e0 = p.dst_bit + p.nbits < b1 ? p.dst_bit + p.nbits : b1;
    const uint32_t* src = p.arena == 1 ? chunks : (p.arena == 2 ? scratch2 : scratch);
    uint32_t x = read_bits32(src, p.src_bit + (s0 - p.dst_bit));
    const uint32_t nb = (uint32_t)(e0 - s0);
    if (nb < 32) x &= (1u << nb) - 1u;
    v |= x << (uint32_t)(s0 - b0);
  }
  out[w] = v;
}

// ------------------------------- launchers ---------------------------------
void launch_lf_hist(const LfArgs* a, uint32_t k, uint32_t nchunks, hipStream_t s) {
  if (k && nchunks) hipLaunchKernelGGL(lf_hist_kernel, dim3(nchunks, 1, k), dim3(256), 0, s, make_batch(a, k));
}
// (a frame's chunks are consecutive workgroups of its z slice: the look-back
// only waits on lower-indexed workgroups)
void launch_lf_code(const LfArgs* a, uint32_t k, uint32_t nchunks, hipStream_t s) {
  if (k && nchunks) hipLaunchKernelGGL(lf_code_kernel, dim3(nchunks, 1, k), dim3(256), 0, s, make_batch(a, k));
}
void launch_concat(const ConcatPiece* pieces, uint32_t npieces, uint64_t out_words,
                   const uint32_t* scratch, const uint32_t* chunks, const uint32_t* scratch2,
                   uint32_t* out, hipStream_t s) {
  if (out_words == 0) return;
  const uint32_t gx = (uint32_t)((out_words + kConcatThreads - 1) / kConcatThreads);
  hipLaunchKernelGGL(concat_kernel, dim3(gx), dim3(kConcatThreads), 0, s, pieces, npieces,
                     scratch, chunks, scratch2, out, out_words);
}


}  // namespace jxg
