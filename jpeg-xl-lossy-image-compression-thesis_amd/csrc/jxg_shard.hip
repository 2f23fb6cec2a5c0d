// jxg_shard.hip -- multi-GPU group sharding: every rank owns a
// balanced contiguous raster range of pass groups, and every LF group has one
// owner rank (jxg_host.cpp shard_map: the rank holding most of its pass
// groups).  The LF-group streams need the per-block records (strategy, quant
// field, quantized DC) of all their blocks, so a rank sends the records of
// each of its groups whose LF group another rank owns -- to that rank only
// (one all_to_all over RCCL / xGMI) -- instead of all-gathering every record.
// Group record: [acs 1024 B][qf 1024 B][dc X 4 KB][dc Y 4 KB][dc B 4 KB]
// [ytox 16 B][ytob 16 B] (the chroma-from-luma factors of its 4 x 4 colour tiles).
// pack: send-buffer slot i <- group list[i]; unpack: group list[i] <- slot i.
#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

constexpr size_t kGroupRecord = 1024 * 2 + 1024 * 4 * 3 + 32;

__device__ __forceinline__ void group_record(const PackArgs& a, uint32_t g, uint8_t* rec,
                                             bool pack) {
  const int gx = (int)(g % a.gxs), gy = (int)(g / a.gxs);
  const int b = threadIdx.x, bx = gx * 32 + (b & 31), by = gy * 32 + (b >> 5);
  if (b < 16) {
    const int tx = gx * 4 + (b & 3), ty = gy * 4 + (b >> 2);
    if (tx < (int)a.tiles_x && ty < (int)a.tiles_y) {
      const size_t t = (size_t)ty * a.tiles_x + tx, nt = (size_t)a.tiles_x * a.tiles_y;
      int8_t* cr = reinterpret_cast<int8_t*>(rec + 2048 + 12288);
      if (pack) {
        cr[b] = a.cmap[t];
        cr[16 + b] = a.cmap[nt + t];
      } else {
        a.cmap[t] = cr[b];
        a.cmap[nt + t] = cr[16 + b];
      }
    }
  }
  if (bx >= (int)a.bxs || by >= (int)a.bys) return;
  const size_t nb = (size_t)a.bxs * a.bys, gb = (size_t)by * a.bxs + bx;
  int32_t* dcr = reinterpret_cast<int32_t*>(rec + 2048);
  if (pack) {
    rec[b] = a.acs[gb];
    rec[1024 + b] = a.qf[gb];
    for (int c = 0; c < 3; c++) dcr[c * 1024 + b] = a.dc[c * nb + gb];
  } else {
    a.acs[gb] = rec[b];
    a.qf[gb] = rec[1024 + b];
    for (int c = 0; c < 3; c++) a.dc[c * nb + gb] = dcr[c * 1024 + b];
  }
}

__global__ __launch_bounds__(1024) void pack_kernel(PackArgs a) {
  group_record(a, a.list[blockIdx.x], a.xbuf + blockIdx.x * kGroupRecord, true);
}
__global__ __launch_bounds__(1024) void unpack_kernel(PackArgs a) {
  group_record(a, a.list[blockIdx.x], a.xbuf + blockIdx.x * kGroupRecord, false);
}

// A rank's sections -> their codestream offsets in the node-shared host buffer
// (jxg_shard_write_host / jxg_shard_write_next), one launch instead of one
// D2H copy per run of consecutive sections (a kind-1 shard of an 8K frame has
// ~12 runs: its LF groups' sections and one per pass-group row; ~20 us of host
// time per copy call).  The buffer is page-locked host memory the device
// writes through its mapping (jxg_host_register).  Thread = one destination
// dword: a dword inside the piece is one store, a dword the piece shares with
// a neighbouring section (another rank's, written concurrently) takes byte
// stores of the piece's bytes only.
__global__ __launch_bounds__(256) void scatter_kernel(ScatterArgs a) {
  uint32_t i = 0;
  while (i + 1 < a.n && blockIdx.x >= a.p[i + 1].wg0) i++;
  const ScatterPiece P = a.p[i];
  const uint64_t lo = P.dst, hi = P.dst + P.len;
  const uint64_t w0 = (lo >> 2) + (uint64_t)(blockIdx.x - P.wg0) * 1024, w1 = (hi + 3) >> 2;
#pragma unroll
  for (int it = 0; it < 4; it++) {
    const uint64_t w = w0 + (uint64_t)it * 256 + threadIdx.x;
    if (w >= w1) break;
    const uint64_t b0 = w << 2;
    if (b0 >= lo && b0 + 4 <= hi) {
      const uint8_t* q = a.src + P.src + (b0 - lo);
      reinterpret_cast<uint32_t*>(a.dst)[w] =
          (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
    } else {
      for (uint64_t b = b0; b < b0 + 4; b++)
        if (b >= lo && b < hi) a.dst[b] = a.src[P.src + (b - lo)];
    }
  }
  __threadfence_system();
}
void launch_scatter(const ScatterArgs& a, uint32_t nwg, hipStream_t s) {
  if (a.n && nwg) hipLaunchKernelGGL(scatter_kernel, dim3(nwg), dim3(256), 0, s, a);
}

void launch_pack(const PackArgs& a, hipStream_t s) {
  if (a.n) hipLaunchKernelGGL(pack_kernel, dim3(a.n), dim3(1024), 0, s, a);
}
void launch_unpack(const PackArgs& a, hipStream_t s) {
  if (a.n) hipLaunchKernelGGL(unpack_kernel, dim3(a.n), dim3(1024), 0, s, a);
}

}  // namespace jxg
