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

void launch_pack(const PackArgs& a, hipStream_t s) {
  if (a.n) hipLaunchKernelGGL(pack_kernel, dim3(a.n), dim3(1024), 0, s, a);
}
void launch_unpack(const PackArgs& a, hipStream_t s) {
  if (a.n) hipLaunchKernelGGL(unpack_kernel, dim3(a.n), dim3(1024), 0, s, a);
}

}  // namespace jxg
