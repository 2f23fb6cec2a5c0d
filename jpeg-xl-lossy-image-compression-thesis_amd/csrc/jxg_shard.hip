// jxg_shard.hip -- multi-GPU group sharding: every rank owns a
// balanced contiguous raster range of pass groups.  After its front end, a
// rank packs the per-block records of its groups (strategy, quant field,
// quantized DC -- what the LF-group streams of other ranks read) into its slot
// of an exchange buffer; the caller all-gathers the buffer over RCCL (xGMI)
// and every rank unpacks the other slots into its frame arrays.
// Group record: [acs 1024 B][qf 1024 B][dc X 4 KB][dc Y 4 KB][dc B 4 KB].
#include "jxg_device.h"
#include "jxg_kernels.h"

namespace jxg {

constexpr size_t kGroupRecord = 1024 * 2 + 1024 * 4 * 3;

__host__ __device__ __forceinline__ uint32_t shard_g0(uint32_t ngroups, uint32_t r,
                                                      uint32_t world) {
  return (uint32_t)(((uint64_t)ngroups * r) / world);
}

__device__ __forceinline__ void group_record(const PackArgs& a, uint32_t g, uint8_t* rec,
                                             bool pack) {
  const int gx = (int)(g % a.gxs), gy = (int)(g / a.gxs);
  const int b = threadIdx.x, bx = gx * 32 + (b & 31), by = gy * 32 + (b >> 5);
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
  const uint32_t g = shard_g0(a.ngroups, a.rank, a.world) + blockIdx.x;
  group_record(a, g, a.xbuf + a.rank * a.slot_bytes + blockIdx.x * kGroupRecord, true);
}

__global__ __launch_bounds__(1024) void unpack_kernel(PackArgs a) {
  const uint32_t r = blockIdx.y;
  if (r == a.rank) return;
  const uint32_t g0 = shard_g0(a.ngroups, r, a.world), g1 = shard_g0(a.ngroups, r + 1, a.world);
  const uint32_t g = g0 + blockIdx.x;
  if (g >= g1) return;
  group_record(a, g, a.xbuf + r * a.slot_bytes + blockIdx.x * kGroupRecord, false);
}

void launch_pack(const PackArgs& a, hipStream_t s) {
  const uint32_t n = shard_g0(a.ngroups, a.rank + 1, a.world) - shard_g0(a.ngroups, a.rank, a.world);
  if (n) hipLaunchKernelGGL(pack_kernel, dim3(n), dim3(1024), 0, s, a);
}
void launch_unpack(const PackArgs& a, hipStream_t s) {
  const uint32_t maxg = (a.ngroups + a.world - 1) / a.world;
  hipLaunchKernelGGL(unpack_kernel, dim3(maxg, a.world), dim3(1024), 0, s, a);
}

}  // namespace jxg
