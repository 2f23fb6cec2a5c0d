// Calibration of rocprofv3's FETCH_SIZE for the load widths the front kernel
// uses: each kernel reads a known number of bytes from
// its own 1 GiB buffer (past the 256 MiB Infinity Cache, so every byte comes
// from HBM once) and writes one word per thread (so the loads stay).
//   dword3   lane = 12 consecutive bytes, three dword loads (load_xyb_tile's
//            4-pixel chunks of RGB8, 12 B per lane, lanes consecutive)
//   ubyte3   lane = one pixel, three byte loads (the ring / AQ region loads)
//   dwordx4  lane = 16 consecutive bytes, one 16-byte load (the guide's
//            calibrated case: FETCH_SIZE = half the bytes)
// Run: rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./tools/ubench_fetch
// and compare each kernel's FETCH_SIZE (KiB) with the bytes printed here.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ __launch_bounds__(256) void k_dword3(const uint32_t* __restrict__ p, size_t nlanes,
                                                uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < nlanes; i += (size_t)gridDim.x * 256) {
    const uint32_t* q = p + 3 * i;
    acc += q[0] ^ (q[1] << 1) ^ (q[2] << 2);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
__global__ __launch_bounds__(256) void k_ubyte3(const uint8_t* __restrict__ p, size_t npx,
                                                uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < npx; i += (size_t)gridDim.x * 256) {
    const uint8_t* q = p + 3 * i;
    acc += q[0] + 3u * q[1] + 7u * q[2];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
__global__ __launch_bounds__(256) void k_dwordx4(const uint4* __restrict__ p, size_t nlanes,
                                                 uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < nlanes; i += (size_t)gridDim.x * 256) {
    const uint4 v = p[i];
    acc += v.x ^ (v.y << 1) ^ (v.z << 2) ^ (v.w << 3);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const size_t bytes = 3ull << 28;  // 768 MiB per kernel, a multiple of 12 and 16
  const int nwg = 4096;
  uint8_t *a, *b, *c;
  uint32_t* out;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&c, bytes));
  CK(hipMalloc(&out, (size_t)nwg * 256 * 4));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 2, bytes));
  CK(hipMemset(c, 3, bytes));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k_dword3, dim3(nwg), dim3(256), 0, 0, (const uint32_t*)a, bytes / 12, out);
  hipLaunchKernelGGL(k_ubyte3, dim3(nwg), dim3(256), 0, 0, (const uint8_t*)b, bytes / 3, out);
  hipLaunchKernelGGL(k_dwordx4, dim3(nwg), dim3(256), 0, 0, (const uint4*)c, bytes / 16, out);
  CK(hipDeviceSynchronize());
  std::printf("bytes read per kernel: %zu (%.1f KiB)\n", bytes, bytes / 1024.0);
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(c));
  CK(hipFree(out));
  return 0;
}
