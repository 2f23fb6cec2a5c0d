// jxg_synth.hip -- the benchmark's deterministic synthetic RGB8 input
// (SURVEY.md §8(d) synth_rgb8: 64x64 tiles of {flat, gradients, stripes,
// checker, quadrant edge, uniform noise, smooth + noise}, splitmix64 hashes,
// integer only) generated directly in device memory, so the bench and the
// GPU tests need no host-side generation and no H2D copy (numpy needs minutes
// at 16384^2).  Bytes equal jxg/synth.py synth_rgb8 and oracle/synth.c
// (tests/test_synth.py, tests/test_gpu_configs.py).
#include "jxg_kernels.h"

namespace jxg {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// numpy floor division by a positive divisor
__device__ __forceinline__ int floordiv(int a, int b) {
  const int q = a / b;
  return (a % b != 0 && a < 0) ? q - 1 : q;
}

// one thread per pixel; the tile hash is recomputed per pixel (cheap)
__global__ __launch_bounds__(256) void synth_kernel(uint8_t* out, uint32_t w, uint32_t h,
                                                    size_t stride, uint64_t seed) {
  const uint32_t x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  const uint32_t ntx = (w + 63) / 64;
  const int lx = (int)(x & 63), ly = (int)(y & 63);
  const uint64_t th = splitmix64(seed ^ (uint64_t)((y / 64) * ntx + x / 64));
  const int kind = (int)(th % 9);
  const int period = (int)(2 + (th >> 56) % 14);
  const bool black = ((th >> 40) % 5) == 0;
  const uint64_t n64 = splitmix64((seed * 0x100000001B3ull) ^ (((uint64_t)y << 32) | x));
  uint8_t* p = out + (size_t)y * stride + 3 * (size_t)x;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const int c0 = (int)((th >> (8 + 8 * c)) & 0xFF), c1 = (int)((th >> (32 + 8 * c)) & 0xFF);
    const int noise = (int)((n64 >> (8 * c)) & 0xFF);
    const int hgrad = c0 + floordiv((c1 - c0) * lx, 63);
    const int vgrad = c0 + floordiv((c1 - c0) * ly, 63);
    int v;
    switch (kind) {
      case 0: v = black ? 0 : c0; break;
      case 1: v = hgrad; break;
      case 2: v = vgrad; break;
      case 3: v = ((ly / period) % 2 == 0) ? c0 : c1; break;
      case 4: v = ((lx / period) % 2 == 0) ? c0 : c1; break;
      case 5: v = (((lx / period + ly / period) % 2) == 0) ? c0 : c1; break;
      case 6: v = ((lx < 32) ^ (ly < 32)) ? c0 : c1; break;
      case 7: v = noise; break;
      default: v = floordiv(hgrad + vgrad, 2) + (noise % 17) - 8; break;
    }
    p[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

hipError_t launch_synth(uint8_t* out, uint32_t w, uint32_t h, size_t stride, uint64_t seed,
                        hipStream_t s) {
  if (!w || !h) return hipSuccess;
  hipLaunchKernelGGL(synth_kernel, dim3((w + 255) / 256, h), dim3(256), 0, s, out, w, h, stride,
                     seed);
  return hipGetLastError();
}

}  // namespace jxg
