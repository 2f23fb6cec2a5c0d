// Microbenchmark (development tool, not part of the encoder): dependent-chain
// latency of the instruction kinds an rANS encoder step can be built from, one
// wave, s_memtime around N dependent steps.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_ans.hip -o tools/ubench_ans
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N 4096
#define KERNEL(name, init, body)                                              \
  __global__ void name(uint32_t* out, uint32_t seed) {                        \
    __shared__ uint16_t tab[65536];                                           \
    for (int i = threadIdx.x; i < 65536; i += 64) tab[i] = (i * 2654435761u) >> 20; \
    __syncthreads();                                                          \
    const uint32_t lane = threadIdx.x;                                        \
    (void)lane;                                                               \
    init;                                                                     \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                               \
    for (int i = 0; i < N; i++) {                                             \
      body;                                                                   \
    }                                                                         \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                               \
    if (threadIdx.x == 0) {                                                   \
      out[0] = (uint32_t)x;                                                   \
      out[1] = (uint32_t)(t1 - t0);                                           \
    }                                                                         \
    if (x == 0x12345678u) out[2] = 1;                                         \
  }

KERNEL(k_add, uint32_t x = seed + lane, x = x + 7u; asm volatile("" : "+v"(x)))
KERNEL(k_mulhi, uint32_t x = seed + lane, x = __umulhi(x, 0x9E3779B9u); asm volatile("" : "+v"(x)))
KERNEL(k_mad24, uint32_t x = seed + lane,
       asm volatile("v_mad_i32_i24 %0, %0, %1, %0" : "+v"(x) : "v"(-7)))
KERNEL(k_cvt64, uint32_t x = seed + lane,
       double d = (double)x; asm volatile("" : "+v"(d)); x = (uint32_t)d + 1u;
       asm volatile("" : "+v"(x)))
KERNEL(k_fma64, double d = seed + lane; uint32_t x = 0,
       d = __builtin_fma(d, 0.999, 1.0); asm volatile("" : "+v"(d)); x = (uint32_t)(d > 5e9))
KERNEL(k_cvt32, uint32_t x = seed + lane,
       float f = (float)x; asm volatile("" : "+v"(f)); x = (uint32_t)f + 1u;
       asm volatile("" : "+v"(x)))
KERNEL(k_fma32, float fx = seed + lane; uint32_t x = 0,
       fx = __builtin_fmaf(fx, 0.999f, 1.0f); asm volatile("" : "+v"(fx)); x = (uint32_t)(fx > 5e9f))
KERNEL(k_dpp, uint32_t x = seed + lane,
       x = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x13C, 0xF, 0xF, false);
       asm volatile("" : "+v"(x)))
KERNEL(k_lds_uni, uint32_t x = seed, x = tab[x & 0xFFFF] + x; asm volatile("" : "+v"(x)))
KERNEL(k_lds_div, uint32_t x = seed + lane * 977u,
       x = tab[x & 0xFFFF] + x; asm volatile("" : "+v"(x)))
KERNEL(k_lds_div_dpp, uint32_t x = seed + lane * 977u,
       x = tab[x & 0xFFFF] + x;
       x = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x13C, 0xF, 0xF, false);
       asm volatile("" : "+v"(x)))
KERNEL(k_readlane, uint32_t x = seed + lane,
       x = __builtin_amdgcn_readlane(x, 5) + lane; asm volatile("" : "+v"(x)))

typedef void (*kfn)(uint32_t*, uint32_t);
int main() {
  uint32_t* d;
  if (hipMalloc(&d, 64) != hipSuccess) return 1;
  uint32_t h[2];
  struct {
    const char* name;
    kfn f;
  } ks[] = {{"v_add_u32 (+asm barrier)", k_add},
            {"v_mul_hi_u32", k_mulhi},
            {"v_mad_i32_i24", k_mad24},
            {"cvt_f64_u32 + cvt_u32_f64 + add", k_cvt64},
            {"v_fma_f64 (+cmp off-chain)", k_fma64},
            {"cvt_f32_u32 + cvt_u32_f32 + add", k_cvt32},
            {"v_fma_f32", k_fma32},
            {"v_mov_dpp wave_ror:1", k_dpp},
            {"ds_read_u16 uniform + add", k_lds_uni},
            {"ds_read_u16 64 addresses + add", k_lds_div},
            {"ds_read_u16 64 addr + add + dpp", k_lds_div_dpp},
            {"v_readlane + add (VALU reads sgpr)", k_readlane}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; rep++) {
      hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, d, 12345u);
      if (hipMemcpy(h, d, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    }
    printf("%-40s %8.1f ticks/step\n", k.name, (double)h[1] / N);
  }
  return 0;
}
