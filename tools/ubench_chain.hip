// Microbenchmark (development tool, not part of the encoder): cycles per
// step of dependent single-wave chains of the instruction kinds the ANS
// state recurrence uses.  One wave, s_memtime around 4096 dependent steps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N 4096

__global__ void k_salu(uint32_t* out, uint32_t seed) {
  uint32_t x = __builtin_amdgcn_readfirstlane(seed + threadIdx.x);
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    x = x * 3u + 7u;  // s_mul_i32 + s_add
    asm volatile("" : "+s"(x));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = x; out[1] = (uint32_t)(t1 - t0); }
}
__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
  uint32_t x = __builtin_amdgcn_readfirstlane(seed + threadIdx.x);
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    x = __umulhi(x, 0x9E3779B9u) + 12345u;
    asm volatile("" : "+s"(x));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = x; out[1] = (uint32_t)(t1 - t0); }
}
// SALU -> VALU (compare, ballot) -> SALU (bcnt)
__global__ void k_ballot(uint32_t* out, uint32_t seed) {
  uint32_t x = __builtin_amdgcn_readfirstlane(seed);
  const uint32_t v = threadIdx.x * 1000u;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    x = (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(v <= (x & 0xFFFF))) + x * 5u;
    asm volatile("" : "+s"(x));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = x; out[1] = (uint32_t)(t1 - t0); }
}
// SALU index -> v_readlane -> SALU
__global__ void k_readlane(uint32_t* out, uint32_t seed) {
  uint32_t x = __builtin_amdgcn_readfirstlane(seed);
  const uint32_t v = threadIdx.x * 2654435761u;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    x = __builtin_amdgcn_readlane(v, x & 63) + x;
    asm volatile("" : "+s"(x));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = x; out[1] = (uint32_t)(t1 - t0); }
}
// uniform LDS lookup chain: SALU address -> ds_read -> readfirstlane
__global__ void k_lds(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t tab[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) tab[i] = (i * 2654435761u) >> 3;
  __syncthreads();
  uint32_t x = __builtin_amdgcn_readfirstlane(seed);
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    x = __builtin_amdgcn_readfirstlane(tab[x & 4095]) + x;
    asm volatile("" : "+s"(x));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = x; out[1] = (uint32_t)(t1 - t0); }
}
// VALU-only uniform chain with an LDS lookup (x in a VGPR)
__global__ void k_vlds(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t tab[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) tab[i] = (i * 2654435761u) >> 3;
  __syncthreads();
  uint32_t x = seed;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    x = tab[x & 4095] + x;
    asm volatile("" : "+v"(x));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = x; out[1] = (uint32_t)(t1 - t0); }
}
// VALU dependent chain
__global__ void k_valu(uint32_t* out, uint32_t seed) {
  uint32_t x = seed + threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    x = (x ^ 0x5bd1e995u) + 7u;
    asm volatile("" : "+v"(x));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = x; out[1] = (uint32_t)(t1 - t0); }
}
// VALU mul_hi chain
__global__ void k_vmulhi(uint32_t* out, uint32_t seed) {
  uint32_t x = seed + threadIdx.x;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    x = __umulhi(x, 0x9E3779B9u) + 12345u;
    asm volatile("" : "+v"(x));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = x; out[1] = (uint32_t)(t1 - t0); }
}
// SALU independent instruction stream (issue rate): 4 independent chains
__global__ void k_salu4(uint32_t* out, uint32_t seed) {
  uint32_t a = __builtin_amdgcn_readfirstlane(seed), b = a + 1, c = a + 2, d = a + 3;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    a = a + 7u; b = b ^ 9u; c = c + 11u; d = d ^ 13u;
    asm volatile("" : "+s"(a), "+s"(b), "+s"(c), "+s"(d));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = a + b + c + d; out[1] = (uint32_t)(t1 - t0); }
}

typedef void (*kfn)(uint32_t*, uint32_t);
int main() {
  uint32_t* d;
  hipMalloc(&d, 64);
  uint32_t h[2];
  struct { const char* name; kfn f; int ops; } ks[] = {
      {"salu mul+add (2 dep)", k_salu, 2}, {"salu mulhi+add (2 dep)", k_mulhi, 2},
      {"ballot cmp+bcnt+mul+add", k_ballot, 4}, {"readlane+add", k_readlane, 3},
      {"lds uniform ds_read+readfirstlane+add", k_lds, 4}, {"valu lds read+add", k_vlds, 3},
      {"valu xor+add (2 dep)", k_valu, 2}, {"valu mulhi+add", k_vmulhi, 2},
      {"salu 4 indep chains (4 ops)", k_salu4, 4}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 2; rep++) {
      hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, d, 12345u);
      hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    }
    // s_memtime counts at the shader clock on gfx9 (ref: 100 MHz on some parts)
    printf("%-40s %8.1f ticks/step\n", k.name, (double)h[1] / N);
  }
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  printf("clock rate attr %d kHz\n", clk);
  return 0;
}
