// Host-side cost of the HIP calls a streamed frame makes (no kernel work):
// per-call wall time of hipLaunchKernelGGL (a kernel with a 192-byte argument
// struct, like MergeArgs), hipMemcpyAsync H2D / D2H from pinned memory
// (4 KB / 64 KB / 512 KB), hipEventRecord, hipStreamSynchronize on an idle
// stream, and the same launches from 2 and 4 threads at once (does the
// runtime serialise them?).  Streams: 1 or 12 (round robin), as the pipeline's
// lanes.  Build: hipcc -O2 --offload-arch=gfx950 tools/ubench_api.hip -o tools/ubench_api
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

struct Args {
  unsigned char pad[192];
};
__global__ void empty_kernel(Args a) {
  if (threadIdx.x == 1023 && a.pad[0] == 255) a.pad[1] = 0;  // never true in practice
}

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e = (x);                                            \
    if (e != hipSuccess) {                                         \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));           \
      return 1;                                                    \
    }                                                              \
  } while (0)

using Clock = std::chrono::steady_clock;
static double us_since(Clock::time_point t) {
  return std::chrono::duration<double, std::micro>(Clock::now() - t).count();
}

int main() {
  CK(hipSetDevice(0));
  std::vector<hipStream_t> st(12);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void *h = nullptr, *d = nullptr;
  CK(hipHostMalloc(&h, 1 << 20));
  CK(hipMalloc(&d, 1 << 20));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  Args a{};
  const int N = 2000;
  for (int ns : {1, 12}) {
    // warm
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL(empty_kernel, dim3(40), dim3(256), 0, st[i % ns], a);
    CK(hipDeviceSynchronize());
    auto t = Clock::now();
    for (int i = 0; i < N; i++) hipLaunchKernelGGL(empty_kernel, dim3(40), dim3(256), 0, st[i % ns], a);
    double us = us_since(t) / N;
    CK(hipDeviceSynchronize());
    std::printf("streams %2d  hipLaunchKernel (192-B args)        %6.2f us/call\n", ns, us);
    for (size_t bytes : {4096ul, 65536ul, 524288ul}) {
      t = Clock::now();
      for (int i = 0; i < N / 4; i++) CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st[i % ns]));
      us = us_since(t) / (N / 4);
      CK(hipDeviceSynchronize());
      std::printf("streams %2d  hipMemcpyAsync H2D %6zu B          %6.2f us/call\n", ns, bytes, us);
      t = Clock::now();
      for (int i = 0; i < N / 4; i++) CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, st[i % ns]));
      us = us_since(t) / (N / 4);
      CK(hipDeviceSynchronize());
      std::printf("streams %2d  hipMemcpyAsync D2H %6zu B          %6.2f us/call\n", ns, bytes, us);
    }
    t = Clock::now();
    for (int i = 0; i < N; i++) CK(hipEventRecord(ev, st[i % ns]));
    us = us_since(t) / N;
    CK(hipDeviceSynchronize());
    std::printf("streams %2d  hipEventRecord                      %6.2f us/call\n", ns, us);
    t = Clock::now();
    for (int i = 0; i < N; i++) CK(hipStreamSynchronize(st[i % ns]));
    us = us_since(t) / N;
    std::printf("streams %2d  hipStreamSynchronize (idle)         %6.2f us/call\n", ns, us);
    // one launch + one event sync round trip (a tiny kernel's latency)
    t = Clock::now();
    for (int i = 0; i < N / 4; i++) {
      hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st[0], a);
      CK(hipStreamSynchronize(st[0]));
    }
    us = us_since(t) / (N / 4);
    std::printf("streams %2d  launch + hipStreamSynchronize       %6.2f us/round trip\n", ns, us);
  }
  // concurrency: T threads launching on their own streams at once
  for (int T : {2, 4}) {
    std::vector<std::thread> th;
    auto t = Clock::now();
    for (int k = 0; k < T; k++)
      th.emplace_back([&, k]() {
        for (int i = 0; i < N; i++) hipLaunchKernelGGL(empty_kernel, dim3(40), dim3(256), 0, st[k], a);
      });
    for (auto& x : th) x.join();
    double us = us_since(t) / N;
    CK(hipDeviceSynchronize());
    std::printf("threads %d   hipLaunchKernel, each on its stream  %6.2f us per call per thread (%.2f us aggregate)\n",
                T, us, us / T);
  }
  CK(hipHostFree(h));
  CK(hipFree(d));
  return 0;
}
