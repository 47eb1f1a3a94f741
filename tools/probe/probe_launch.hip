// Dependent-launch latency probe (test infrastructure): back-to-back kernels on one stream.
//   empty        1 workgroup, no memory
//   chain<n>     1 workgroup, n dependent global loads
//   wide<g>      g workgroups of 512 threads that exit at once (the decode's idle grids)
//   wload<g>     g workgroups of 512 threads, each lane loading 20 x 16 B (a pred kernel's
//                register-resident weights) from a 3 MB L2-resident buffer
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty(int* p) {
  if (threadIdx.x == 0 && p[0] == 12345) p[1] = 1;
}
__global__ void k_chain(int* p, int n) {
  if (threadIdx.x) return;
  int i = 0;
  for (int k = 0; k < n; ++k) i = p[i + 2];
  if (i == 12345) p[1] = i;
}
__global__ void __launch_bounds__(512) k_wide(int* p) {
  if (p[0] == 12345) p[1] = blockIdx.x;
}
__global__ void __launch_bounds__(512) k_wload(const uint4* w, int* p) {
  const uint4* src = w + (size_t)blockIdx.x * 512 * 20 + threadIdx.x;
  uint4 acc = uint4{0, 0, 0, 0};
#pragma unroll
  for (int b = 0; b < 20; ++b) {
    const uint4 v = src[b * 512];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if (acc.x == 12345u && acc.y == 7u) p[1] = 1;
}

int main() {
  int* d;
  uint4* w;
  hipMalloc(&d, 1 << 20);
  hipMemset(d, 0, 1 << 20);
  hipMalloc(&w, 64 << 20);
  hipMemset(w, 0, 64 << 20);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int N = 2000;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 50; ++i) launch();
    hipStreamSynchronize(s);
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < N; ++i) launch();
    hipStreamSynchronize(s);
    auto t1 = std::chrono::high_resolution_clock::now();
    printf("%-10s %.2f us per launch\n", name, std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
  };
  run("empty", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d); });
  run("chain1", [&] { hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, s, d, 1); });
  run("chain4", [&] { hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, s, d, 4); });
  run("chain8", [&] { hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, s, d, 8); });
  run("wide10", [&] { hipLaunchKernelGGL(k_wide, dim3(10), dim3(512), 0, s, d); });
  run("wide64", [&] { hipLaunchKernelGGL(k_wide, dim3(64), dim3(512), 0, s, d); });
  run("wide500", [&] { hipLaunchKernelGGL(k_wide, dim3(500), dim3(512), 0, s, d); });
  run("wload5", [&] { hipLaunchKernelGGL(k_wload, dim3(5), dim3(512), 0, s, w, d); });
  run("wload10", [&] { hipLaunchKernelGGL(k_wload, dim3(10), dim3(512), 0, s, w, d); });
  run("wload240", [&] { hipLaunchKernelGGL(k_wload, dim3(240), dim3(512), 0, s, w, d); });
  return 0;
}
