// hipGraphLaunch ordering probe (development probe, test infrastructure): is a graph launched
// on a stream ordered after the kernels enqueued on that stream before it, with one or several
// host threads capturing and launching at once?  A slow kernel writes v into a buffer, a
// captured chain of kernels adds 1 to every element 32 times, the host checks v + 32.
//   build: hipcc --offload-arch=gfx950 -O3 probe_graph_order.hip -o probe_graph_order -lpthread
#include <hip/hip_runtime.h>
#include <cstdio>
#include <thread>
#include <vector>

__global__ void k_slow_set(int* p, int n, int v, int spin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  long long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < spin) {
  }
  if (i < n) p[i] = v;
}
__global__ void k_inc(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1;
}

static int run(int tid, bool null_stream, int* errs) {
  const int n = 1 << 16;
  int* d;
  if (hipMalloc(&d, n * sizeof(int)) != hipSuccess) return 1;
  hipStream_t st = nullptr, cap;
  if (!null_stream) (void)hipStreamCreate(&st);
  (void)hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
  std::vector<int> h(n);
  int bad = 0;
  for (int rep = 0; rep < 20; ++rep) {
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
    for (int k = 0; k < 32; ++k) hipLaunchKernelGGL(k_inc, dim3(n / 256), dim3(256), 0, cap, d, n);
    (void)hipStreamEndCapture(cap, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    const int v = 1000 * tid + rep;
    hipLaunchKernelGGL(k_slow_set, dim3(n / 256), dim3(256), 0, st, d, n, v, 200000);
    (void)hipGraphLaunch(ge, st);
    (void)hipMemcpyAsync(h.data(), d, n * sizeof(int), hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    for (int i = 0; i < n; ++i)
      if (h[i] != v + 32) {
        ++bad;
        break;
      }
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
  }
  errs[tid] = bad;
  (void)hipFree(d);
  if (st) (void)hipStreamDestroy(st);
  (void)hipStreamDestroy(cap);
  return 0;
}

int main() {
  int errs[8] = {};
  run(0, true, errs);
  printf("1 thread, null stream:    %d of 20 reps wrong\n", errs[0]);
  run(0, false, errs);
  printf("1 thread, created stream: %d of 20 reps wrong\n", errs[0]);
  std::vector<std::thread> ths;
  for (int t = 0; t < 4; ++t) ths.emplace_back([&, t] { run(t, false, errs); });
  for (auto& t : ths) t.join();
  printf("4 threads, own streams:   %d %d %d %d of 20 reps wrong\n", errs[0], errs[1], errs[2], errs[3]);
  return 0;
}
