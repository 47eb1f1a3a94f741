// Back-to-back dependent launch cost on one stream: plain launches vs the same launches captured
// in a hipGraph (development probe, test infrastructure).  Kernels: an empty one and one that
// reads / writes a small buffer (a decode tail step's shape: a few workgroups, microseconds).
//   build: hipcc --offload-arch=gfx950 -O3 probe_launch_gap.hip -o probe_launch_gap
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int* p) {
  if (p == nullptr) return;
}
__global__ void k_small(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] + 1;
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));           \
      return 1;                                                       \
    }                                                                 \
  } while (0)

template <class F>
static int timed(hipStream_t st, F enqueue, int reps, const char* what, int per) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  enqueue();
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) enqueue();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-34s %7.2f us per kernel\n", what, ms * 1e3 / (reps * per));
  return 0;
}

int main() {
  int* buf;
  CK(hipMalloc(&buf, 1 << 20));
  CK(hipMemset(buf, 0, 1 << 20));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  constexpr int N = 128;  // launches per chunk (32 decode steps x 4)
  auto plain_empty = [&] {
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, buf);
  };
  auto plain_small = [&] {
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, st, buf, 64 * 256);
  };
  if (timed(st, plain_empty, 20, "plain, empty kernel", N)) return 1;
  if (timed(st, plain_small, 20, "plain, 64 x 256 small kernel", N)) return 1;
  for (int v = 0; v < 2; ++v) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    if (v == 0) plain_empty();
    else plain_small();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    auto launch = [&] { (void)hipGraphLaunch(ge, st); };
    if (timed(st, launch, 20, v == 0 ? "graph, empty kernel" : "graph, 64 x 256 small kernel", N)) return 1;
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipStreamSynchronize(st));
  CK(hipFree(buf));
  return 0;
}
