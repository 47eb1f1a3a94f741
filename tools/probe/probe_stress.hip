// probe_stress.hip -- development probe: synthetic co-runner kernels for tools/diag_fz_concurrency.py
// (which class of neighbour workgroup disturbs the featurizer's logmel kernel).  Each launcher
// enqueues `iters` launches of one kernel on the given stream.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC probe_stress.hip -o ../../build_dev/libprobe_stress.so
#include <hip/hip_runtime.h>

typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_empty(int* sink) {
  if (threadIdx.x == 1000) sink[0] = 1;
}

__global__ void __launch_bounds__(256) k_lds(int* sink, int reps) {
  __shared__ __attribute__((aligned(16))) uint4 buf[2][256 + 8];
  uint4 v = uint4{threadIdx.x, blockIdx.x, 3u, 4u};
  for (int r = 0; r < reps; ++r) {
    buf[r & 1][threadIdx.x] = v;
    __syncthreads();
    v = buf[r & 1][(threadIdx.x * 7 + r) & 255];
    v.x += 1;
  }
  if (v.x == 0xdeadbeef) sink[0] = (int)v.y;
}

__global__ void __launch_bounds__(256) k_mfma(int* sink, int reps) {
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  uint4 a = uint4{threadIdx.x, 1u, 2u, 3u}, b = uint4{blockIdx.x, 5u, 6u, 7u};
  for (int r = 0; r < reps; ++r) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), acc, 0, 0, 0);
    a.x += 1;
  }
  if (acc[0] == 12345.0f) sink[0] = 1;
}

__global__ void __launch_bounds__(256) k_valu(int* sink, int reps) {
  float x = threadIdx.x, y = blockIdx.x;
  for (int r = 0; r < reps; ++r) {
    x = fmaf(x, 1.0001f, y);
    y = fmaf(y, 0.9999f, x);
  }
  if (x == 12345.0f) sink[0] = 1;
}

__global__ void __launch_bounds__(256) k_glb(const float4* __restrict__ src, int* sink, int reps, int n4) {
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < reps; ++r) {
    const float4 v = src[(blockIdx.x * 256 + threadIdx.x + r * 977) % n4];
    acc.x += v.x;
    acc.y += v.y;
  }
  if (acc.x == 12345.0f) sink[0] = 1;
}

static int* g_sink = nullptr;
static float4* g_src = nullptr;
constexpr int N4 = 1 << 22;

extern "C" int probe_stress(int kind, int grid, int reps, int iters, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!g_sink && hipMalloc(&g_sink, 64) != hipSuccess) return -1;
  if (!g_src) {
    if (hipMalloc(&g_src, N4 * sizeof(float4)) != hipSuccess) return -1;
    if (hipMemset(g_src, 0, N4 * sizeof(float4)) != hipSuccess) return -1;
  }
  for (int i = 0; i < iters; ++i) {
    switch (kind) {
      case 0: hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, st, g_sink); break;
      case 1: hipLaunchKernelGGL(k_lds, dim3(grid), dim3(256), 0, st, g_sink, reps); break;
      case 2: hipLaunchKernelGGL(k_mfma, dim3(grid), dim3(256), 0, st, g_sink, reps); break;
      case 3: hipLaunchKernelGGL(k_valu, dim3(grid), dim3(256), 0, st, g_sink, reps); break;
      case 4: hipLaunchKernelGGL(k_glb, dim3(grid), dim3(256), 0, st, g_src, g_sink, reps, N4); break;
      default: return -1;
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
