// Development probe (tools/coresident/run.py): can a register- and LDS-light kernel share CUs with
// the encoder's 256x256 tick workgroups (232 VGPRs x 8 waves = 464 of 512 per SIMD, 144 KiB of the
// 160 KiB LDS), and what does it cost the tick?  4-wave workgroups, <= 48 VGPRs, 8 KiB of LDS: per
// iteration every lane loads 16 B of a buffer sized to sit in L2 / MALL (the decode's weight-slice
// reads), folds it into an fp32 sum through LDS, and the last iteration writes one word per lane.
// Bounded: `iters` iterations per launch, no waits on other workgroups.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(256) probe_slim_kernel(const float4* __restrict__ buf, uint32_t n4, int iters,
                                                         float* __restrict__ out) {
  __shared__ float red[2048];
  const uint32_t tid = threadIdx.x;
  uint32_t i = (blockIdx.x * 256u + tid) * 17u;
  float acc = 0.0f;
  for (int it = 0; it < iters; ++it) {
    const float4 v = buf[i % n4];
    acc = __builtin_fmaf(v.x, v.y, acc) + v.z * v.w;
    red[(tid * 8u + (uint32_t)it) & 2047u] = acc;
    __syncthreads();
    acc += red[(tid * 8u + 5u + (uint32_t)it) & 2047u] * 1e-7f;
    i += 4099u * 256u;
  }
  out[blockIdx.x * 256u + tid] = acc;
}

extern "C" int probe_slim_launch(const void* buf, uint64_t bytes, int iters, int grid, void* out, void* stream) {
  if (!buf || !out || bytes < 16 || iters <= 0 || grid <= 0 || grid > 4096) return -1;
  hipLaunchKernelGGL(probe_slim_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float4*)buf,
                     (uint32_t)(bytes / 16), iters, (float*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
