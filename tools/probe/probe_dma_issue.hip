// LDS-DMA issue cost beside MFMAs (development probe, test infrastructure).
// One 256-thread workgroup per CU (4 waves, one per SIMD; 144 KiB of dynamic LDS keeps it
// alone), each wave issuing ITER "stages" of 128 v_mfma_i32_16x16x64_i8 on 64 independent
// accumulators with NP global_load_lds_dwordx4 pieces (1 KiB each, L2-resident source)
// interleaved evenly, one vmcnt(0) + barrier per stage -- the shape of a one-wave-per-SIMD
// encoder main loop.  Prints cycles per stage for each NP; NP = 0 is the MFMA floor (2048).
//   build: hipcc --offload-arch=gfx950 -O3 probe_dma_issue.hip -o probe_dma_issue
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

template <int NP, int WPS, bool BAR = true, int NACC = 32>
__global__ void __launch_bounds__(256 * WPS, 1) k_probe(const char* __restrict__ src, int iters, int* out,
                                                          long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v4i a = *(const v4i*)(src + lane * 16), b = *(const v4i*)(src + 4096 + lane * 16);
  v4i acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = v4i{0, 0, 0, 0};
  const char* s0 = src + ((blockIdx.x * 4 + wave) & 255) * 16384 + lane * 16;
  const long long t0 = __builtin_amdgcn_s_memtime();
  constexpr int G = 16 / WPS, NPW = NP / WPS;  // 8-MFMA groups and pieces per wave per stage
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[(8 * g + i) % NACC] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[(8 * g + i) % NACC], 0, 0, 0);
#pragma unroll
      for (int p = 0; p < NPW; ++p)
        if ((p * G) / NPW == g)
          __builtin_amdgcn_global_load_lds((glb_void*)(s0 + (it & 7) * 2048 + (p & 31) * 64),
                                           (lds_void*)(lds + (wave & 3) * 32768 + (p & 31) * 1024), 16, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (BAR) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  int r = 0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) r ^= acc[i][0] ^ acc[i][1] ^ acc[i][2] ^ acc[i][3];
  if (r == 0x12345678) out[threadIdx.x] = r;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

template <int NP, int WPS, bool BAR = true, int NACC = 32>
static void run(const char* src, int* out, long long* cyc) {
  const int iters = 200;
  hipFuncSetAttribute((const void*)k_probe<NP, WPS, BAR, NACC>, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024);
  hipLaunchKernelGGL((k_probe<NP, WPS, BAR, NACC>), dim3(256), dim3(256 * WPS), 144 * 1024, 0, src, iters, out, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_probe<NP, WPS, BAR, NACC>), dim3(256), dim3(256 * WPS), 144 * 1024, 0, src, iters, out, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  long long c = 0;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  // s_memtime counts the shader clock; per stage: 128 MFMAs per SIMD (WPS waves x 128 / WPS)
  printf("waves/SIMD %d  pieces/stage/SIMD %2d  barrier %d  accumulators %2d  %8.1f cycles/stage (s_memtime)  %7.3f us/stage (events)\n", WPS, NP, (int)BAR, NACC,
         (double)c / iters, ms * 1e3 / iters);
}

int main() {
  char* src;
  int* out;
  long long* cyc;
  hipMalloc(&src, 8 << 20);
  hipMemset(src, 1, 8 << 20);
  hipMalloc(&out, 4096);
  hipMalloc(&cyc, 8);
  run<0, 1>(src, out, cyc);
  run<4, 1>(src, out, cyc);
  run<8, 1>(src, out, cyc);
  run<16, 1>(src, out, cyc);
  run<32, 1>(src, out, cyc);
  run<0, 2>(src, out, cyc);
  run<8, 2>(src, out, cyc);
  run<16, 2>(src, out, cyc);
  // the one-wave issue rate without the per-stage barrier, and with 64 accumulators
  run<0, 1, false, 32>(src, out, cyc);
  run<0, 1, false, 64>(src, out, cyc);
  run<0, 1, true, 64>(src, out, cyc);
  run<0, 2, false, 32>(src, out, cyc);
  run<16, 1, false, 64>(src, out, cyc);
  return 0;
}
