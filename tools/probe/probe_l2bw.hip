// Per-CU L2 -> CU load throughput by load path (development probe, test infrastructure).
// One workgroup per CU (dynamic LDS keeps it alone), W waves; every wave streams 1 KiB pieces
// (64 lanes x 16 B) of an L2-resident window, PIF pieces in flight per wave between waits:
//   mode 0: global_load_lds_dwordx4 (LDS-DMA, the encoder's staging path)
//   mode 1: global_load_dwordx4 into VGPRs, then ds_write_b128 to LDS
//   mode 2: global_load_dwordx4 into VGPRs only (xor-reduced to keep them live)
// Prints GB/s per CU for each (mode, waves, pieces in flight).
//   build: hipcc --offload-arch=gfx950 -O3 probe_l2bw.hip -o probe_l2bw
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// bytes of the window the 32 workgroups of one XCD sweep together (each starts at its own 1/32);
// <= 4 MiB stays in the XCD's L2, larger windows stream from MALL / HBM

template <int MODE, int PIF>
__global__ void k_bw(const char* __restrict__ src, int iters, int* out, int WIN) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // workgroups of one XCD (id % 8) share a window, so it stays in that XCD's L2
  const char* base = src + (size_t)(blockIdx.x & 7) * WIN + lane * 16;
  v4i x = v4i{0, 0, 0, 0};
  int off = ((blockIdx.x >> 3) * (WIN / 32) + wave * PIF * 1024) % WIN;
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int p = 0; p < PIF; ++p)
        __builtin_amdgcn_global_load_lds((glb_void*)(base + ((off + p * 1024) % WIN)),
                                         (lds_void*)(lds + (wave * PIF + p) % 128 * 1024), 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      v4i v[PIF];
#pragma unroll
      for (int p = 0; p < PIF; ++p) v[p] = __builtin_nontemporal_load((const v4i*)(base + ((off + p * 1024) % WIN)));
      if (MODE == 1) {
#pragma unroll
        for (int p = 0; p < PIF; ++p) *(v4i*)(lds + (wave * PIF + p) % 128 * 1024 + lane * 16) = v[p];
      } else {
#pragma unroll
        for (int p = 0; p < PIF; ++p) x ^= v[p];
      }
    }
    off = (off + nw * PIF * 1024) % WIN;
  }
  __syncthreads();
  int r = x[0] ^ x[1] ^ x[2] ^ x[3] ^ ((int*)lds)[threadIdx.x];
  if (r == 0x12345678) out[threadIdx.x] = r;
}

template <int MODE, int PIF>
static void run(const char* src, int* out, int waves, int win) {
  const int iters = 4000 / waves * 4 / PIF * 8;
  const auto k = k_bw<MODE, PIF>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 144 * 1024);
  hipLaunchKernelGGL(k, dim3(256), dim3(64 * waves), 144 * 1024, 0, src, iters, out, win);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k, dim3(256), dim3(64 * waves), 144 * 1024, 0, src, iters, out, win);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double bytes_per_cu = (double)iters * waves * PIF * 1024;
  printf("win %6d KiB mode %d waves %2d pif %2d: %7.1f GB/s per CU (%.3f ms)\n", win >> 10, MODE, waves, PIF, bytes_per_cu / (ms * 1e-3) / 1e9, ms);
}

template <int MODE>
static void sweep(const char* src, int* out, int win) {
  for (int w : {8, 16}) {
    run<MODE, 2>(src, out, w, win);
    run<MODE, 4>(src, out, w, win);
    run<MODE, 8>(src, out, w, win);
    run<MODE, 16>(src, out, w, win);
  }
}

int main() {
  char* src;
  int* out;
  const int wmax = 64 << 20;
  hipMalloc(&src, 8 * (size_t)wmax);
  hipMemset(src, 1, 8 * (size_t)wmax);
  hipMalloc(&out, 4096 * sizeof(int));
  for (int win : {256 << 10, 2 << 20, 16 << 20, 64 << 20}) {
    sweep<0>(src, out, win);
    sweep<2>(src, out, win);
  }
  hipFree(src);
  hipFree(out);
  return 0;
}
