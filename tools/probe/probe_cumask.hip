// probe_cumask.hip -- which (XCC, SE, CU) a CU-masked stream's workgroups land on
// (test infrastructure: decides how bench.py reserves CUs for the decode).
// Usage: probe_cumask <mask spec>...; each spec is a comma list of set bit ranges "a-b".
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <set>
#include <tuple>

__global__ void where_kernel(unsigned* out) {
  if (threadIdx.x) return;
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  out[2 * blockIdx.x] = hw;
  out[2 * blockIdx.x + 1] = xcc;
  // keep the workgroup resident a little so the dispatcher spreads over every allowed CU
  const long long t0 = clock64();
  while (clock64() - t0 < 20000) {}
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  printf("CUs %d\n", ncu);
  const int NB = 4096;
  unsigned* d;
  hipMalloc(&d, NB * 8);
  unsigned* h = (unsigned*)malloc(NB * 8);
  for (int a = 1; a < argc; ++a) {
    uint32_t mask[16] = {0};
    char buf[256];
    strncpy(buf, argv[a], 255);
    for (char* tok = strtok(buf, ","); tok; tok = strtok(nullptr, ",")) {
      int lo, hi;
      if (sscanf(tok, "%d-%d", &lo, &hi) != 2) hi = lo = atoi(tok);
      for (int b = lo; b <= hi && b < 512; ++b) mask[b / 32] |= 1u << (b % 32);
    }
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (ncu + 31) / 32, mask) != hipSuccess) {
      printf("%s: create failed\n", argv[a]);
      continue;
    }
    hipMemsetAsync(d, 0xff, NB * 8, s);
    hipLaunchKernelGGL(where_kernel, dim3(NB), dim3(64), 0, s, d);
    hipStreamSynchronize(s);
    hipMemcpy(h, d, NB * 8, hipMemcpyDeviceToHost);
    std::set<std::tuple<int, int, int, int>> cus;
    std::set<int> xccs;
    int first_xcc[8];
    for (int i = 0; i < 8; ++i) first_xcc[i] = h[2 * i + 1] & 0xf;
    for (int i = 0; i < NB; ++i) {
      const unsigned hw = h[2 * i], x = h[2 * i + 1] & 0xf;
      cus.insert({(int)x, (int)((hw >> 13) & 7), (int)((hw >> 12) & 1), (int)((hw >> 8) & 0xf)});
      xccs.insert(x);
    }
    printf("%s: %zu distinct CUs over %zu XCCs; wg0..7 xcc:", argv[a], cus.size(), xccs.size());
    for (int i = 0; i < 8; ++i) printf(" %d", first_xcc[i]);
    printf("\n  (xcc,se,sh,cu):");
    int n = 0;
    for (auto& c : cus) {
      if (n++ < 48) printf(" (%d,%d,%d,%d)", std::get<0>(c), std::get<1>(c), std::get<2>(c), std::get<3>(c));
    }
    printf("\n");
    hipStreamDestroy(s);
  }
  return 0;
}
