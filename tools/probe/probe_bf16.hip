// Generic bf16 MFMA probe (test infrastructure): reads <dir>/A.bin, Bt.bin (uint16 bf16 bits,
// [ntile][16][32]) and C.bin (f32 [ntile][16][16]); writes D.bin = one
// v_mfma_f32_16x16x32_bf16 per tile.  Cases are built and analysed by probe_bf16.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <string>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

__global__ void k_bf16_16(const uint16_t* A, const uint16_t* Bt, const float* C, float* D, int ntile) {
  int tile = blockIdx.x;
  if (tile >= ntile) return;
  int l = threadIdx.x;
  const uint16_t* a = A + (size_t)tile * 512;
  const uint16_t* b = Bt + (size_t)tile * 512;
  v8bf fa = *(const v8bf*)(a + (l & 15) * 32 + 8 * (l >> 4));
  v8bf fb = *(const v8bf*)(b + (l & 15) * 32 + 8 * (l >> 4));
  v4f c;
  for (int r = 0; r < 4; ++r) c[r] = C[(size_t)tile * 256 + (4 * (l >> 4) + r) * 16 + (l & 15)];
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(size_t)tile * 256 + (4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

template <class T>
static std::vector<T> rd(const std::string& p) {
  FILE* f = fopen(p.c_str(), "rb");
  if (!f) { fprintf(stderr, "open %s\n", p.c_str()); exit(1); }
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  std::vector<T> v(n / sizeof(T));
  if (fread(v.data(), 1, n, f) != (size_t)n) exit(1);
  fclose(f);
  return v;
}

int main(int argc, char** argv) {
  std::string d = argc > 1 ? argv[1] : ".";
  auto A = rd<uint16_t>(d + "/A.bin");
  auto B = rd<uint16_t>(d + "/Bt.bin");
  auto C = rd<float>(d + "/C.bin");
  const int nt = (int)(A.size() / 512);
  if ((int)(B.size() / 512) != nt || (int)(C.size() / 256) != nt) { fprintf(stderr, "size mismatch\n"); return 1; }
  uint16_t *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, A.size() * 2);
  hipMalloc(&dB, B.size() * 2);
  hipMalloc(&dC, C.size() * 4);
  hipMalloc(&dD, C.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_bf16_16, dim3(nt), dim3(64), 0, 0, dA, dB, dC, dD, nt);
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 1; }
  std::vector<float> D(C.size());
  hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
  FILE* f = fopen((d + "/D.bin").c_str(), "wb");
  fwrite(D.data(), 4, D.size(), f);
  fclose(f);
  printf("tiles %d\n", nt);
  return 0;
}
