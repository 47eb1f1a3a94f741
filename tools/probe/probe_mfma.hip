// MFMA numerics/layout probe for gfx950 (test infrastructure, not product code).
// Writes raw inputs/outputs to <outdir>/*.bin; tools/probe/analyze_mfma.py checks
// layout hypotheses (int8) and accumulation models (f32 / bf16).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>
#include <string>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

// ---- int8 16x16x64: A[16][64], Bt[16][64] (B transposed), D[16][16]
__global__ void k_i8_16(const int8_t* A, const int8_t* Bt, int* D, int ntile) {
  int tile = blockIdx.x; if (tile >= ntile) return;
  int l = threadIdx.x;
  const int8_t* a = A + tile * 1024; const int8_t* b = Bt + tile * 1024;
  v4i fa = *(const v4i*)(a + (l & 15) * 64 + 16 * (l >> 4));
  v4i fb = *(const v4i*)(b + (l & 15) * 64 + 16 * (l >> 4));
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa, fb, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[tile * 256 + (4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}
// ---- int8 32x32x32: A[32][32], Bt[32][32], D[32][32]
__global__ void k_i8_32(const int8_t* A, const int8_t* Bt, int* D, int ntile) {
  int tile = blockIdx.x; if (tile >= ntile) return;
  int l = threadIdx.x;
  const int8_t* a = A + tile * 1024; const int8_t* b = Bt + tile * 1024;
  v4i fa = *(const v4i*)(a + (l & 31) * 32 + 16 * (l >> 5));
  v4i fb = *(const v4i*)(b + (l & 31) * 32 + 16 * (l >> 5));
  v16i c; for (int r = 0; r < 16; ++r) c[r] = 0;
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[tile * 1024 + ((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}
// ---- f32 16x16x4 chained over K=64: A[16][64], Bt[16][64], C[16][16] -> D
__global__ void k_f32_16(const float* A, const float* Bt, const float* C, float* D, int ntile) {
  int tile = blockIdx.x; if (tile >= ntile) return;
  int l = threadIdx.x;
  const float* a = A + tile * 1024; const float* b = Bt + tile * 1024;
  v4f c; for (int r = 0; r < 4; ++r) c[r] = C[tile * 256 + (4 * (l >> 4) + r) * 16 + (l & 15)];
  for (int kb = 0; kb < 16; ++kb)
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[(l & 15) * 64 + 4 * kb + (l >> 4)], b[(l & 15) * 64 + 4 * kb + (l >> 4)], c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[tile * 256 + (4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}
// ---- bf16 16x16x32 single instruction: A[16][32], Bt[16][32] (bf16 bits), C, D [16][16]
__global__ void k_bf16_16(const uint16_t* A, const uint16_t* Bt, const float* C, float* D, int ntile) {
  int tile = blockIdx.x; if (tile >= ntile) return;
  int l = threadIdx.x;
  const uint16_t* a = A + tile * 512; const uint16_t* b = Bt + tile * 512;
  v8bf fa = *(const v8bf*)(a + (l & 15) * 32 + 8 * (l >> 4));
  v8bf fb = *(const v8bf*)(b + (l & 15) * 32 + 8 * (l >> 4));
  v4f c; for (int r = 0; r < 4; ++r) c[r] = C[tile * 256 + (4 * (l >> 4) + r) * 16 + (l & 15)];
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[tile * 256 + (4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}
// ---- bf16 32x32x16 single instruction: A[32][16], Bt[32][16], C, D [32][32]
__global__ void k_bf16_32(const uint16_t* A, const uint16_t* Bt, const float* C, float* D, int ntile) {
  int tile = blockIdx.x; if (tile >= ntile) return;
  int l = threadIdx.x;
  const uint16_t* a = A + tile * 512; const uint16_t* b = Bt + tile * 512;
  v8bf fa = *(const v8bf*)(a + (l & 31) * 16 + 8 * (l >> 5));
  v8bf fb = *(const v8bf*)(b + (l & 31) * 16 + 8 * (l >> 5));
  v16f c; for (int r = 0; r < 16; ++r) c[r] = C[tile * 1024 + ((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)];
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[tile * 1024 + ((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

static uint64_t g_s = 0x1234567ull;
static uint64_t nxt() { g_s += 0x9E3779B97F4A7C15ull; uint64_t z = g_s; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return z ^ (z >> 31); }
static double unif() { return (nxt() >> 11) * (1.0 / 9007199254740992.0); }
static double gauss() { double u = unif() + 1e-300, v = unif(); return sqrt(-2 * log(u)) * cos(6.283185307179586 * v); }
static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16; return (uint16_t)u; }

template <class T> static void dump(const std::string& dir, const char* name, const std::vector<T>& v) {
  std::string p = dir + "/" + name; FILE* f = fopen(p.c_str(), "wb"); if (!f) { perror(p.c_str()); exit(1); }
  fwrite(v.data(), sizeof(T), v.size(), f); fclose(f);
}
template <class T> static T* todev(const std::vector<T>& v) { T* d; CK(hipMalloc(&d, v.size() * sizeof(T))); CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice)); return d; }
template <class T> static std::vector<T> tohost(const T* d, size_t n) { std::vector<T> v(n); CK(hipMemcpy(v.data(), d, n * sizeof(T), hipMemcpyDeviceToHost)); return v; }

int main(int argc, char** argv) {
  std::string dir = argc > 1 ? argv[1] : ".";
  const int NT = 512;
  // int8
  {
    std::vector<int8_t> A(NT * 1024), B(NT * 1024);
    for (auto& x : A) x = (int8_t)((int)(nxt() % 256) - 128);
    for (auto& x : B) x = (int8_t)((int)(nxt() % 256) - 128);
    int8_t *dA = todev(A), *dB = todev(B); int* dD; CK(hipMalloc(&dD, NT * 1024 * 4));
    k_i8_16<<<NT, 64>>>(dA, dB, dD, NT); CK(hipDeviceSynchronize());
    auto D16 = tohost(dD, NT * 256);
    k_i8_32<<<NT, 64>>>(dA, dB, dD, NT); CK(hipDeviceSynchronize());
    auto D32 = tohost(dD, NT * 1024);
    dump(dir, "i8_A.bin", A); dump(dir, "i8_B.bin", B); dump(dir, "i8_D16.bin", D16); dump(dir, "i8_D32.bin", D32);
  }
  // f32 chain
  {
    std::vector<float> A(NT * 1024), B(NT * 1024), C(NT * 256);
    for (auto& x : A) x = (float)(gauss() * pow(2.0, (int)(nxt() % 13) - 6));
    for (auto& x : B) x = (float)gauss();
    for (auto& x : C) x = (float)(gauss() * 4);
    float *dA = todev(A), *dB = todev(B), *dC = todev(C), *dD; CK(hipMalloc(&dD, NT * 256 * 4));
    k_f32_16<<<NT, 64>>>(dA, dB, dC, dD, NT); CK(hipDeviceSynchronize());
    dump(dir, "f32_A.bin", A); dump(dir, "f32_B.bin", B); dump(dir, "f32_C.bin", C); dump(dir, "f32_D.bin", tohost(dD, NT * 256));
  }
  // bf16: several distributions
  for (int dist = 0; dist < 5; ++dist) {
    std::vector<uint16_t> A(NT * 512), B(NT * 512); std::vector<float> C(NT * 1024);
    for (size_t i = 0; i < A.size(); ++i) {
      double a = gauss(), b = gauss();
      if (dist == 2 || dist == 3) a *= pow(2.0, (int)(nxt() % 41) - 20);
      if (dist == 4) { a = (unif() * 2 - 1) * 0.1; b = tanh(gauss()); }
      A[i] = f2bf((float)a); B[i] = f2bf((float)b);
    }
    for (auto& c : C) {
      double v = 0;
      if (dist == 1) v = gauss() * 10;
      if (dist == 3) v = gauss() * pow(2.0, (int)(nxt() % 21) - 10);
      if (dist == 4) v = gauss() * 0.1;
      c = (float)v;
    }
    uint16_t *dA = todev(A), *dB = todev(B); float *dC = todev(C), *dD; CK(hipMalloc(&dD, NT * 1024 * 4));
    k_bf16_16<<<NT, 64>>>(dA, dB, dC, dD, NT); CK(hipDeviceSynchronize());
    auto D16 = tohost(dD, NT * 256);
    k_bf16_32<<<NT, 64>>>(dA, dB, dC, dD, NT); CK(hipDeviceSynchronize());
    auto D32 = tohost(dD, NT * 1024);
    char nm[64];
    snprintf(nm, 64, "bf_A%d.bin", dist); dump(dir, nm, A);
    snprintf(nm, 64, "bf_B%d.bin", dist); dump(dir, nm, B);
    snprintf(nm, 64, "bf_C%d.bin", dist); dump(dir, nm, C);
    snprintf(nm, 64, "bf_D16_%d.bin", dist); dump(dir, nm, D16);
    snprintf(nm, 64, "bf_D32_%d.bin", dist); dump(dir, nm, D32);
  }
  printf("probe done\n");
  return 0;
}
