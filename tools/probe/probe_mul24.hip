// probe_mul24.hip -- compile-only reproducer of a ROCm 7.2 (clang 22.0.0git) AMDGPU miscompile:
// a 64-bit multiply of (x & 0xffffff) by a constant that is not a power of two loses the mask.
// The backend matches a 24-bit multiply (v_mul_u32_u24 reads only the low 24 bits, so the `and`
// is dropped as redundant) and later widens it to v_mad_u64_u32, which reads all 32 bits.
//   hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S probe_mul24.hip -o - | grep -A2 global_load_dword
// kA / kD (and, ubfe): v_mad_u64_u32 on the UNMASKED word (wrong address when bits 24-31 are set);
// kB (16-bit mask): v_mul_u32_u24_sdwa WORD_0 (correct); kC (opaque v_and): v_and + v_mad (correct);
// kE (32-bit product): v_mul_u32_u24 (correct while the product fits 32 bits).
// The decode's list entries carry flags above bit 24, so decoder.hip extracts rows through an
// opaque v_and (entry_row); tests/test_isa_lint.py scans every kernel source's IR for the pattern.
#include <hip/hip_runtime.h>

__global__ void kA(const int* in, const float* base, float4* out) {
  const int row = in[threadIdx.x] & 0xffffff;
  out[threadIdx.x] = *(const float4*)(base + (size_t)row * 1280 + 4 * threadIdx.x);
}
__global__ void kB(const int* in, const float* base, float4* out) {
  const int row = in[threadIdx.x] & 0xffff;
  out[threadIdx.x] = *(const float4*)(base + (size_t)row * 1280 + 4 * threadIdx.x);
}
__global__ void kC(const int* in, const float* base, float4* out) {
  int row;
  asm("v_and_b32 %0, 0xffffff, %1" : "=v"(row) : "v"(in[threadIdx.x]));
  out[threadIdx.x] = *(const float4*)(base + (size_t)row * 1280 + 4 * threadIdx.x);
}
__global__ void kD(const int* in, const float* base, float4* out) {
  const int row = (int)__builtin_amdgcn_ubfe((unsigned)in[threadIdx.x], 0, 24);
  out[threadIdx.x] = *(const float4*)(base + (size_t)row * 1280 + 4 * threadIdx.x);
}
__global__ void kE(const int* in, const float* base, float4* out) {
  const unsigned row = (unsigned)in[threadIdx.x] & 0xffffffu;
  out[threadIdx.x] = *(const float4*)(base + (size_t)(row * 1280u) + 4 * threadIdx.x);
}
