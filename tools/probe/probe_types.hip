#include <hip/hip_runtime.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
__global__ void k(v4i* a, v4i* c, v16i* d, v4f* e, v8bf* f) {
  c[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[0], a[1], c[0], 0, 0, 0);
  d[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[0], a[1], d[0], 0, 0, 0);
  e[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[0], f[1], e[0], 0, 0, 0);
  e[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(1.0f, 2.0f, e[1], 0, 0, 0);
}
