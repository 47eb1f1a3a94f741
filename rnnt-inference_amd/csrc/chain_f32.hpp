// chain_f32.hpp -- fp32 k-ordered fma chains on v_mfma_f32_16x16x4_f32 (shared by the fp32
// encoder and the fp32 decoder).
//
// gfx950's v_mfma_f32_16x16x4_f32 is bit-identical to a k-ordered fmaf chain (tools/probe,
// DESIGN.md), so a dot product written as a chain of these instructions over k = 0, 1, 2, ...
// reproduces the CPU restatement's `acc = fmaf(x[k], w[k], acc)` loop exactly.  Operands use the
// chain-permuted k layout (rnnt_device.hpp chain_pos): one lane's 8 consecutive floats of a
// 32-wide block feed 8 consecutive MFMAs.
#pragma once
#include "rnnt_device.hpp"

namespace rnnt {

#define MFMA4(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

// acc[j] += chain over k in [0, K) of A(row) . B_j, K a multiple of 16; a/b point at this
// lane's first element (row base + 8q); blocks of 32 feed 8 MFMAs, a final half block 4.
template <int NJ = 4>
__device__ __forceinline__ void chain_rows(const float* __restrict__ a, const float* const* b, int K, v4f* acc) {
  const int nb = K >> 5;
  for (int blk = 0; blk < nb; ++blk) {
    const float4 a0 = *(const float4*)(a + 32 * blk), a1 = *(const float4*)(a + 32 * blk + 4);
    float4 b0[NJ], b1[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      b0[j] = *(const float4*)(b[j] + 32 * blk);
      b1[j] = *(const float4*)(b[j] + 32 * blk + 4);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      acc[j] = MFMA4(a0.x, b0[j].x, acc[j]);
      acc[j] = MFMA4(a0.y, b0[j].y, acc[j]);
      acc[j] = MFMA4(a0.z, b0[j].z, acc[j]);
      acc[j] = MFMA4(a0.w, b0[j].w, acc[j]);
      acc[j] = MFMA4(a1.x, b1[j].x, acc[j]);
      acc[j] = MFMA4(a1.y, b1[j].y, acc[j]);
      acc[j] = MFMA4(a1.z, b1[j].z, acc[j]);
      acc[j] = MFMA4(a1.w, b1[j].w, acc[j]);
    }
  }
  if (K & 16) {  // half block: instructions i = 0..3 (k = 32 nb + 4i + q)
    const float4 a0 = *(const float4*)(a + 32 * nb);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float4 b0 = *(const float4*)(b[j] + 32 * nb);
      acc[j] = MFMA4(a0.x, b0.x, acc[j]);
      acc[j] = MFMA4(a0.y, b0.y, acc[j]);
      acc[j] = MFMA4(a0.z, b0.z, acc[j]);
      acc[j] = MFMA4(a0.w, b0.w, acc[j]);
    }
  }
}

}  // namespace rnnt
