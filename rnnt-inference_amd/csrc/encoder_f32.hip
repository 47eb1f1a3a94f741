// encoder_f32.hip -- fp32 transcription (BASELINE config 2: the encoder LSTM stack in fp32).
//
// The reference's run_mode="f32" encoder (models/modeling_rnnt.py:116-144 with torch LSTM
// layers, the `P.lstm` op of the f32 graph) with the fp32 restatement's arithmetic
// (oracle_lstm_f32_layer): per gate row, ax = b_ih + x.W_ih^T and ah = b_hh + h.W_hh^T, each as
// k-ordered fp32 fma chains over 512-k segments summed in segment order (ENC_F32_SEG), gate =
// ax + ah, Cephes-exp sigmoid / tanh, c = f*c + i*g, h = o*tanh(c).  A chain runs on
// v_mfma_f32_16x16x4_f32, which is bit-identical to a k-ordered fmaf chain on gfx950
// (tools/probe), so the output is bit-exact with the CPU restatement (and within the reference's
// fp32 tolerance through it).
//
// Layouts: gate rows interleaved (packed row 4u+g), every k axis chain-permuted inside 32-wide
// blocks (chain_pos), so one lane's 8 consecutive floats feed 8 chained MFMAs.
#include "rnnt_device.hpp"
#include "encoder_f32.hpp"
#include "chain_f32.hpp"

namespace rnnt {

// ---- wavefront tick: workgroup = one 16-row gate tile (4 units) over a 32-row batch group (2
// MFMA batch tiles, two independent accumulators per wave); wave w runs one 512-k segment chain:
// the x chain's ceil(I / 512) segments, then the h chain's 2.  Partial sums meet in LDS and wave 0
// adds them in segment order and runs the cell.  A tick's critical path is one segment (128
// dependent MFMAs per batch tile) instead of a whole chain (up to 512 for layer 2's x), and its
// 1.3 M MFMAs spread over 3-6x the waves, so the chip's fp32 MFMA pipes, not the longest chain,
// bound the tick.
constexpr int F32_NJ = 2;  // 16-row batch tiles per wave
#ifndef RNNT_F32_PF  // development: tools/build_variants.sh "pf2:-DRNNT_F32_PF=2"
#define RNNT_F32_PF 2
#endif
#ifndef RNNT_F32_GT  // development: gate tiles per wave
#define RNNT_F32_GT 2
#endif
constexpr int F32_PF = RNNT_F32_PF;  // 32-k blocks of operands in flight per chain
constexpr int F32_GT = RNNT_F32_GT;  // 16-row gate tiles per wave (sharing each activation block)
// GT x NJ chains (GT 16-row gate tiles x NJ 16-row batch tiles) over the same k range, with the
// operands of the next D 32-k blocks in flight (a register ring: block j in slot j % D).  Each
// activation block feeds GT gate tiles and each weight block NJ batch tiles, so a wave moves
// (GT + NJ) / (GT NJ) of the bytes one chain would per MFMA.  K's final half block (K & 16:
// instructions i = 0..3, k = 32 nb + 4i + q) rides in the ring as block nb.
template <int GT, int NJ, int D>
__device__ __forceinline__ void chain_tiles(const float* const* a, const float* const* b, int K, v4f (*acc)[NJ]) {
  const int nb = K >> 5, nl = nb + ((K & 16) ? 1 : 0);  // full blocks, blocks to load
  float4 ra0[D][GT], ra1[D][GT], rb0[D][NJ], rb1[D][NJ];
  auto load = [&](int i, int j) __attribute__((always_inline)) {  // block j into slot i
#pragma unroll
    for (int g = 0; g < GT; ++g) {
      ra0[i][g] = *(const float4*)(a[g] + 32 * j);
      ra1[i][g] = *(const float4*)(a[g] + 32 * j + 4);
    }
#pragma unroll
    for (int t = 0; t < NJ; ++t) {
      rb0[i][t] = *(const float4*)(b[t] + 32 * j);
      rb1[i][t] = *(const float4*)(b[t] + 32 * j + 4);
    }
  };
  auto step4 = [&](const float4* av, const float4* bv) __attribute__((always_inline)) {  // 4 k of every chain
#pragma unroll
    for (int g = 0; g < GT; ++g)
#pragma unroll
      for (int t = 0; t < NJ; ++t) {
        acc[g][t] = MFMA4(av[g].x, bv[t].x, acc[g][t]);
        acc[g][t] = MFMA4(av[g].y, bv[t].y, acc[g][t]);
        acc[g][t] = MFMA4(av[g].z, bv[t].z, acc[g][t]);
        acc[g][t] = MFMA4(av[g].w, bv[t].w, acc[g][t]);
      }
  };
#pragma unroll
  for (int i = 0; i < D; ++i)
    if (i < nl) load(i, i);
  for (int blk = 0; blk < nb; blk += D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      if (blk + i < nb) {  // uniform
        step4(ra0[i], rb0[i]);
        step4(ra1[i], rb1[i]);
        if (blk + i + D < nl) load(i, blk + i + D);
      }
    }
  }
  if (K & 16) {  // the half block, in slot nb % D
#pragma unroll
    for (int i = 0; i < D; ++i)
      if (i == nb % D) step4(ra0[i], rb0[i]);
  }
}

// workgroups of one job: 256 / F32_GT gate-tile groups x the batch groups; jobs longest K first
constexpr int F32_WAVES = (2048 + ENC_F32_SEG - 1) / ENC_F32_SEG + 1024 / ENC_F32_SEG;  // layer 2: 4 + 2
__global__ void __launch_bounds__(F32_WAVES * 64) lstm_f32_tick_kernel(EncF32TickArgs args, int nbg) {
  __shared__ v4f part[F32_WAVES][F32_GT][F32_NJ][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  constexpr int NGG = G4 / (16 * F32_GT);  // gate-tile groups per layer-step
  const int per_job = NGG * nbg;
  const int jsel = blockIdx.x / per_job, rest = blockIdx.x % per_job;
  const EncF32StepArgs& a = args.job[jsel];
  const int gt0 = (rest % NGG) * F32_GT;       // 16-row gate tiles gt0 .. (units 4gt .. 4gt+3 each)
  const int n0 = (rest / NGG) * (16 * F32_NJ);
  const int sx = (a.I + ENC_F32_SEG - 1) / ENC_F32_SEG, sh = H / ENC_F32_SEG;
  if (wave < sx + sh) {
    const bool xs = wave < sx;
    const int k0 = (xs ? wave : wave - sx) * ENC_F32_SEG;
    const int K = xs ? (a.I - k0 < ENC_F32_SEG ? a.I - k0 : ENC_F32_SEG) : ENC_F32_SEG;
    v4f acc[F32_GT][F32_NJ];
    const float* ap[F32_GT];
    const float* bp[F32_NJ];
#pragma unroll
    for (int g = 0; g < F32_GT; ++g) {
      const int gt = gt0 + g;
      float4 b0 = float4{0.0f, 0.0f, 0.0f, 0.0f};  // a chain's first segment starts at its bias
      if (k0 == 0) b0 = *(const float4*)((xs ? a.bih : a.bhh) + gt * 16 + 4 * q);
#pragma unroll
      for (int j = 0; j < F32_NJ; ++j) acc[g][j] = v4f{b0.x, b0.y, b0.z, b0.w};
      const int row = gt * 16 + c;  // packed gate row fed by this lane (A operand)
      ap[g] = (xs ? a.wih + (size_t)row * a.Ip : a.whh + (size_t)row * H) + 8 * q + k0;
    }
#pragma unroll
    for (int j = 0; j < F32_NJ; ++j)
      bp[j] = (xs ? a.x + (size_t)(n0 + j * 16 + c) * a.Ip : a.h_in + (size_t)(n0 + j * 16 + c) * H) + 8 * q + k0;
    chain_tiles<F32_GT, F32_NJ, F32_PF>(ap, bp, K, acc);
#pragma unroll
    for (int g = 0; g < F32_GT; ++g)
#pragma unroll
      for (int j = 0; j < F32_NJ; ++j) part[wave][g][j][lane] = acc[g][j];
  }
  __syncthreads();
  if (wave) return;
  // C/D: lane (q, c) holds rows 4q..4q+3 of a tile = gates i,f,g,o of unit 4gt+q, batch row c
#pragma unroll
  for (int g = 0; g < F32_GT; ++g) {
    const int u = (gt0 + g) * 4 + q;
#pragma unroll
    for (int j = 0; j < F32_NJ; ++j) {
      const int n = n0 + j * 16 + c;
      if (n >= a.n) continue;
      v4f ax = part[0][g][j][lane], ah = part[sx][g][j][lane];
      for (int s = 1; s < sx; ++s) ax = ax + part[s][g][j][lane];  // segment order: ((s0 + s1) + s2) + ...
      for (int s = 1; s < sh; ++s) ah = ah + part[sx + s][g][j][lane];
      const float ig = det_sigmoid(ax[0] + ah[0]);
      const float fg = det_sigmoid(ax[1] + ah[1]);
      const float gg = det_tanh(ax[2] + ah[2]);
      const float og = det_sigmoid(ax[3] + ah[3]);
      float* cp = a.c + (size_t)n * H + u;
      const float cn = fg * *cp + ig * gg;
      *cp = cn;
      const float hh = og * det_tanh(cn);
      a.h_out[(size_t)n * H + chain_pos(u)] = hh;
      if (a.mode == ENC_F32_NEXT) {
        a.y[(size_t)n * H + chain_pos(u)] = hh;
      } else if (a.mode == ENC_F32_STACKED) {
        // StackTime.forward_f32 (modeling_rnnt.py:314-324): frame t -> stacked frame t/2, half
        // t%2, frames t >= x_lens[n] zeroed, odd-T pad frame zero
        float* dst = a.y + (size_t)n * 2 * H + chain_pos(u);
        dst[a.half * H] = a.t < a.lens[n] ? hh : 0.0f;
        if (a.zero_next) dst[H] = 0.0f;
      } else {
        if (a.y) a.y[(size_t)n * H + u] = hh;
        if (a.y2) a.y2[(size_t)n * H + chain_pos(u)] = hh;
        if (a.ybf) a.ybf[(size_t)n * H + u] = f2bf_ftz(hh);
      }
    }
  }
}

int launch_lstm_f32_tick(const EncF32TickArgs& a, hipStream_t st) {
  if (a.njobs <= 0) return 0;
  const int n = a.job[0].n;
  for (int j = 0; j < a.njobs; ++j)
    if (a.job[j].n != n || a.job[j].I % 16 || a.job[j].Ip % 32 || a.job[j].Ip < a.job[j].I) return -1;
  if (n <= 0) return 0;
  for (int j = 0; j < a.njobs; ++j)  // the workgroup's waves cover the segments of the widest input
    if ((a.job[j].I + ENC_F32_SEG - 1) / ENC_F32_SEG + H / ENC_F32_SEG > F32_WAVES) return -1;
  const int nbg = (n + 16 * F32_NJ - 1) / (16 * F32_NJ);  // rows < n_pad (a multiple of 64) stay in bounds
  hipLaunchKernelGGL(lstm_f32_tick_kernel, dim3(a.njobs * (G4 / (16 * F32_GT)) * nbg), dim3(F32_WAVES * 64), 0, st, a, nbg);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// features [T][n_pad][256] natural -> [T][n_pad][256] chain-permuted (channels >= 240 are 0)
__global__ void permute_feats_kernel(const float* __restrict__ x, int64_t rows, float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * FEAT) return;
  const int64_t r = i / FEAT;
  const int k = (int)(i % FEAT);
  y[r * FEAT + chain_pos(k)] = x[i];
}

int launch_permute_feats(const float* x, int64_t rows, float* y, hipStream_t st) {
  const int64_t total = rows * FEAT;
  hipLaunchKernelGGL(permute_feats_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, rows, y);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rnnt
