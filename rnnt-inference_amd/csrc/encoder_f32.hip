// encoder_f32.hip -- fp32 transcription (BASELINE config 2: the encoder LSTM stack in fp32).
//
// The reference's run_mode="f32" encoder (models/modeling_rnnt.py:116-144 with torch LSTM
// layers, the `P.lstm` op of the f32 graph) with the fp32 restatement's arithmetic
// (oracle_lstm_f32_layer): per gate row, ax = b_ih + x.W_ih^T and ah = b_hh + h.W_hh^T as two
// k-ordered fp32 fma chains, gate = ax + ah, Cephes-exp sigmoid / tanh, c = f*c + i*g,
// h = o*tanh(c).  The chains run on v_mfma_f32_16x16x4_f32, which is bit-identical to a
// k-ordered fmaf chain on gfx950 (tools/probe), so the output is bit-exact with the CPU
// restatement (and within the reference's fp32 tolerance through it).
//
// Layouts: gate rows interleaved (packed row 4u+g), every k axis chain-permuted inside 32-wide
// blocks (chain_pos), so one lane's 8 consecutive floats feed 8 chained MFMAs.  One launch =
// one layer x one timestep; workgroup = 4 waves x (16 gate rows) x 64 batch rows.
#include "rnnt_device.hpp"
#include "encoder_f32.hpp"
#include "chain_f32.hpp"

namespace rnnt {

__global__ void __launch_bounds__(256) lstm_f32_step_kernel(EncF32StepArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const int gt = blockIdx.x * 4 + wave;  // 16-row gate tile = units 4gt .. 4gt+3
  const int n0 = blockIdx.y * 64;
  const int row = gt * 16 + c;           // packed gate row fed by this lane (A operand)
  const float* bx[4];
  const float* bh[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bx[j] = a.x + (size_t)(n0 + j * 16 + c) * a.Ip + 8 * q;
    bh[j] = a.h_in + (size_t)(n0 + j * 16 + c) * H + 8 * q;
  }
  v4f ax[4], ah[4];
  const float4 bi = *(const float4*)(a.bih + gt * 16 + 4 * q), bhv = *(const float4*)(a.bhh + gt * 16 + 4 * q);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ax[j] = v4f{bi.x, bi.y, bi.z, bi.w};
    ah[j] = v4f{bhv.x, bhv.y, bhv.z, bhv.w};
  }
  chain_rows(a.wih + (size_t)row * a.Ip + 8 * q, bx, a.I, ax);
  chain_rows(a.whh + (size_t)row * H + 8 * q, bh, H, ah);
  // C/D: lane (q, c) holds rows 4q..4q+3 of the tile = gates i,f,g,o of unit 4gt+q, batch row c
  const int u = gt * 4 + q;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + j * 16 + c;
    if (n >= a.n) continue;
    const float ig = det_sigmoid(ax[j][0] + ah[j][0]);
    const float fg = det_sigmoid(ax[j][1] + ah[j][1]);
    const float gg = det_tanh(ax[j][2] + ah[j][2]);
    const float og = det_sigmoid(ax[j][3] + ah[j][3]);
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

// ---- wavefront tick: workgroup = 8 waves = 4 gate tiles (64 gate rows, 16 units) x {x chain,
// h chain}, over a 32-row batch group (2 MFMA batch tiles, two independent accumulators per
// wave).  The x and h chains of a gate tile run on two waves at once (the chains are k-ordered
// and cannot be split, so the tick's latency is the longest chain, K/4 dependent MFMAs); the h
// wave hands its sums over through LDS and the x wave runs the cell.  The 4 gate tiles of a
// workgroup read the same activation rows at about the same time (per-CU cache reuse); one tick
// reads every weight once.
constexpr int F32_NJ = 2;  // 16-row batch tiles per wave
template <int NJ>
__device__ __forceinline__ void chain_rows_pf(const float* __restrict__ a, const float* const* b, int K, v4f* acc) {
  // chain_rows with the next 32-k block's operands loaded before this block's MFMAs
  const int nb = K >> 5;
  float4 a0 = *(const float4*)a, a1 = *(const float4*)(a + 4), b0[NJ], b1[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    b0[j] = *(const float4*)b[j];
    b1[j] = *(const float4*)(b[j] + 4);
  }
  for (int blk = 0; blk < nb; ++blk) {
    // next block; after the last full block, the half block (rows are padded to 32-k blocks) or a
    // harmless re-read of the current one
    const int nx = (blk + 1 < nb || (K & 16)) ? blk + 1 : blk;
    const float4 na0 = *(const float4*)(a + 32 * nx), na1 = *(const float4*)(a + 32 * nx + 4);
    float4 nb0[NJ], nb1[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      nb0[j] = *(const float4*)(b[j] + 32 * nx);
      nb1[j] = *(const float4*)(b[j] + 32 * nx + 4);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      acc[j] = MFMA4(a0.x, b0[j].x, acc[j]);
      acc[j] = MFMA4(a0.y, b0[j].y, acc[j]);
      acc[j] = MFMA4(a0.z, b0[j].z, acc[j]);
      acc[j] = MFMA4(a0.w, b0[j].w, acc[j]);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      acc[j] = MFMA4(a1.x, b1[j].x, acc[j]);
      acc[j] = MFMA4(a1.y, b1[j].y, acc[j]);
      acc[j] = MFMA4(a1.z, b1[j].z, acc[j]);
      acc[j] = MFMA4(a1.w, b1[j].w, acc[j]);
    }
    a0 = na0;
    a1 = na1;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      b0[j] = nb0[j];
      b1[j] = nb1[j];
    }
  }
  if (K & 16) {  // half block: instructions i = 0..3 (k = 32 nb + 4i + q)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      acc[j] = MFMA4(a0.x, b0[j].x, acc[j]);
      acc[j] = MFMA4(a0.y, b0[j].y, acc[j]);
      acc[j] = MFMA4(a0.z, b0[j].z, acc[j]);
      acc[j] = MFMA4(a0.w, b0[j].w, acc[j]);
    }
  }
}

// workgroups of one job: 64 gate groups x the batch groups; jobs longest K first
__global__ void __launch_bounds__(512) lstm_f32_tick_kernel(EncF32TickArgs args, int nbg) {
  __shared__ v4f ahs[4][F32_NJ][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const int gw = wave & 3, hchain = wave >> 2;
  const int per_job = (G4 / 64) * nbg;
  const int jsel = blockIdx.x / per_job, rest = blockIdx.x % per_job;
  const EncF32StepArgs& a = args.job[jsel];
  const int gt = (rest % (G4 / 64)) * 4 + gw;  // 16-row gate tile = units 4gt .. 4gt+3
  const int n0 = (rest / (G4 / 64)) * (16 * F32_NJ);
  const int row = gt * 16 + c;                 // packed gate row fed by this lane (A operand)
  v4f acc[F32_NJ];
  const float* bp[F32_NJ];
  if (!hchain) {
    const float4 bi = *(const float4*)(a.bih + gt * 16 + 4 * q);
#pragma unroll
    for (int j = 0; j < F32_NJ; ++j) {
      acc[j] = v4f{bi.x, bi.y, bi.z, bi.w};
      bp[j] = a.x + (size_t)(n0 + j * 16 + c) * a.Ip + 8 * q;
    }
    chain_rows_pf<F32_NJ>(a.wih + (size_t)row * a.Ip + 8 * q, bp, a.I, acc);
  } else {
    const float4 bh = *(const float4*)(a.bhh + gt * 16 + 4 * q);
#pragma unroll
    for (int j = 0; j < F32_NJ; ++j) {
      acc[j] = v4f{bh.x, bh.y, bh.z, bh.w};
      bp[j] = a.h_in + (size_t)(n0 + j * 16 + c) * H + 8 * q;
    }
    chain_rows_pf<F32_NJ>(a.whh + (size_t)row * H + 8 * q, bp, H, acc);
#pragma unroll
    for (int j = 0; j < F32_NJ; ++j) ahs[gw][j][lane] = acc[j];
  }
  __syncthreads();
  if (hchain) return;
  // C/D: lane (q, c) holds rows 4q..4q+3 of the tile = gates i,f,g,o of unit 4gt+q, batch row c
  const int u = gt * 4 + q;
#pragma unroll
  for (int j = 0; j < F32_NJ; ++j) {
    const int n = n0 + j * 16 + c;
    if (n >= a.n) continue;
    const v4f ah = ahs[gw][j][lane];
    const float ig = det_sigmoid(acc[j][0] + ah[0]);
    const float fg = det_sigmoid(acc[j][1] + ah[1]);
    const float gg = det_tanh(acc[j][2] + ah[2]);
    const float og = det_sigmoid(acc[j][3] + ah[3]);
    float* cp = a.c + (size_t)n * H + u;
    const float cn = fg * *cp + ig * gg;
    *cp = cn;
    const float hh = og * det_tanh(cn);
    a.h_out[(size_t)n * H + chain_pos(u)] = hh;
    if (a.mode == ENC_F32_NEXT) {
      a.y[(size_t)n * H + chain_pos(u)] = hh;
    } else if (a.mode == ENC_F32_STACKED) {
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

int launch_lstm_f32_tick(const EncF32TickArgs& a, hipStream_t st) {
  if (a.njobs <= 0) return 0;
  const int n = a.job[0].n;
  for (int j = 0; j < a.njobs; ++j)
    if (a.job[j].n != n || a.job[j].I % 16 || a.job[j].Ip % 32 || a.job[j].Ip < a.job[j].I) return -1;
  if (n <= 0) return 0;
  const int nbg = (n + 16 * F32_NJ - 1) / (16 * F32_NJ);  // rows < n_pad (a multiple of 64) stay in bounds
  hipLaunchKernelGGL(lstm_f32_tick_kernel, dim3(a.njobs * (G4 / 64) * nbg), dim3(512), 0, st, a, nbg);
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

int launch_lstm_f32_step(const EncF32StepArgs& a, hipStream_t st) {
  if (a.n <= 0) return 0;
  if (a.I % 16 || a.Ip % 32 || a.Ip < a.I) return -1;
  hipLaunchKernelGGL(lstm_f32_step_kernel, dim3(G4 / 64, (a.n + 63) / 64), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_permute_feats(const float* x, int64_t rows, float* y, hipStream_t st) {
  const int64_t total = rows * FEAT;
  hipLaunchKernelGGL(permute_feats_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, rows, y);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rnnt
