// decoder.hip -- prediction network, joint and greedy decode on CDNA4.
//
// Replaces intel_mlperf::lstm_amx_bf16, amx_linear_bf16_accum_relu, amx_linear_i16o32 and
// greedy_decode_update (reference modeling_rnnt.py:183-205, 259-289, 331-365) and the host
// decode loop of csrc/rnnt_model.hpp:92-124.  Every dot product is an fp32 k-ordered fmaf
// chain on bf16-valued operands, computed with v_mfma_f32_16x16x4_f32 (probe-verified to be
// bit-identical to a sequential fmaf chain), so the decode is bit-exact with the CPU
// restatement and therefore token-identical.
//
// The whole greedy loop runs on the device: one workgroup owns DEC_ROWS utterances and
// iterates emit/advance steps until all of them finish -- no host round trip per step, no
// inter-workgroup synchronisation (rows never interact, decoder.py:125-167).  Two
// algebraic shortcuts, both exact:
//   * the joint's encoder half F[t] = b_t + bf16(f_t).W1t^T depends only on the frame, so it is
//     one batched GEMM over all frames before the loop (launch_joint_trans);
//   * prediction(pre_g, pre_hg, pre_cg) depends only on state that changes on an emit, so it
//     (and the joint's prediction half G) is evaluated once per emit, not once per step.
#include "rnnt_device.hpp"
#include "decoder.hpp"

namespace rnnt {

#define MFMA4(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

// 8 chained MFMAs over one 32-wide k block: w = this lane's 8 bf16 A values (k = 4i+q),
// x = its 8 f32 B values.
__device__ __forceinline__ v4f chain8(const uint4 w, const float* x, v4f acc) {
  acc = MFMA4(bits2f(w.x << 16), x[0], acc);
  acc = MFMA4(bits2f(w.x & 0xffff0000u), x[1], acc);
  acc = MFMA4(bits2f(w.y << 16), x[2], acc);
  acc = MFMA4(bits2f(w.y & 0xffff0000u), x[3], acc);
  acc = MFMA4(bits2f(w.z << 16), x[4], acc);
  acc = MFMA4(bits2f(w.z & 0xffff0000u), x[5], acc);
  acc = MFMA4(bits2f(w.w << 16), x[6], acc);
  acc = MFMA4(bits2f(w.w & 0xffff0000u), x[7], acc);
  return acc;
}
__device__ __forceinline__ void bf8_to_f32(const uint4 v, float* x) {
  x[0] = bits2f(v.x << 16); x[1] = bits2f(v.x & 0xffff0000u);
  x[2] = bits2f(v.y << 16); x[3] = bits2f(v.y & 0xffff0000u);
  x[4] = bits2f(v.z << 16); x[5] = bits2f(v.z & 0xffff0000u);
  x[6] = bits2f(v.w << 16); x[7] = bits2f(v.w & 0xffff0000u);
}

// ---------------------------------------------------------------- F = b_t + f . W1t^T
// rows = (frame, batch row) pairs of fperm [Tp][Npad][1024]; one workgroup = 64 rows x 64 j.
__global__ void __launch_bounds__(256) joint_trans_kernel(DecWeights w, const uint16_t* __restrict__ fperm,
                                                          const int32_t* __restrict__ f_lens,
                                                          float* __restrict__ F, int Npad) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const int row0 = blockIdx.y * 64;
  const int t = row0 / Npad, nb = row0 % Npad;
  if (!__any(f_lens[nb + lane] > t)) return;  // no valid frame in this tile
  const int j0 = blockIdx.x * 64;
  const int row = row0 + wave * 16 + c;
  v4f acc[4];
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    const float4 b = *(const float4*)(w.bt + j0 + jt * 16 + 4 * q);
    acc[jt] = v4f{b.x, b.y, b.z, b.w};
  }
  const uint16_t* xr = fperm + (size_t)row * H + 8 * q;
  const uint16_t* wr = w.w1t + (size_t)(j0 + c) * H + 8 * q;
  for (int b = 0; b < H / 32; ++b) {
    float x[8];
    bf8_to_f32(*(const uint4*)(xr + 32 * b), x);
    uint4 wv[4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) wv[jt] = *(const uint4*)(wr + (size_t)jt * 16 * H + 32 * b);
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) acc[jt] = chain8(wv[jt], x, acc[jt]);
  }
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
    *(float4*)(F + (size_t)row * J + j0 + jt * 16 + 4 * q) = float4{acc[jt][0], acc[jt][1], acc[jt][2], acc[jt][3]};
}

// ---------------------------------------------------------------- greedy decode
constexpr int XP = 640 + 4;  // LDS row pitch (floats) of staged B operands: conflict-free b128 reads
constexpr int HP = 320 + 4;

struct DecSmem {
  float X[DEC_ROWS][XP];   // layer input [x | h_prev] (chain-permuted); y1 for the joint
  float Hs[DEC_ROWS][HP];  // layer output h (chain-permuted): next layer's x / the joint's g
  float L[DEC_ROWS][NLAB_PAD + 1];
  int time[DEC_ROWS], added[DEC_ROWS], idx[DEC_ROWS], preg[DEC_ROWS], slot[DEC_ROWS];
  int fin[DEC_ROWS], need[DEC_ROWS], flen[DEC_ROWS], list[DEC_ROWS];
  int nlist, all_done;
};

// hc row layout: [slot][4][320] with parts 0:h0 1:h1 2:c0 3:c1
__device__ __forceinline__ float* hc_part(float* hc, int row, int slot, int part) {
  return hc + ((size_t)row * 2 + slot) * 4 * P + part * P;
}

// One prediction LSTM layer for the listed rows (lstm_amx_bf16 cell): gates = (b_ih+b_hh) +
// chain over [x | h_prev] of the gate-interleaved weights; c fp32, h bf16.
__device__ void pred_layer(const DecArgs& a, DecSmem& s, int layer, int r0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const uint16_t* W = a.w.wp[layer];
  const float* bias = a.w.bp_lstm[layer];
  const float* xrow = &s.X[c][8 * q];
  const int nl = s.nlist;
  for (int gt = wave * 2; gt < PG4 / 16; gt += 8) {  // two gate tiles (independent chains) per pass
    v4f acc0, acc1;
    {
      const float4 b0 = *(const float4*)(bias + gt * 16 + 4 * q);
      const float4 b1 = *(const float4*)(bias + (gt + 1) * 16 + 4 * q);
      acc0 = v4f{b0.x, b0.y, b0.z, b0.w};
      acc1 = v4f{b1.x, b1.y, b1.z, b1.w};
    }
    const uint16_t* w0 = W + (size_t)(gt * 16 + c) * 640 + 8 * q;
    const uint16_t* w1 = w0 + 16 * 640;
    for (int b = 0; b < 640 / 32; ++b) {
      const uint4 wa = *(const uint4*)(w0 + 32 * b);
      const uint4 wb = *(const uint4*)(w1 + 32 * b);
      float x[8];
      *(float4*)&x[0] = *(const float4*)(xrow + 32 * b);
      *(float4*)&x[4] = *(const float4*)(xrow + 32 * b + 4);
      acc0 = chain8(wa, x, acc0);
      acc1 = chain8(wb, x, acc1);
    }
    // epilogue: lane (q, c) holds i,f,g,o of unit gt*4+q (and (gt+1)*4+q) for listed row c
    if (c < nl) {
      const int m = s.list[c], row = r0 + m, sl = s.slot[m];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const v4f g = half ? acc1 : acc0;
        const int u = (gt + half) * 4 + q;
        const float ig = det_sigmoid(g[0]), fg = det_sigmoid(g[1]), gg = det_tanh(g[2]), og = det_sigmoid(g[3]);
        const float cp = hc_part(a.hc, row, sl, 2 + layer)[u];
        const float cn = fg * cp + ig * gg;
        const float hh = bf_round(og * det_tanh(cn));
        hc_part(a.hc, row, sl ^ 1, 2 + layer)[u] = cn;
        hc_part(a.hc, row, sl ^ 1, layer)[u] = hh;
        s.Hs[c][chain_pos(u)] = hh;
      }
    }
  }
}

__global__ void __launch_bounds__(256) greedy_decode_kernel(DecArgs a) {
  __shared__ DecSmem s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int r0 = blockIdx.x * DEC_ROWS;

  if (tid < DEC_ROWS) {
    const int row = r0 + tid;
    const int fl = row < a.N ? a.f_lens[row] : 0;
    s.flen[tid] = fl;
    s.time[tid] = 0; s.added[tid] = 0; s.idx[tid] = -1; s.preg[tid] = SOS; s.slot[tid] = 0;
    s.fin[tid] = (fl <= 0); s.need[tid] = 1;
  }
  // committed state (slot 0) starts at zero (decoder.py:67-78 / metadata.cpp:25-30)
  for (int i = tid; i < DEC_ROWS * 4 * P; i += 256) {
    const int m = i / (4 * P), k = i % (4 * P);
    if (r0 + m < a.Npad) hc_part(a.hc, r0 + m, 0, 0)[k] = 0.0f;
  }
  for (int i = tid; i < DEC_ROWS * a.max_res; i += 256) {
    const int m = i / a.max_res;
    if (r0 + m < a.N) a.res[(size_t)(r0 + m) * a.max_res + i % a.max_res] = SOS;
  }
  __syncthreads();

  for (int iter = 0; iter < a.max_iter; ++iter) {
    if (tid == 0) {
      int nl = 0, done = 1;
      for (int m = 0; m < DEC_ROWS; ++m) {
        if (!s.fin[m]) {
          done = 0;
          if (s.need[m]) s.list[nl++] = m;
        }
      }
      s.nlist = nl;
      s.all_done = done;
    }
    __syncthreads();
    if (s.all_done) break;

    if (s.nlist > 0) {
      // ---- prediction for rows whose committed state changed (Prediction.forward)
      for (int i = tid; i < DEC_ROWS * 640; i += 256) {
        const int mi = i / 640, k = i % 640;
        float v = 0.0f;
        if (mi < s.nlist) {
          const int m = s.list[mi];
          if (k < P) {
            const int g = s.preg[m];
            v = (g == SOS) ? 0.0f : bf2f(a.w.embed[g * P + k]);  // SOS -> zero embedding
          } else {
            v = hc_part(a.hc, r0 + m, s.slot[m], 0)[k - P];
          }
        }
        s.X[mi][chain_pos(k)] = v;
      }
      __syncthreads();
      pred_layer(a, s, 0, r0);
      __syncthreads();
      for (int i = tid; i < DEC_ROWS * 640; i += 256) {
        const int mi = i / 640, k = i % 640;
        float v = 0.0f;
        if (mi < s.nlist) {
          // chain_pos maps k<320 within the first 320 positions, so Hs copies straight over
          v = (k < P) ? s.Hs[mi][k] : hc_part(a.hc, r0 + s.list[mi], s.slot[s.list[mi]], 1)[k - P];
        }
        s.X[mi][k < P ? k : chain_pos(k)] = v;
      }
      __syncthreads();
      pred_layer(a, s, 1, r0);
      __syncthreads();
      // ---- G = b_p + g . W1p^T for the new candidates (joint prediction half)
      for (int jt = wave; jt < J / 16; jt += 4) {
        const float4 b0 = *(const float4*)(a.w.bp + jt * 16 + 4 * q);
        v4f acc = v4f{b0.x, b0.y, b0.z, b0.w};
        const uint16_t* wr = a.w.w1p + (size_t)(jt * 16 + c) * P + 8 * q;
        const float* xr = &s.Hs[c][8 * q];
        for (int b = 0; b < P / 32; ++b) {
          float x[8];
          *(float4*)&x[0] = *(const float4*)(xr + 32 * b);
          *(float4*)&x[4] = *(const float4*)(xr + 32 * b + 4);
          acc = chain8(*(const uint4*)(wr + 32 * b), x, acc);
        }
        if (c < s.nlist)
          *(float4*)(a.G + (size_t)(r0 + s.list[c]) * J + jt * 16 + 4 * q) = float4{acc[0], acc[1], acc[2], acc[3]};
      }
      __syncthreads();
      if (tid < s.nlist) s.need[s.list[tid]] = 0;
    }

    // ---- joint: y1 = bf16(relu(F[t] + G)), logits = b2 + y1 . W2^T
    for (int i = tid; i < DEC_ROWS * J; i += 256) {
      const int m = i / J, k = i % J, row = r0 + m;
      float v = 0.0f;
      if (!s.fin[m]) {
        const float sum = a.F[((size_t)s.time[m] * a.Npad + row) * J + k] + a.G[(size_t)row * J + k];
        v = bf_round(sum > 0.0f ? sum : 0.0f);
      }
      s.X[m][chain_pos(k)] = v;
    }
    __syncthreads();
    if (wave < 2) {
      const float4 b0 = *(const float4*)(a.w.b2 + wave * 16 + 4 * q);
      v4f acc = v4f{b0.x, b0.y, b0.z, b0.w};
      const uint16_t* wr = a.w.w2 + (size_t)(wave * 16 + c) * J + 8 * q;
      const float* xr = &s.X[c][8 * q];
      for (int b = 0; b < J / 32; ++b) {
        float x[8];
        *(float4*)&x[0] = *(const float4*)(xr + 32 * b);
        *(float4*)&x[4] = *(const float4*)(xr + 32 * b + 4);
        acc = chain8(*(const uint4*)(wr + 32 * b), x, acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) s.L[c][wave * 16 + 4 * q + r] = acc[r];
    }
    __syncthreads();
    // ---- greedy update (greedy_decode_update; decoder.py:137-167), one thread per row
    if (tid < DEC_ROWS && !s.fin[tid]) {
      const int m = tid;
      int best = 0;
      float bv = s.L[m][0];
      for (int j = 1; j < NLAB; ++j)
        if (s.L[m][j] > bv) { bv = s.L[m][j]; best = j; }  // torch.argmax: first maximum
      if (best != BLANK && s.added[m] != MAXSYM) {
        const int id = ++s.idx[m];
        if (id < a.max_res) a.res[(size_t)(r0 + m) * a.max_res + id] = best;
        s.added[m]++;
        s.preg[m] = best;
        s.slot[m] ^= 1;  // commit the candidate (hg, cg) as (pre_hg, pre_cg)
        s.need[m] = 1;
      } else {
        int t = s.time[m] + 1;
        if (t >= s.flen[m]) s.fin[m] = 1;
        if (t > s.flen[m] - 1) t = s.flen[m] - 1;
        s.time[m] = t;
        s.added[m] = 0;
      }
    }
    __syncthreads();
  }
  if (tid < DEC_ROWS && r0 + tid < a.N) a.res_len[r0 + tid] = s.idx[tid] + 1;
}

int launch_joint_trans(const DecWeights& w, const uint16_t* fperm, const int32_t* f_lens, float* F, int Tp,
                       int Npad, hipStream_t st) {
  if (Tp <= 0) return 0;
  hipLaunchKernelGGL(joint_trans_kernel, dim3(J / 64, (Tp * Npad) / 64), dim3(256), 0, st, w, fperm, f_lens, F, Npad);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_greedy_decode(const DecArgs& a, hipStream_t st) {
  const int nwg = (a.N + DEC_ROWS - 1) / DEC_ROWS;
  if (nwg <= 0) return 0;
  hipLaunchKernelGGL(greedy_decode_kernel, dim3(nwg), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rnnt
