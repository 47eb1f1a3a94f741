// decoder_ops.hip -- operator-level prediction / joint / greedy-update kernels.
//
// The fused device loop (decoder.hip) is what the engine runs; these kernels back the
// individual torch.ops.intel_mlperf operators the reference's Python decode loop calls
// (models/decoder.py:171-212 greedy_decode_quant), with the same arithmetic as the fused loop
// and the CPU restatement (oracle pred_row / joint_F / joint_G / joint_logits), so an op-by-op
// loop produces the same tokens:
//   lstm_amx_bf16              modeling_rnnt.py:202   -> op_lstm_bf16_kernel (one layer per launch)
//   amx_linear_bf16_accum_relu modeling_rnnt.py:269-275 -> op_joint_hidden_kernel
//   amx_linear_i16o32          modeling_rnnt.py:280-283 -> op_joint_logits_kernel
//   greedy_decode_update       modeling_rnnt.py:331-365 -> op_greedy_update_kernel
// Row tiles are 16 rows; every dot product is a bf16 MFMA chain (v_mfma_f32_16x16x32_bf16,
// natural k order, from the bias) exactly as in the fused loop.
#include "decoder_ops.hpp"
#include "rnnt_device.hpp"

namespace rnnt {

typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
__device__ __forceinline__ v4f mfma_bf16o(const uint4 a, const uint4 b, const v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}
// acc + chain over nblk 32-k blocks: w = this lane's A row at k offset 8q, x = its B row (LDS)
__device__ __forceinline__ v4f chain_blocks(const uint16_t* w, const uint16_t* x, int nblk, v4f acc) {
  for (int b = 0; b < nblk; ++b) acc = mfma_bf16o(*(const uint4*)(w + 32 * b), *(const uint4*)(x + 32 * b), acc);
  return acc;
}

constexpr int OXP = 640 + 16;  // LDS pitch (bf16) of staged [x | h] rows (+32 B: conflict-free b128 reads)
constexpr int OFP = 1024 + 16;  // staged f rows
constexpr int OGP = 320 + 16;   // staged g rows
constexpr int OYP = 512 + 16;  // staged y1 rows (+32 B: conflict-free ds_read_b128 fragments)

// one prediction LSTM layer: gates = (b_ih + x.W_ih) + (b_hh + h.W_hh); c fp32, h bf16.
// Grid: x = 10 groups of 8 gate tiles (2 per wave), y = 16-row tiles.
__global__ void __launch_bounds__(256) op_lstm_bf16_kernel(DecWeights w, int layer, const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ h_in, const float* __restrict__ c_in,
                                                           uint16_t* __restrict__ h_out, float* __restrict__ c_out) {
  __shared__ __attribute__((aligned(16))) uint16_t X[16][OXP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int r0 = blockIdx.y * 16;
  for (int i = tid; i < 16 * 640; i += 256) {
    const int m = i / 640, k = i % 640;
    const uint16_t v = k < P ? x[(size_t)(r0 + m) * P + k] : h_in[(size_t)(r0 + m) * P + k - P];
    X[m][k] = (v & 0x7f80u) ? v : (uint16_t)(v & 0x8000u);  // subnormal bf16 -> 0 (MFMA contract)
  }
  __syncthreads();
  const int gt = blockIdx.x * 8 + wave * 2;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int t = gt + half;
    const uint16_t* wr = w.wp[layer] + (size_t)(t * 16 + c) * 640 + 8 * q;
    const float4 bi = *(const float4*)(w.bih_p[layer] + t * 16 + 4 * q);
    const float4 bh = *(const float4*)(w.bhh_p[layer] + t * 16 + 4 * q);
    v4f ax = chain_blocks(wr, &X[c][8 * q], P / 32, v4f{bi.x, bi.y, bi.z, bi.w});
    v4f ah = chain_blocks(wr + P, &X[c][P + 8 * q], P / 32, v4f{bh.x, bh.y, bh.z, bh.w});
    const v4f g = ax + ah;
    const int u = t * 4 + q, row = r0 + c;
    const float ig = det_sigmoid(g[0]), fg = det_sigmoid(g[1]), gg = det_tanh(g[2]), og = det_sigmoid(g[3]);
    const float cn = fg * c_in[(size_t)row * P + u] + ig * gg;
    c_out[(size_t)row * P + u] = cn;
    h_out[(size_t)row * P + u] = f2bf_ftz(og * det_tanh(cn));
  }
}

// y1 = bf16(relu(F + G)), F = b_t + bf16(f).W1t^T, G = b_p + g.W1p^T.  Grid: x = 8 groups of 64
// columns (one 16-column tile per wave), y = 16-row tiles.
__global__ void __launch_bounds__(256) op_joint_hidden_kernel(DecWeights w, const float* __restrict__ f,
                                                              const uint16_t* __restrict__ g, uint16_t* __restrict__ y1) {
  __shared__ __attribute__((aligned(16))) uint16_t Fx[16][OFP];
  __shared__ __attribute__((aligned(16))) uint16_t Gx[16][OGP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int r0 = blockIdx.y * 16;
  for (int i = tid; i < 16 * H; i += 256) {
    const int m = i / H, k = i % H;
    Fx[m][k] = f2bf_ftz(f[(size_t)(r0 + m) * H + k]);
  }
  for (int i = tid; i < 16 * P; i += 256) {
    const int m = i / P, k = i % P;
    const uint16_t v = g[(size_t)(r0 + m) * P + k];
    Gx[m][k] = (v & 0x7f80u) ? v : (uint16_t)(v & 0x8000u);
  }
  __syncthreads();
  const int jt = blockIdx.x * 4 + wave;
  const float4 bt = *(const float4*)(w.bt + jt * 16 + 4 * q), bp = *(const float4*)(w.bp + jt * 16 + 4 * q);
  const v4f F = chain_blocks(w.w1t + (size_t)(jt * 16 + c) * H + 8 * q, &Fx[c][8 * q], H / 32, v4f{bt.x, bt.y, bt.z, bt.w});
  const v4f G = chain_blocks(w.w1p + (size_t)(jt * 16 + c) * P + 8 * q, &Gx[c][8 * q], P / 32, v4f{bp.x, bp.y, bp.z, bp.w});
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float s = F[r] + G[r];
    y1[(size_t)(r0 + c) * J + jt * 16 + 4 * q + r] = f2bf_ftz(s > 0.0f ? s : 0.0f);
  }
}

// logits [rows][32] = b2 + y1.W2^T as 4 blocked chains of 128 k combined in order (the fused
// joint's contract); columns 29..31 are exact zeros (zero weights and bias).
__global__ void __launch_bounds__(256) op_joint_logits_kernel(DecWeights w, const uint16_t* __restrict__ y1,
                                                              float* __restrict__ logits) {
  __shared__ __attribute__((aligned(16))) uint16_t X[16][OYP];
  __shared__ float Lp[4][16][NLAB_PAD + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int r0 = blockIdx.x * 16;
  for (int i = tid; i < 16 * J; i += 256) {
    const int m = i / J, k = i % J;
    const uint16_t v = y1[(size_t)(r0 + m) * J + k];
    X[m][k] = (v & 0x7f80u) ? v : (uint16_t)(v & 0x8000u);
  }
  __syncthreads();
  const int lh = wave & 1, kb0 = 2 * (wave >> 1);
  const uint16_t* wr = w.w2 + (size_t)(lh * 16 + c) * J + 8 * q;
  v4f s0 = v4f{0.0f, 0.0f, 0.0f, 0.0f};
  if (kb0 == 0) {
    const float4 b = *(const float4*)(w.b2 + lh * 16 + 4 * q);
    s0 = v4f{b.x, b.y, b.z, b.w};
  }
  s0 = chain_blocks(wr + 128 * kb0, &X[c][128 * kb0 + 8 * q], 4, s0);
  const v4f s1 = chain_blocks(wr + 128 * (kb0 + 1), &X[c][128 * (kb0 + 1) + 8 * q], 4, v4f{0.0f, 0.0f, 0.0f, 0.0f});
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    Lp[kb0][c][lh * 16 + 4 * q + r] = s0[r];
    Lp[kb0 + 1][c][lh * 16 + 4 * q + r] = s1[r];
  }
  __syncthreads();
  for (int i = tid; i < 16 * NLAB_PAD; i += 256) {
    const int m = i / NLAB_PAD, j = i % NLAB_PAD;
    logits[(size_t)(r0 + m) * NLAB_PAD + j] = ((Lp[0][m][j] + Lp[1][m][j]) + Lp[2][m][j]) + Lp[3][m][j];
  }
}

// greedy_decode_update (spec: decoder.py:125-167), one thread per row; finished = time_idx >=
// f_lens (see GreedyUpdateArgs).
__global__ void op_greedy_update_kernel(GreedyUpdateArgs a) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= a.n) return;
  const int fl = a.f_lens[n];
  if (a.time_idx[n] >= fl) return;  // finished
  const int sym = a.sym64 ? (int)((const int64_t*)a.symbols)[n] : ((const int32_t*)a.symbols)[n];
  if (sym != BLANK && a.symbols_added[n] != MAXSYM) {  // 4. emit
    const int id = ++a.res_idx[n];
    if (id < a.max_res) a.res[(size_t)n * a.max_res + id] = sym;
    a.symbols_added[n]++;
    a.pre_g[n] = sym;
    for (int l = 0; l < 2; ++l)
      for (int k = 0; k < P; ++k) {
        const size_t o = (size_t)n * P + k;
        a.pre_hg[l][o] = a.hg[l][o];
        a.pre_cg[l][o] = a.cg[l][o];
      }
  } else {  // 5. advance
    const int t = a.time_idx[n] + 1;
    a.time_idx[n] = t;  // t >= fl: finished (the spec's finish |= time >= f_lens)
    const int tf = t < fl ? t : fl - 1;  // the spec clamps time to eos before the gather
    for (int k = 0; k < H; ++k) a.fi[(size_t)n * H + k] = a.f[((size_t)tf * a.f_batch + n) * H + k];
    a.symbols_added[n] = 0;
  }
}

int launch_op_lstm_bf16(const DecWeights& w, int layer, const uint16_t* x, const uint16_t* h_in, const float* c_in,
                        uint16_t* h_out, float* c_out, int n_pad, hipStream_t st) {
  hipLaunchKernelGGL(op_lstm_bf16_kernel, dim3(PG4 / 128, n_pad / 16), dim3(256), 0, st, w, layer, x, h_in, c_in, h_out,
                     c_out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_op_joint_hidden(const DecWeights& w, const float* f, const uint16_t* g, uint16_t* y1, int n_pad,
                           hipStream_t st) {
  hipLaunchKernelGGL(op_joint_hidden_kernel, dim3(J / 64, n_pad / 16), dim3(256), 0, st, w, f, g, y1);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_op_joint_logits(const DecWeights& w, const uint16_t* y1, float* logits, int n_pad, hipStream_t st) {
  hipLaunchKernelGGL(op_joint_logits_kernel, dim3(n_pad / 16), dim3(256), 0, st, w, y1, logits);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_op_greedy_update(const GreedyUpdateArgs& a, hipStream_t st) {
  if (a.n <= 0) return 0;
  hipLaunchKernelGGL(op_greedy_update_kernel, dim3((a.n + 127) / 128), dim3(128), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rnnt
