// decoder_f32.hip -- fp32 prediction network, joint and greedy decode (run_mode="f32").
//
// The reference's fp32 decoder: Prediction.forward with `P.lstm` (models/modeling_rnnt.py:183-205),
// Joint.forward's fp32 branch `linear1_trans(f) += linear1_pred(g); relu; linear2` (:285-288) and
// GreedyDecoder.greedy_decode_f32 (models/decoder.py:102-169), with the CPU restatement's
// arithmetic (oracle/rnnt_oracle.c pred_row / joint_F / joint_G / joint_logits, bf16 = 0):
// every dot product a k-ordered fp32 fma chain from its bias, run as a chain of
// v_mfma_f32_16x16x4_f32 (chain_f32.hpp), Cephes-exp sigmoid / tanh.  Bit-exact with the
// restatement, which is pinned to the reference's own fp32 greedy decode (tests/golden).
//
// Schedule: the greedy loop in lock-step over the batch (TorchModel::decode's loop,
// csrc/rnnt_model.hpp:92-124).  Per step three launches: prediction layer 0, layer 1 (for every
// unfinished row: the prediction is a pure function of the committed state, so recomputing it
// each step returns the value the restatement caches), and the joint + argmax + greedy update
// per 16-row tile.  F = b_t + f.W1t^T is one GEMM over every frame up front.  This path exists
// for the fp32 configuration (BASELINE config 1) and as the GPU fp32 reference of the accuracy
// check; the int8 + bf16 path is the throughput path (decoder.hip).
#include "chain_f32.hpp"
#include "decoder_f32.hpp"

namespace rnnt {

__global__ void dec32_init_kernel(DecF32Args a) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= a.Npad) return;
  a.s.time[n] = 0;
  a.s.added[n] = 0;
  a.s.idx[n] = -1;
  a.s.preg[n] = SOS;
  const int fin = (n >= a.N || a.f_lens[n] <= 0) ? 1 : 0;  // decoder.py:106 (f_lens == 0: finished)
  a.s.fin[n] = fin;
  if (!fin) atomicAdd(a.s.unfinished, 1);
  const size_t NP = (size_t)a.Npad * P;
  for (int l = 0; l < 2; ++l)
    for (int k = 0; k < P; ++k) {
      a.s.ph[l * NP + (size_t)n * P + k] = 0.0f;
      a.s.pc[l * NP + (size_t)n * P + k] = 0.0f;
    }
}

// One prediction LSTM layer (P = 320) for 64 rows x 64 gate rows per workgroup: wave = one
// 16-row gate tile (units 4gt..4gt+3, gates i,f,g,o), 4 batch tiles.  Layer 0's input is the
// embedding row of the last emitted label (row 28 = the zeroed SOS embedding), layer 1's the
// candidate layer-0 h just computed.
template <int L>
__global__ void __launch_bounds__(256) dec32_pred_kernel(DecF32Args a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const int gt = blockIdx.x * 4 + wave;
  const int n0 = blockIdx.y * 64;
  {  // nothing to do for a tile of finished rows
    const int n = n0 + lane;
    const bool live = n < a.N && !a.s.fin[n];
    if (!__any(live)) return;
  }
  const size_t NP = (size_t)a.Npad * P;
  const float* bx[4];
  const float* bh[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + j * 16 + c;
    if (L == 0) {
      const int g = a.s.preg[n];
      bx[j] = a.w.emb + (size_t)(g < 0 ? 28 : g) * P + 8 * q;
    } else {
      bx[j] = a.s.gh + (size_t)n * P + 8 * q;
    }
    bh[j] = a.s.ph + L * NP + (size_t)n * P + 8 * q;
  }
  const float4 bi = *(const float4*)(a.w.bih[L] + gt * 16 + 4 * q);
  const float4 bhv = *(const float4*)(a.w.bhh[L] + gt * 16 + 4 * q);
  v4f ax[4], ah[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ax[j] = v4f{bi.x, bi.y, bi.z, bi.w};
    ah[j] = v4f{bhv.x, bhv.y, bhv.z, bhv.w};
  }
  const int row = gt * 16 + c;
  chain_rows<4>(a.w.wih[L] + (size_t)row * P + 8 * q, bx, P, ax);
  chain_rows<4>(a.w.whh[L] + (size_t)row * P + 8 * q, bh, P, ah);
  const int u = gt * 4 + q;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + j * 16 + c;
    if (n >= a.N || a.s.fin[n]) continue;
    const float ig = det_sigmoid(ax[j][0] + ah[j][0]);
    const float fg = det_sigmoid(ax[j][1] + ah[j][1]);
    const float gg = det_tanh(ax[j][2] + ah[j][2]);
    const float og = det_sigmoid(ax[j][3] + ah[j][3]);
    const size_t o = L * NP + (size_t)n * P;
    const float cn = fg * a.s.pc[o + u] + ig * gg;
    a.s.gc[o + u] = cn;
    a.s.gh[o + chain_pos(u)] = og * det_tanh(cn);
  }
}

// Joint + argmax + greedy update for 16 rows (decoder.py:125-167 / oracle_greedy_decode):
// G = b_p + g.W1p^T (each wave 8 of the 32 16-column tiles), y1 = relu(F[time] + G) staged in
// LDS, logits = b2 + y1.W2^T (two 16-label tiles), first-maximum argmax over the 29 labels,
// then emit (res append, commit the candidate prediction state) or advance.
__global__ void __launch_bounds__(256) dec32_joint_kernel(DecF32Args a) {
  __shared__ __attribute__((aligned(16))) float y1s[16][J];
  __shared__ float Ls[16][NLAB_PAD + 1];
  __shared__ int emit[16];
  __shared__ int any;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int n0 = blockIdx.x * 16;
  if (tid == 0) any = 0;
  __syncthreads();
  if (tid < 16 && n0 + tid < a.N && !a.s.fin[n0 + tid]) any = 1;
  __syncthreads();
  if (!any) return;
  const size_t NP = (size_t)a.Npad * P;
  {
    const float* arow = a.s.gh + NP + (size_t)(n0 + c) * P + 8 * q;  // candidate layer-1 h = g
    const float* b[8];
    v4f acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int col = (wave * 8 + t) * 16 + c;
      b[t] = a.w.w1p + (size_t)col * P + 8 * q;
      const float bb = a.w.bp[col];
      acc[t] = v4f{bb, bb, bb, bb};
    }
    chain_rows<8>(arow, b, P, acc);
    // lane (q, c): acc[t][i] = G[row 4q + i][column (wave*8 + t)*16 + c]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * q + i, n = n0 + r;
      const float* Fr = a.F + ((size_t)a.s.time[n] * a.Npad + n) * J;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int col = (wave * 8 + t) * 16 + c;
        const float s = Fr[col] + acc[t][i];
        y1s[r][chain_pos(col)] = s > 0.0f ? s : 0.0f;
      }
    }
  }
  __syncthreads();
  if (wave < 2) {
    const float* ar = &y1s[c][0] + 8 * q;
    const float* bw[1] = {a.w.w2 + (size_t)(16 * wave + c) * J + 8 * q};
    const float bb = a.w.b2[16 * wave + c];
    v4f l[1] = {v4f{bb, bb, bb, bb}};
    chain_rows<1>(ar, bw, J, l);
#pragma unroll
    for (int i = 0; i < 4; ++i) Ls[4 * q + i][16 * wave + c] = l[0][i];
  }
  __syncthreads();
  if (tid < 16) {
    const int n = n0 + tid;
    int e = 0;
    if (n < a.N && !a.s.fin[n]) {
      int best = 0;
      float bv = Ls[tid][0];
      for (int j = 1; j < NLAB; ++j)
        if (Ls[tid][j] > bv) { bv = Ls[tid][j]; best = j; }  // torch.argmax: first maximum
      if (best != BLANK && a.s.added[n] != MAXSYM) {
        const int id = ++a.s.idx[n];
        if (id < a.max_res) a.res[(size_t)n * a.max_res + id] = best;
        a.s.added[n]++;
        a.s.preg[n] = best;
        e = 1;
      } else {
        const int fl = a.f_lens[n];
        int t = a.s.time[n] + 1;
        if (t >= fl) {
          a.s.fin[n] = 1;
          atomicSub(a.s.unfinished, 1);
          t = fl - 1;
        }
        a.s.time[n] = t;
        a.s.added[n] = 0;
      }
    }
    emit[tid] = e;
  }
  __syncthreads();
  // commit the emitting rows' candidate state (pre_hg/pre_cg <- hg/cg, decoder.py:147-151)
  for (int i = tid; i < 16 * 2 * P; i += 256) {
    const int r = i / (2 * P), rem = i % (2 * P), l = rem / P, k = rem % P;
    if (emit[r]) {
      const size_t o = l * NP + (size_t)(n0 + r) * P + k;
      a.s.ph[o] = a.s.gh[o];
      a.s.pc[o] = a.s.gc[o];
    }
  }
}

__global__ void dec32_finish_kernel(DecF32Args a) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n < a.N) a.res_len[n] = a.s.idx[n] + 1;
}

// intel_mlperf::lstm, one layer (modeling_rnnt.py:204, the run_mode="f32" prediction LSTM) for
// n_pad rows on natural-layout operands: the same two k-ordered chains as dec32_pred_kernel
// (b_ih + x.W_ih^T and b_hh + h.W_hh^T, v_mfma_f32_16x16x4_f32), with each lane's chain-ordered
// operands (natural k = 32 blk + 4 i + q, i = 0..7) gathered from the rows; then the cell.
__global__ void __launch_bounds__(256) op_lstm_f32_kernel(DecF32Weights w, int L, const float* __restrict__ x,
                                                          const float* __restrict__ h_in,
                                                          const float* __restrict__ c_in, float* __restrict__ h_out,
                                                          float* __restrict__ c_out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const int gt = blockIdx.x * 4 + wave;
  const int n0 = blockIdx.y * 64;
  const float4 bi = *(const float4*)(w.bih[L] + gt * 16 + 4 * q);
  const float4 bh = *(const float4*)(w.bhh[L] + gt * 16 + 4 * q);
  v4f ax[4], ah[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ax[j] = v4f{bi.x, bi.y, bi.z, bi.w};
    ah[j] = v4f{bh.x, bh.y, bh.z, bh.w};
  }
  const float* wx = w.wih[L] + (size_t)(gt * 16 + c) * P + 8 * q;
  const float* wh = w.whh[L] + (size_t)(gt * 16 + c) * P + 8 * q;
  for (int blk = 0; blk < P / 32; ++blk) {
    const float4 x0 = *(const float4*)(wx + 32 * blk), x1 = *(const float4*)(wx + 32 * blk + 4);
    const float4 h0 = *(const float4*)(wh + 32 * blk), h1 = *(const float4*)(wh + 32 * blk + 4);
    const float wxv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    const float whv[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const size_t r = (size_t)(n0 + j * 16 + c) * P + 32 * blk + q;
      float xv[8], hv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xv[i] = x[r + 4 * i];
        hv[i] = h_in[r + 4 * i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        ax[j] = MFMA4(wxv[i], xv[i], ax[j]);
        ah[j] = MFMA4(whv[i], hv[i], ah[j]);
      }
    }
  }
  const int u = gt * 4 + q;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const size_t o = (size_t)(n0 + j * 16 + c) * P + u;
    const float ig = det_sigmoid(ax[j][0] + ah[j][0]);
    const float fg = det_sigmoid(ax[j][1] + ah[j][1]);
    const float gg = det_tanh(ax[j][2] + ah[j][2]);
    const float og = det_sigmoid(ax[j][3] + ah[j][3]);
    const float cn = fg * c_in[o] + ig * gg;
    c_out[o] = cn;
    h_out[o] = og * det_tanh(cn);
  }
}

int launch_op_lstm_f32(const DecF32Weights& w, int layer, const float* x, const float* h_in, const float* c_in,
                       float* h_out, float* c_out, int n_pad, hipStream_t st) {
  if (n_pad <= 0 || n_pad % 64) return -1;
  hipLaunchKernelGGL(op_lstm_f32_kernel, dim3(PG4 / 64, n_pad / 64), dim3(256), 0, st, w, layer, x, h_in, c_in, h_out,
                     c_out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// F[r][j] = b_t[j] + chain_k fc[r][k] W1t[j][k] for all rows r of [Tp][Npad]: wave = one 16-column
// tile (A = W1t rows), 4 row tiles of 16 (B = frame rows).
__global__ void __launch_bounds__(256) dec32_F_kernel(DecF32Weights w, const float* __restrict__ fc,
                                                      float* __restrict__ F) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const int gt = blockIdx.x * 4 + wave;
  const size_t r0 = (size_t)blockIdx.y * 64;
  const float* b[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = fc + (r0 + j * 16 + c) * H + 8 * q;
  const float4 bt = *(const float4*)(w.bt + gt * 16 + 4 * q);
  v4f acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = v4f{bt.x, bt.y, bt.z, bt.w};
  chain_rows<4>(w.w1t + (size_t)(gt * 16 + c) * H + 8 * q, b, H, acc);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    *(float4*)(F + (r0 + j * 16 + c) * J + gt * 16 + 4 * q) = float4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
}

int launch_f32_joint_trans(const DecF32Weights& w, const float* fc, float* F, int Tp, int Npad, hipStream_t st) {
  if (Tp <= 0) return 0;
  if (Npad % 64) return -1;
  hipLaunchKernelGGL(dec32_F_kernel, dim3(J / 64, (unsigned)((size_t)Tp * Npad / 64)), dim3(256), 0, st, w, fc, F);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_greedy_decode_f32(const DecF32Args& a, int32_t* host_flags, hipEvent_t* evs, hipStream_t st) {
  if (a.Npad % 64 || a.N > a.Npad) return -1;
  if (hipMemsetAsync(a.s.unfinished, 0, sizeof(int32_t), st) != hipSuccess) return -1;
  if (hipMemsetAsync(a.res, 0xff, (size_t)a.N * a.max_res * sizeof(int32_t), st) != hipSuccess) return -1;
  hipLaunchKernelGGL(dec32_init_kernel, dim3((a.Npad + 63) / 64), dim3(64), 0, st, a);
  constexpr int CHUNK = 32;
  int step = 0, chunk = 0;
  bool done = false;
  while (!done && step < a.max_iter) {
    for (int i = 0; i < CHUNK && step < a.max_iter; ++i, ++step) {
      hipLaunchKernelGGL(dec32_pred_kernel<0>, dim3(PG4 / 64, a.Npad / 64), dim3(256), 0, st, a);
      hipLaunchKernelGGL(dec32_pred_kernel<1>, dim3(PG4 / 64, a.Npad / 64), dim3(256), 0, st, a);
      hipLaunchKernelGGL(dec32_joint_kernel, dim3(a.Npad / 16), dim3(256), 0, st, a);
    }
    if (hipMemcpyAsync(host_flags + (chunk & 1), a.s.unfinished, sizeof(int32_t), hipMemcpyDeviceToHost, st) !=
        hipSuccess)
      return -1;
    if (hipEventRecord(evs[chunk & 1], st) != hipSuccess) return -1;
    if (chunk > 0) {
      if (hipEventSynchronize(evs[(chunk - 1) & 1]) != hipSuccess) return -1;
      done = host_flags[(chunk - 1) & 1] == 0;
    }
    ++chunk;
  }
  hipLaunchKernelGGL(dec32_finish_kernel, dim3((a.N + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? step : -1;
}

}  // namespace rnnt
