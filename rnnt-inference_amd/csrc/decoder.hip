// decoder.hip -- prediction network, joint and greedy decode on CDNA4.
//
// Replaces intel_mlperf::lstm_amx_bf16, amx_linear_bf16_accum_relu, amx_linear_i16o32 and
// greedy_decode_update (reference modeling_rnnt.py:183-205, 259-289, 331-365) and the host
// decode loop of csrc/rnnt_model.hpp:92-124.  Every bf16 dot product runs on
// v_mfma_f32_16x16x32_bf16 in natural k order (instruction b covers k = 32b..32b+31, lane group
// q = lane>>4 holds k = 32b+8q..+7), chained through the accumulator from the bias; the CPU
// restatement defines these dot products as that instruction's accumulation (oracle
// mfma_group, pinned to hardware outputs by tests/test_mfma_model.py), so the decode is
// bit-exact with it and therefore token-identical.
//
// The greedy loop runs lock-step over the batch like the reference's (rnnt_model.hpp:92-124):
// per step, weight-stationary kernels run the prediction network for the rows that emitted,
// then one kernel does joint + argmax + greedy_decode_update for every live row, walking each
// row through its blank frames until it emits; the host only enqueues steps and polls a
// live-row counter one 32-step chunk behind (no per-step round trip).  Three exact shortcuts:
//   * the joint's encoder half F[t] = b_t + bf16(f_t).W1t^T depends only on the frame, so it is
//     one batched GEMM over all frames before the loop (launch_joint_trans);
//   * prediction(pre_g, pre_hg, pre_cg) depends only on state that changes on an emit, so it
//     (and the joint's prediction half G) is evaluated once per emit, not once per step;
//   * layer 0's input half b_ih + emb[g].W_ih^T depends only on the label: a [29][1280] table
//     computed once per engine with the same instruction sequence (launch_dec_xtab).
#include "rnnt_device.hpp"
#include "decoder.hpp"

namespace rnnt {

typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

__device__ __forceinline__ v4f mfma_bf16(const uint4 a, const uint4 b, const v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}
// 8 bf16-valued floats -> packed bf16 bits (exact: the values are bf16 already)
__device__ __forceinline__ uint4 pack8(const float4 lo, const float4 hi) {
  return uint4{(f2bits(lo.x) >> 16) | (f2bits(lo.y) & 0xffff0000u), (f2bits(lo.z) >> 16) | (f2bits(lo.w) & 0xffff0000u),
               (f2bits(hi.x) >> 16) | (f2bits(hi.y) & 0xffff0000u), (f2bits(hi.z) >> 16) | (f2bits(hi.w) & 0xffff0000u)};
}

// ---------------------------------------------------------------- layer-0 input table
// xtab[g][r] = b_ih0[r] + emb[g].W_ih0[r]^T (g < 28), xtab[28] = b_ih0 (SOS: zero embedding).
// One workgroup per 16 gate rows; one wave per 16 labels (rows 28..31 are zero embeddings).
__global__ void __launch_bounds__(128) dec_xtab_kernel(DecWeights w, float* __restrict__ xtab) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const int gt = blockIdx.x;
  const int g = wave * 16 + c;  // label of this lane's B column
  const float4 b = *(const float4*)(w.bih_p[0] + gt * 16 + 4 * q);
  v4f acc = v4f{b.x, b.y, b.z, b.w};
  const uint16_t* wr = w.wp[0] + (size_t)(gt * 16 + c) * 640 + 8 * q;  // W_ih half
  for (int kb = 0; kb < P / 32; ++kb) {
    const uint4 xv = g < 28 ? *(const uint4*)(w.embed + (size_t)g * P + 32 * kb + 8 * q) : uint4{0u, 0u, 0u, 0u};
    acc = mfma_bf16(*(const uint4*)(wr + 32 * kb), xv, acc);
  }
  if (g <= 28) *(float4*)(xtab + (size_t)g * PG4 + gt * 16 + 4 * q) = float4{acc[0], acc[1], acc[2], acc[3]};
}

// ---------------------------------------------------------------- F = b_t + f . W1t^T
// rows = (frame, batch row) pairs of fbf [Tp][Npad][1024] (bf16, natural k).  A workgroup owns
// 64 output columns j and 256 rows: the 64 x 1024 W1t slice is staged in LDS once and read as
// A fragments by 4 waves of 4 row tiles each (16 MFMA tiles per wave).
constexpr int JT_ROWS = 256;
constexpr int JT_PITCH = H + 8;  // bf16 elements per staged W1t row: +16 B, conflict-free b128 reads
__global__ void __launch_bounds__(256) joint_trans_kernel(DecWeights w, const uint16_t* __restrict__ fbf,
                                                          const int32_t* __restrict__ f_lens,
                                                          float* __restrict__ F, int Npad, int nrows) {
  extern __shared__ __attribute__((aligned(16))) uint16_t Ws[];  // [64][JT_PITCH]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int j0 = blockIdx.x * 64;
  const int row0 = blockIdx.y * JT_ROWS;
  // live 16-row tiles of this wave (row = t * Npad + n valid iff t < f_lens[n])
  bool live[4];
  bool any = false;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = row0 + wave * 64 + i * 16 + c;
    const int t = row / Npad, n = row % Npad;
    live[i] = __any(row < nrows && f_lens[n] > t);
    any |= live[i];
  }
  for (int i = tid; i < 64 * (H / 8); i += 256) {
    const int r = i / (H / 8), k8 = (i % (H / 8)) * 8;
    *(uint4*)(Ws + r * JT_PITCH + k8) = *(const uint4*)(w.w1t + (size_t)(j0 + r) * H + k8);
  }
  __syncthreads();
  if (!any) return;
  v4f acc[4][4];
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    const float4 b = *(const float4*)(w.bt + j0 + jt * 16 + 4 * q);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][jt] = v4f{b.x, b.y, b.z, b.w};
  }
  const uint16_t* xr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) xr[i] = fbf + (size_t)(row0 + wave * 64 + i * 16 + c) * H + 8 * q;
  for (int kb = 0; kb < H / 32; ++kb) {
    uint4 a[4], b[4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) a[jt] = *(const uint4*)(Ws + (jt * 16 + c) * JT_PITCH + 32 * kb + 8 * q);
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = live[i] ? *(const uint4*)(xr[i] + 32 * kb) : uint4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) acc[i][jt] = mfma_bf16(a[jt], b[i], acc[i][jt]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (!live[i]) continue;
    const int row = row0 + wave * 64 + i * 16 + c;
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
      *(float4*)(F + (size_t)row * J + j0 + jt * 16 + 4 * q) =
          float4{acc[i][jt][0], acc[i][jt][1], acc[i][jt][2], acc[i][jt][3]};
  }
}

// ---------------------------------------------------------------- greedy decode
// Lock-step over the batch, like the reference's loop (rnnt_model.hpp:92-124), but only the
// rows that emitted at the previous step re-run the prediction network:
//   pred(layer 0) -> pred(layer 1) -> G  for the listed rows      (weight-stationary grids)
//   joint + argmax + greedy update for every unfinished row -> next step's emit list

__device__ __forceinline__ float* hc_part(float* hc, int row, int slot, int part) {
  return hc + ((size_t)row * 2 + slot) * 4 * P + part * P;  // parts 0:h0 1:h1 2:c0 3:c1
}

__global__ void __launch_bounds__(256) dec_init_kernel(DecArgs a) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= a.Npad) return;
  const int fl = row < a.N ? a.f_lens[row] : 0;
  DecState& s = a.s;
  s.time[row] = 0; s.added[row] = 0; s.idx[row] = -1; s.preg[row] = SOS; s.slot[row] = 0;
  s.fin[row] = fl <= 0;
  float* h = hc_part(a.hc, row, 0, 0);
  for (int k = 0; k < 4 * P; ++k) h[k] = 0.0f;  // committed state starts at zero (metadata.cpp:25-30)
  if (fl > 0) {
    s.list[atomicAdd(&s.count[0], 1)] = row;  // every live row needs its first (SOS) prediction
    atomicAdd(s.unfinished, 1);
  }
}

// One prediction LSTM layer for the listed rows (lstm_amx_bf16 cell): gates =
// (b_ih + x.W_ih^T) + (b_hh + h.W_hh^T); c fp32, h bf16.  A workgroup (8 waves) owns 8*NT gate
// tiles; wave w holds tiles NT*w .. NT*w+NT-1: their W_hh (and, layer 1, W_ih) rows stay in
// registers for the launch (10 x 16 B per tile and chain per lane: NT = 2 for layer 0, whose
// input half comes from the label table, 1 for layer 1).  Grid: x = 80 / (8 NT) gate groups,
// y = row groups striding over the emit list's 16-row tiles.
constexpr int PRED_THREADS = 512;
#ifndef RNNT_PRED_RG
#define RNNT_PRED_RG 48
#endif
#ifndef RNNT_G_RG
#define RNNT_G_RG 96
#endif
#ifndef RNNT_JOINT_G
#define RNNT_JOINT_G 512
#endif
constexpr int PRED_ROW_GROUPS = RNNT_PRED_RG;
constexpr int G_ROW_GROUPS = RNNT_G_RG;
constexpr int JOINT_GROUPS = RNNT_JOINT_G;

template <int LAYER>
__global__ void __launch_bounds__(PRED_THREADS) dec_pred_kernel(DecArgs a, int parity) {
  constexpr int NT = LAYER ? 1 : 2;      // gate tiles per wave
  constexpr int KX = LAYER ? 2 * P : P;  // staged k: layer 1 [x | h], layer 0 [h]
  constexpr int XP = KX + 8;             // bf16 pitch: +16 B per row (conflict-free b128 reads)
  __shared__ __attribute__((aligned(16))) uint16_t X[16][XP];
  __shared__ int rows[16], slots[16], pregs[16];
  const DecState& s = a.s;
  const int cnt = s.count[parity];
  const int ntiles = (cnt + 15) >> 4;
  if ((int)blockIdx.y >= ntiles) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int* list = s.list + parity * a.Npad;
  const int t0 = (blockIdx.x * 8 + wave) * NT;  // this wave's gate tiles t0 .. t0 + NT - 1
  uint4 wh[NT][P / 32], wx[NT][LAYER ? P / 32 : 1];
  float4 bh[NT], bx[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    const uint16_t* wr = a.w.wp[LAYER] + (size_t)((t0 + tt) * 16 + c) * 640 + 8 * q;
#pragma unroll
    for (int b = 0; b < P / 32; ++b) wh[tt][b] = *(const uint4*)(wr + P + 32 * b);
    if (LAYER) {
#pragma unroll
      for (int b = 0; b < P / 32; ++b) wx[tt][b] = *(const uint4*)(wr + 32 * b);
      bx[tt] = *(const float4*)(a.w.bih_p[LAYER] + (t0 + tt) * 16 + 4 * q);
    }
    bh[tt] = *(const float4*)(a.w.bhh_p[LAYER] + (t0 + tt) * 16 + 4 * q);
  }
  for (int rt = blockIdx.y; rt < ntiles; rt += gridDim.y) {
    if (tid < 16) {
      const int row = (rt * 16 + tid < cnt) ? list[rt * 16 + tid] : -1;
      rows[tid] = row;
      slots[tid] = row >= 0 ? s.slot[row] : 0;
      pregs[tid] = row >= 0 ? s.preg[row] : SOS;
    }
    __syncthreads();
    // stage the listed rows' inputs as bf16: layer 0 h0 (committed slot); layer 1
    // [h0 of the candidate slot | h1 committed]
    for (int i = tid; i < 16 * (KX / 8); i += PRED_THREADS) {
      const int m = i / (KX / 8), k = (i % (KX / 8)) * 8, row = rows[m];
      uint4 v = uint4{0u, 0u, 0u, 0u};
      if (row >= 0) {
        const int sl = slots[m];
        const float* src = LAYER == 0 ? hc_part(a.hc, row, sl, 0) + k
                                      : (k < P ? hc_part(a.hc, row, sl ^ 1, 0) + k : hc_part(a.hc, row, sl, 1) + k - P);
        v = pack8(*(const float4*)src, *(const float4*)(src + 4));
      }
      *(uint4*)&X[m][k] = v;
    }
    __syncthreads();
    const int row = rows[c];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      v4f ah = v4f{bh[tt].x, bh[tt].y, bh[tt].z, bh[tt].w};
#pragma unroll
      for (int b = 0; b < P / 32; ++b) ah = mfma_bf16(wh[tt][b], *(const uint4*)&X[c][(LAYER ? P : 0) + 32 * b + 8 * q], ah);
      v4f ax;
      if (LAYER) {
        ax = v4f{bx[tt].x, bx[tt].y, bx[tt].z, bx[tt].w};
#pragma unroll
        for (int b = 0; b < P / 32; ++b) ax = mfma_bf16(wx[tt][b], *(const uint4*)&X[c][32 * b + 8 * q], ax);
      } else {
        const int g = pregs[c] == SOS ? 28 : pregs[c];
        const float4 xt = *(const float4*)(a.w.xtab + (size_t)g * PG4 + (t0 + tt) * 16 + 4 * q);
        ax = v4f{xt.x, xt.y, xt.z, xt.w};
      }
      if (row >= 0) {
        const v4f gs = ax + ah;
        const int sl = slots[c];
        const int u = (t0 + tt) * 4 + q;
        const float ig = det_sigmoid(gs[0]), fg = det_sigmoid(gs[1]), gg = det_tanh(gs[2]), og = det_sigmoid(gs[3]);
        const float cp = hc_part(a.hc, row, sl, 2 + LAYER)[u];
        const float cn = fg * cp + ig * gg;
        const float hh = bf_round_ftz(og * det_tanh(cn));
        hc_part(a.hc, row, sl ^ 1, 2 + LAYER)[u] = cn;
        hc_part(a.hc, row, sl ^ 1, LAYER)[u] = hh;
      }
    }
    __syncthreads();  // X / rows are restaged by the next tile
  }
}

// G = b_p + g . W1p^T for the listed rows' new candidates.  One workgroup (8 waves, 4 column
// tiles each: all 512 columns, weights in registers) per row group striding over 16-row
// tiles.  Also clears the other parity's emit list for the joint that follows.
constexpr int GXP = P + 8;
__global__ void __launch_bounds__(512) dec_g_kernel(DecArgs a, int parity) {
  __shared__ __attribute__((aligned(16))) uint16_t X[16][GXP];
  __shared__ int rows[16], slots[16];
  DecState& s = a.s;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) s.count[parity ^ 1] = 0;
  const int cnt = s.count[parity];
  const int ntiles = (cnt + 15) >> 4;
  if ((int)blockIdx.y >= ntiles) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int* list = s.list + parity * a.Npad;
  uint4 wv[4][P / 32];
  float4 b0[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int jt = wave * 4 + jj;
    const uint16_t* w0 = a.w.w1p + (size_t)(jt * 16 + c) * P + 8 * q;
#pragma unroll
    for (int b = 0; b < P / 32; ++b) wv[jj][b] = *(const uint4*)(w0 + 32 * b);
    b0[jj] = *(const float4*)(a.w.bp + jt * 16 + 4 * q);
  }
  for (int rt = blockIdx.y; rt < ntiles; rt += gridDim.y) {
    if (tid < 16) {
      const int row = (rt * 16 + tid < cnt) ? list[rt * 16 + tid] : -1;
      rows[tid] = row;
      slots[tid] = row >= 0 ? s.slot[row] : 0;
    }
    __syncthreads();
    for (int i = tid; i < 16 * (P / 8); i += 512) {
      const int m = i / (P / 8), k = (i % (P / 8)) * 8, row = rows[m];
      uint4 v = uint4{0u, 0u, 0u, 0u};
      if (row >= 0) {
        const float* src = hc_part(a.hc, row, slots[m] ^ 1, 1) + k;
        v = pack8(*(const float4*)src, *(const float4*)(src + 4));
      }
      *(uint4*)&X[m][k] = v;
    }
    __syncthreads();
    const int row = rows[c];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      v4f acc = v4f{b0[jj].x, b0[jj].y, b0[jj].z, b0[jj].w};
#pragma unroll
      for (int b = 0; b < P / 32; ++b) acc = mfma_bf16(wv[jj][b], *(const uint4*)&X[c][32 * b + 8 * q], acc);
      if (row >= 0)
        *(float4*)(a.G + (size_t)row * J + (wave * 4 + jj) * 16 + 4 * q) = float4{acc[0], acc[1], acc[2], acc[3]};
    }
    __syncthreads();
  }
}

// joint (y1 = bf16(relu(F[t] + G)), logits = b2 + y1.W2^T) + argmax + greedy_decode_update
// (decoder.py:137-167) for 16 rows per workgroup.  A blank (or a forced advance after
// max_symbols_per_step) moves the row to its next frame with the SAME prediction, so the
// workgroup evaluates up to RNNT_JOINT_ITERS frames per launch, stopping a row at its first
// emission (it then needs a new prediction: next step's emit list) or at its last frame; rows
// still in a blank run stay live for the next step.  Identical results for any cap; the cap
// trades lock-step steps against the length of each step.
#ifndef RNNT_JOINT_ITERS
#define RNNT_JOINT_ITERS 2
#endif
constexpr int YP = J + 8;
__global__ void __launch_bounds__(256) dec_joint_kernel(DecArgs a, int parity) {
  __shared__ __attribute__((aligned(16))) uint16_t X[16][YP];
  __shared__ float L[16][NLAB_PAD + 1];
  __shared__ float Lp[4][16][NLAB_PAD + 1];
  __shared__ int live[16], tidx[16];
  DecState& s = a.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  // logits = ((s0 + s1) + s2) + s3, s_b = y1[128b : 128b+128] . W2^T (s0 from b2): wave w runs
  // label half w&1 over k blocks 2(w>>1) and 2(w>>1)+1 as two independent 4-instruction chains
  const int lh = wave & 1, kb0 = 2 * (wave >> 1);
  uint4 wv[8];
  {
    const uint16_t* wr = a.w.w2 + (size_t)(lh * 16 + c) * J + 8 * q;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      wv[b] = *(const uint4*)(wr + 128 * kb0 + 32 * b);
      wv[4 + b] = *(const uint4*)(wr + 128 * (kb0 + 1) + 32 * b);
    }
  }
  v4f bias = v4f{0.0f, 0.0f, 0.0f, 0.0f};
  if (kb0 == 0) {
    const float4 b0 = *(const float4*)(a.w.b2 + lh * 16 + 4 * q);
    bias = v4f{b0.x, b0.y, b0.z, b0.w};
  }
  for (int rtile = blockIdx.x; rtile < (a.N + 15) / 16; rtile += gridDim.x) {
    const int r0 = rtile * 16;
    if (tid < 16) {
      const int row = r0 + tid;
      const int lv = (row < a.N) && !s.fin[row];
      live[tid] = lv;
      tidx[tid] = lv ? s.time[row] : 0;
    }
    __syncthreads();
    for (int it = 0; it < RNNT_JOINT_ITERS; ++it) {
      bool any = false;
#pragma unroll
      for (int m = 0; m < 16; ++m) any |= live[m] != 0;
      if (!any) break;
      for (int i = tid; i < 16 * (J / 8); i += 256) {
        const int m = i / (J / 8), k = (i % (J / 8)) * 8, row = r0 + m;
        uint4 v = uint4{0u, 0u, 0u, 0u};
        if (live[m]) {
          const float* fr = a.F + ((size_t)tidx[m] * a.Npad + row) * J + k;
          const float* gr = a.G + (size_t)row * J + k;
          float y[8];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const float4 f4 = *(const float4*)(fr + 4 * h);
            const float4 g4 = *(const float4*)(gr + 4 * h);
            const float s0 = f4.x + g4.x, s1 = f4.y + g4.y, s2 = f4.z + g4.z, s3 = f4.w + g4.w;
            y[4 * h + 0] = bf_round_ftz(s0 > 0.0f ? s0 : 0.0f);
            y[4 * h + 1] = bf_round_ftz(s1 > 0.0f ? s1 : 0.0f);
            y[4 * h + 2] = bf_round_ftz(s2 > 0.0f ? s2 : 0.0f);
            y[4 * h + 3] = bf_round_ftz(s3 > 0.0f ? s3 : 0.0f);
          }
          v = pack8(float4{y[0], y[1], y[2], y[3]}, float4{y[4], y[5], y[6], y[7]});
        }
        *(uint4*)&X[m][k] = v;
      }
      __syncthreads();
      {
        v4f s0 = bias, s1 = v4f{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          s0 = mfma_bf16(wv[b], *(const uint4*)&X[c][128 * kb0 + 32 * b + 8 * q], s0);
          s1 = mfma_bf16(wv[4 + b], *(const uint4*)&X[c][128 * (kb0 + 1) + 32 * b + 8 * q], s1);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          Lp[kb0][c][lh * 16 + 4 * q + r] = s0[r];
          Lp[kb0 + 1][c][lh * 16 + 4 * q + r] = s1[r];
        }
      }
      __syncthreads();
      for (int i = tid; i < 16 * NLAB_PAD; i += 256) {
        const int m = i / NLAB_PAD, j = i % NLAB_PAD;
        L[m][j] = ((Lp[0][m][j] + Lp[1][m][j]) + Lp[2][m][j]) + Lp[3][m][j];
      }
      __syncthreads();
      if (tid < 16 && live[tid]) {
        const int m = tid, row = r0 + m;
        int best = 0;
        float bv = L[m][0];
        for (int j = 1; j < NLAB; ++j)
          if (L[m][j] > bv) { bv = L[m][j]; best = j; }  // torch.argmax: first maximum
        if (best != BLANK && s.added[row] != MAXSYM) {
          const int id = ++s.idx[row];
          if (id < a.max_res) a.res[(size_t)row * a.max_res + id] = best;
          s.added[row]++;
          s.preg[row] = best;
          s.slot[row] ^= 1;  // commit the candidate (hg, cg) as (pre_hg, pre_cg)
          s.list[(parity ^ 1) * a.Npad + atomicAdd(&s.count[parity ^ 1], 1)] = row;
          live[m] = 0;
        } else {
          const int fl = a.f_lens[row];
          int t = tidx[m] + 1;
          if (t >= fl) {
            s.fin[row] = 1;
            atomicSub(s.unfinished, 1);
            live[m] = 0;
            t = fl - 1;
          }
          tidx[m] = t;
          s.time[row] = t;
          s.added[row] = 0;
        }
      }
      __syncthreads();
    }
    __syncthreads();  // live / tidx / X are reused by the next row tile
  }
}

__global__ void dec_finish_kernel(DecArgs a) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row < a.N) a.res_len[row] = a.s.idx[row] + 1;
}

int launch_greedy_decode(const DecArgs& a, int32_t* host_flags, hipEvent_t* evs, hipStream_t st) {
  const int rt = a.Npad / 16;
  if (hipMemsetAsync(a.s.count, 0, 4 * sizeof(int32_t), st) != hipSuccess) return -1;
  if (hipMemsetAsync(a.s.unfinished, 0, 4 * sizeof(int32_t), st) != hipSuccess) return -1;
  if (hipMemsetAsync(a.res, 0xff, (size_t)a.N * a.max_res * sizeof(int32_t), st) != hipSuccess) return -1;
  hipLaunchKernelGGL(dec_init_kernel, dim3((a.Npad + 255) / 256), dim3(256), 0, st, a);
  constexpr int CHUNK = 32;
  int step = 0, chunk = 0;
  int live_bound = a.N;  // unfinished rows at the end of the last chunk read back (an upper bound)
  bool done = false;
  while (!done && step < a.max_iter) {
    // row-tile workgroups per launch: one resident round, and no more than the live rows need
    const int lt = (live_bound + 15) / 16 < rt ? (live_bound + 15) / 16 : rt;
    const int lt1 = lt > 0 ? lt : 1;
    const int rg_pred = lt1 < PRED_ROW_GROUPS ? lt1 : PRED_ROW_GROUPS;
    const int rg_g = lt1 < G_ROW_GROUPS ? lt1 : G_ROW_GROUPS;
    const int rg_joint = rt < JOINT_GROUPS ? rt : JOINT_GROUPS;
    for (int i = 0; i < CHUNK && step < a.max_iter; ++i, ++step) {
      const int p = step & 1;
      hipLaunchKernelGGL(dec_pred_kernel<0>, dim3(PG4 / 256, rg_pred), dim3(PRED_THREADS), 0, st, a, p);
      hipLaunchKernelGGL(dec_pred_kernel<1>, dim3(PG4 / 128, rg_pred), dim3(PRED_THREADS), 0, st, a, p);
      hipLaunchKernelGGL(dec_g_kernel, dim3(1, rg_g), dim3(512), 0, st, a, p);
      hipLaunchKernelGGL(dec_joint_kernel, dim3(rg_joint), dim3(256), 0, st, a, p);
    }
    // poll the live-row counter one chunk behind, so the host never drains the queue
    if (hipMemcpyAsync(host_flags + (chunk & 1), a.s.unfinished, sizeof(int32_t), hipMemcpyDeviceToHost, st) !=
        hipSuccess)
      return -1;
    if (hipEventRecord(evs[chunk & 1], st) != hipSuccess) return -1;
    if (chunk > 0) {
      if (hipEventSynchronize(evs[(chunk - 1) & 1]) != hipSuccess) return -1;
      live_bound = host_flags[(chunk - 1) & 1];
      done = live_bound == 0;
    }
    ++chunk;
  }
  hipLaunchKernelGGL(dec_finish_kernel, dim3((a.N + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? step : -1;
}

int launch_joint_trans(const DecWeights& w, const uint16_t* fbf, const int32_t* f_lens, float* F, int Tp, int Npad,
                       hipStream_t st) {
  if (Tp <= 0) return 0;
  static bool attr = false;
  const int smem = 64 * JT_PITCH * 2;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)joint_trans_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, smem) !=
        hipSuccess)
      return -1;
    attr = true;
  }
  const int nrows = Tp * Npad;
  hipLaunchKernelGGL(joint_trans_kernel, dim3(J / 64, (nrows + JT_ROWS - 1) / JT_ROWS), dim3(256), smem, st, w, fbf,
                     f_lens, F, Npad, nrows);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dec_xtab(const DecWeights& w, float* xtab, hipStream_t st) {
  hipLaunchKernelGGL(dec_xtab_kernel, dim3(PG4 / 16), dim3(128), 0, st, w, xtab);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rnnt
