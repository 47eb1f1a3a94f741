// decoder.hip -- prediction network, joint and greedy decode on CDNA4.
//
// Replaces intel_mlperf::lstm_amx_bf16, amx_linear_bf16_accum_relu, amx_linear_i16o32 and
// greedy_decode_update (reference modeling_rnnt.py:183-205, 259-289, 331-365) and the host
// decode loop of csrc/rnnt_model.hpp:92-124.  Every dot product is an fp32 k-ordered fmaf
// chain on bf16-valued operands, computed with v_mfma_f32_16x16x4_f32 (probe-verified to be
// bit-identical to a sequential fmaf chain), so the decode is bit-exact with the CPU
// restatement and therefore token-identical.
//
// The greedy loop runs lock-step over the batch like the reference's (rnnt_model.hpp:92-124):
// per step, weight-stationary kernels run the prediction network for the rows that emitted,
// then one kernel does joint + argmax + greedy_decode_update for every live row, walking each
// row through its blank frames until it emits; the host only enqueues steps and polls a
// live-row counter one 32-step chunk behind (no per-step round trip).  Two algebraic shortcuts, both exact:
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
// Lock-step over the batch, like the reference's loop (rnnt_model.hpp:92-124), but only the
// rows that emitted at the previous step re-run the prediction network:
//   pred(layer 0) -> pred(layer 1) -> G  for the listed rows      (weight-stationary grids)
//   joint + argmax + greedy update for every unfinished row -> next step's emit list
constexpr int XP = 640 + 4;  // LDS row pitch (floats) of staged B operands: conflict-free b128 reads
constexpr int GP = 320 + 4;
constexpr int YP = 512 + 4;

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
// (b_ih + chain over x) + (b_hh + chain over h_prev); c fp32, h bf16.  A workgroup (8 waves)
// owns PRED_TILES gate tiles; wave w runs tile w % PRED_TILES's x chain (first half of the
// waves) or h chain (second half) -- 80 chained MFMAs and 10 KB of weights per wave, held in
// registers for the launch -- and the h-chain partials meet the x chains in LDS.  Grid: x =
// 1280 / (16 PRED_TILES) gate groups, y = row groups striding over the emit list's 16-row
// tiles (one resident round).
constexpr int PRED_TILES = 4;
constexpr int PRED_THREADS = PRED_TILES * 2 * 64;
#ifndef RNNT_PRED_RG
#define RNNT_PRED_RG 25
#endif
#ifndef RNNT_G_RG
#define RNNT_G_RG 96
#endif
#ifndef RNNT_JOINT_G
#define RNNT_JOINT_G 512
#endif
// decode grids are kept small: every resident decode workgroup, even an idle one, keeps an
// encoder tick workgroup (a whole CU) of the batch in flight beside it from starting
constexpr int PRED_ROW_GROUPS = RNNT_PRED_RG;
constexpr int G_ROW_GROUPS = RNNT_G_RG;
constexpr int JOINT_GROUPS = RNNT_JOINT_G;
__global__ void __launch_bounds__(PRED_THREADS) dec_pred_kernel(DecArgs a, int layer, int parity) {
  __shared__ __attribute__((aligned(16))) float X[16][XP];
  __shared__ v4f Hp[PRED_TILES][64];
  __shared__ int rows[16], slots[16], pregs[16];
  const DecState& s = a.s;
  const int cnt = s.count[parity];
  const int ntiles = (cnt + 15) >> 4;
  if ((int)blockIdx.y >= ntiles) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int tile = wave % PRED_TILES, part = wave / PRED_TILES;  // part 0: x chain from b_ih, 1: h from b_hh
  const int* list = s.list + parity * a.Npad;
  const int gt = blockIdx.x * PRED_TILES + tile;
  // k blocks of [W_ih | W_hh]: part p reads blocks 10p .. 10p+9 (offset p*320 in the row)
  const uint16_t* w0 = a.w.wp[layer] + (size_t)(gt * 16 + c) * 640 + part * P + 8 * q;
  uint4 wv[P / 32];
#pragma unroll
  for (int b = 0; b < P / 32; ++b) {
#ifdef RNNT_DEV_PRED_NOWLOAD
    wv[b] = uint4{(uint32_t)b, 0u, 0u, 0u};
#else
    wv[b] = *(const uint4*)(w0 + 32 * b);
#endif
  }
  const float4 bias = *(const float4*)((part ? a.w.bhh_p[layer] : a.w.bih_p[layer]) + gt * 16 + 4 * q);
  for (int rt = blockIdx.y; rt < ntiles; rt += gridDim.y) {
    if (tid < 16) {
      const int row = (rt * 16 + tid < cnt) ? list[rt * 16 + tid] : -1;
      rows[tid] = row;
      slots[tid] = row >= 0 ? s.slot[row] : 0;
      pregs[tid] = row >= 0 ? s.preg[row] : SOS;
    }
    __syncthreads();
    // stage [x | h_prev] for the 16 listed rows: 16 x 160 float4 groups
#ifdef RNNT_DEV_PRED_NOSTAGE
    for (int i = tid; i < 0; i += PRED_THREADS) {
#else
    for (int i = tid; i < 16 * 160; i += PRED_THREADS) {
#endif
      const int mi = i / 160, k = (i % 160) * 4, row = rows[mi];
      float4 v = float4{0.0f, 0.0f, 0.0f, 0.0f};
      if (row >= 0) {
        const int sl = slots[mi];
        if (layer == 0) {
          if (k < P) {
            const int g = pregs[mi];
            if (g != SOS) {  // SOS -> zero embedding (modeling_rnnt.py:195-200)
              const uint2 e2 = *(const uint2*)(a.w.embed + g * P + k);
              v = float4{bits2f(e2.x << 16), bits2f(e2.x & 0xffff0000u), bits2f(e2.y << 16), bits2f(e2.y & 0xffff0000u)};
            }
          } else {
            v = *(const float4*)(hc_part(a.hc, row, sl, 0) + k - P);
          }
        } else {
          v = (k < P) ? *(const float4*)(hc_part(a.hc, row, sl ^ 1, 0) + k) : *(const float4*)(hc_part(a.hc, row, sl, 1) + k - P);
        }
      }
      X[mi][chain_pos(k)] = v.x;
      X[mi][chain_pos(k + 1)] = v.y;
      X[mi][chain_pos(k + 2)] = v.z;
      X[mi][chain_pos(k + 3)] = v.w;
    }
    __syncthreads();
    const float* xr = &X[c][part * P + 8 * q];
    v4f acc = v4f{bias.x, bias.y, bias.z, bias.w};
#ifndef RNNT_DEV_PRED_NOMFMA
#pragma unroll
    for (int b = 0; b < P / 32; ++b) {
      float x[8];
      *(float4*)&x[0] = *(const float4*)(xr + 32 * b);
      *(float4*)&x[4] = *(const float4*)(xr + 32 * b + 4);
      acc = chain8(wv[b], x, acc);
    }
#else
    asm volatile("" ::"v"(wv[0].x), "v"(wv[9].w), "v"(xr[0]));
#endif
    if (part) Hp[tile][lane] = acc;
    __syncthreads();
    const int row = rows[c];
    if (!part && row >= 0) {
      const v4f g = acc + Hp[tile][lane];
      const int sl = slots[c];
      const int u = gt * 4 + q;
      const float ig = det_sigmoid(g[0]), fg = det_sigmoid(g[1]), gg = det_tanh(g[2]), og = det_sigmoid(g[3]);
      const float cp = hc_part(a.hc, row, sl, 2 + layer)[u];
      const float cn = fg * cp + ig * gg;
      const float hh = bf_round(og * det_tanh(cn));
      hc_part(a.hc, row, sl ^ 1, 2 + layer)[u] = cn;
      hc_part(a.hc, row, sl ^ 1, layer)[u] = hh;
    }
    __syncthreads();  // X / rows / Hp are restaged by the next tile
  }
}

// G = b_p + g . W1p^T for the listed rows' new candidates.  Grid: x = 64-column group (one
// 16-column tile per wave, its weights in registers), y = row groups striding over 16-row
// tiles (one resident round: 8 x 96).  Also clears the other parity's emit list for the
// joint that follows.
__global__ void __launch_bounds__(256) dec_g_kernel(DecArgs a, int parity) {
  __shared__ __attribute__((aligned(16))) float X[16][GP];
  __shared__ int rows[16], slots[16];
  DecState& s = a.s;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) s.count[parity ^ 1] = 0;
  const int cnt = s.count[parity];
  const int ntiles = (cnt + 15) >> 4;
  if ((int)blockIdx.y >= ntiles) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int* list = s.list + parity * a.Npad;
  const int jt = blockIdx.x * 4 + wave;
  const uint16_t* w0 = a.w.w1p + (size_t)(jt * 16 + c) * P + 8 * q;
  uint4 wv[P / 32];
#pragma unroll
  for (int b = 0; b < P / 32; ++b) wv[b] = *(const uint4*)(w0 + 32 * b);
  const float4 b0 = *(const float4*)(a.w.bp + jt * 16 + 4 * q);
  for (int rt = blockIdx.y; rt < ntiles; rt += gridDim.y) {
    if (tid < 16) {
      const int row = (rt * 16 + tid < cnt) ? list[rt * 16 + tid] : -1;
      rows[tid] = row;
      slots[tid] = row >= 0 ? s.slot[row] : 0;
    }
    __syncthreads();
    for (int i = tid; i < 16 * (P / 4); i += 256) {
      const int mi = i / (P / 4), k = (i % (P / 4)) * 4, row = rows[mi];
      const float4 v = row >= 0 ? *(const float4*)(hc_part(a.hc, row, slots[mi] ^ 1, 1) + k) : float4{0.0f, 0.0f, 0.0f, 0.0f};
      X[mi][chain_pos(k)] = v.x;
      X[mi][chain_pos(k + 1)] = v.y;
      X[mi][chain_pos(k + 2)] = v.z;
      X[mi][chain_pos(k + 3)] = v.w;
    }
    __syncthreads();
    v4f acc = v4f{b0.x, b0.y, b0.z, b0.w};
    const float* xr = &X[c][8 * q];
#pragma unroll
    for (int b = 0; b < P / 32; ++b) {
      float x[8];
      *(float4*)&x[0] = *(const float4*)(xr + 32 * b);
      *(float4*)&x[4] = *(const float4*)(xr + 32 * b + 4);
      acc = chain8(wv[b], x, acc);
    }
    const int row = rows[c];
    if (row >= 0) *(float4*)(a.G + (size_t)row * J + jt * 16 + 4 * q) = float4{acc[0], acc[1], acc[2], acc[3]};
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
__global__ void __launch_bounds__(256) dec_joint_kernel(DecArgs a, int parity) {
  __shared__ __attribute__((aligned(16))) float X[16][YP];
  __shared__ float L[16][NLAB_PAD + 1];
  __shared__ float Lp[4][16][NLAB_PAD + 1];
  __shared__ int live[16], tidx[16];
  DecState& s = a.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
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
    for (int i = tid; i < 16 * (J / 4); i += 256) {
      const int m = i / (J / 4), k = (i % (J / 4)) * 4, row = r0 + m;
      float4 v = float4{0.0f, 0.0f, 0.0f, 0.0f};
      if (live[m]) {
        const float4 f4 = *(const float4*)(a.F + ((size_t)tidx[m] * a.Npad + row) * J + k);
        const float4 g4 = *(const float4*)(a.G + (size_t)row * J + k);
        const float s0 = f4.x + g4.x, s1 = f4.y + g4.y, s2 = f4.z + g4.z, s3 = f4.w + g4.w;
        v = float4{bf_round(s0 > 0.0f ? s0 : 0.0f), bf_round(s1 > 0.0f ? s1 : 0.0f), bf_round(s2 > 0.0f ? s2 : 0.0f),
                   bf_round(s3 > 0.0f ? s3 : 0.0f)};
      }
      X[m][chain_pos(k)] = v.x;
      X[m][chain_pos(k + 1)] = v.y;
      X[m][chain_pos(k + 2)] = v.z;
      X[m][chain_pos(k + 3)] = v.w;
    }
    __syncthreads();
    {  // logits = ((s0 + s1) + s2) + s3, s_b = y1[128b : 128b+128] . W2^T (s0 from b2): wave w
       // runs label half w&1 over k blocks 2(w>>1) and 2(w>>1)+1 as two independent chains
      const int lh = wave & 1, kb0 = 2 * (wave >> 1);
      const uint16_t* wr = a.w.w2 + (size_t)(lh * 16 + c) * J + 8 * q;
      const float* xr = &X[c][8 * q];
      uint4 wv[8];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        wv[b] = *(const uint4*)(wr + 128 * kb0 + 32 * b);
        wv[4 + b] = *(const uint4*)(wr + 128 * (kb0 + 1) + 32 * b);
      }
      v4f s0 = v4f{0.0f, 0.0f, 0.0f, 0.0f}, s1 = s0;
      if (kb0 == 0) {
        const float4 b0 = *(const float4*)(a.w.b2 + lh * 16 + 4 * q);
        s0 = v4f{b0.x, b0.y, b0.z, b0.w};
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        float x0[8], x1[8];
        *(float4*)&x0[0] = *(const float4*)(xr + 128 * kb0 + 32 * b);
        *(float4*)&x0[4] = *(const float4*)(xr + 128 * kb0 + 32 * b + 4);
        *(float4*)&x1[0] = *(const float4*)(xr + 128 * (kb0 + 1) + 32 * b);
        *(float4*)&x1[4] = *(const float4*)(xr + 128 * (kb0 + 1) + 32 * b + 4);
        s0 = chain8(wv[b], x0, s0);
        s1 = chain8(wv[4 + b], x1, s1);
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
  // row-tile workgroups per column group, sized so each launch is ONE resident round:
  // 20 x 25 for the prediction layers (2 x 8 waves per CU), 8 x 96 for G (3 per CU)
  const int rg_pred = rt < PRED_ROW_GROUPS ? rt : PRED_ROW_GROUPS, rg_g = rt < G_ROW_GROUPS ? rt : G_ROW_GROUPS;
  const int rg_joint = rt < JOINT_GROUPS ? rt : JOINT_GROUPS;
  if (hipMemsetAsync(a.s.count, 0, 4 * sizeof(int32_t), st) != hipSuccess) return -1;
  if (hipMemsetAsync(a.s.unfinished, 0, 4 * sizeof(int32_t), st) != hipSuccess) return -1;
  if (hipMemsetAsync(a.res, 0xff, (size_t)a.N * a.max_res * sizeof(int32_t), st) != hipSuccess) return -1;
  hipLaunchKernelGGL(dec_init_kernel, dim3((a.Npad + 255) / 256), dim3(256), 0, st, a);
  constexpr int CHUNK = 32;
  int step = 0, chunk = 0;
  bool done = false;
  while (!done && step < a.max_iter) {
    for (int i = 0; i < CHUNK && step < a.max_iter; ++i, ++step) {
      const int p = step & 1;
      hipLaunchKernelGGL(dec_pred_kernel, dim3(PG4 / (16 * PRED_TILES), rg_pred), dim3(PRED_THREADS), 0, st, a, 0, p);
      hipLaunchKernelGGL(dec_pred_kernel, dim3(PG4 / (16 * PRED_TILES), rg_pred), dim3(PRED_THREADS), 0, st, a, 1, p);
      hipLaunchKernelGGL(dec_g_kernel, dim3(J / 64, rg_g), dim3(256), 0, st, a, p);
      hipLaunchKernelGGL(dec_joint_kernel, dim3(rg_joint), dim3(256), 0, st, a, p);
    }
    // poll the live-row counter one chunk behind, so the host never drains the queue
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
  hipLaunchKernelGGL(dec_finish_kernel, dim3((a.N + 255) / 256), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? step : -1;
}

int launch_joint_trans(const DecWeights& w, const uint16_t* fperm, const int32_t* f_lens, float* F, int Tp,
                       int Npad, hipStream_t st) {
  if (Tp <= 0) return 0;
  hipLaunchKernelGGL(joint_trans_kernel, dim3(J / 64, (Tp * Npad) / 64), dim3(256), 0, st, w, fperm, f_lens, F, Npad);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}



}  // namespace rnnt
