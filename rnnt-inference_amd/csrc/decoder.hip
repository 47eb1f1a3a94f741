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
// The step is latency-bound (four dependent launches), so each kernel keeps its chain of
// dependent memory round trips short: emit-list entries carry (row, slot, label), the list
// entries of a workgroup's first tile are loaded beside the list length, the cell state is
// fetched beside the input staging, and the joint walks a compact list of unfinished rows.
#include <cstdlib>
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
// emit-list entry: row | committed slot << 24 | label-table index << 25 (28 = SOS)
__device__ __forceinline__ int emit_entry(int row, int slot, int label) { return row | (slot << 24) | (label << 25); }
// The row goes through an opaque v_and: ROCm 7.2's AMDGPU backend miscompiles a 64-bit multiply
// of (x & 0xffffff) by a constant that is not a power of two -- it matches a 24-bit multiply
// (which ignores the high byte, so the mask is dropped as redundant) and then widens it to
// v_mad_u64_u32, which multiplies all 32 bits: `base + (size_t)entry_row(e) * 1280` would be
// addressed with the slot and label bits still in place (tools/probe/probe_mul24.hip; guarded by
// tests/test_isa_lint.py).
__device__ __forceinline__ int entry_row(int e) {
  int r;
  asm("v_and_b32 %0, 0xffffff, %1" : "=v"(r) : "v"(e));
  return r;
}
__device__ __forceinline__ int entry_slot(int e) { return (e >> 24) & 1; }
__device__ __forceinline__ int entry_label(int e) { return (e >> 25) & 31; }
// list counters: DecState::count = {emit p0, live p0, emit p1, live p1} -- one parity's two
// counters adjacent, so the joint appends to both with one 64-bit atomic
__host__ __device__ constexpr int EMIT_N(int p) { return 2 * p; }
__host__ __device__ constexpr int LIVE_N(int p) { return 2 * p + 1; }
// live-list entry: a row still decoding with the greedy state the joint reads and updates, so the
// joint's update needs no dependent state loads (the DecState arrays are still written: they are
// the state the op-level entry points, the stream calls and dec_finish read)
__device__ __forceinline__ int4 live_entry(int row, int slot, int added, int time, int flen, int idx) {
  return int4{row | (slot << 24) | (added << 25), time | (flen << 16), idx, 0};
}

// development instrumentation (-DRNNT_DEV_STAMPS, tools/build_variants.sh stamps): thread 0 of
// each working workgroup of the step kernels records s_memrealtime (100 MHz) at kernel start,
// once its list entries are known, after the input staging and after its first tile.
#ifdef RNNT_DEV_STAMPS
__device__ unsigned long long g_st[1 << 22];
__device__ unsigned int g_st_n;
#define ST_MARK(v) unsigned long long v = threadIdx.x == 0 ? __builtin_amdgcn_s_memrealtime() : 0ull
#define ST_SET(v) if (threadIdx.x == 0 && v == 0ull) v = __builtin_amdgcn_s_memrealtime()
#define ST_FLUSH(kid, a0, a1, a2, a3)                                                  \
  if (threadIdx.x == 0) {                                                              \
    const unsigned k_ = atomicAdd(&g_st_n, 1u);                                        \
    if (k_ < (1u << 22) / 6) {                                                         \
      g_st[6 * k_] = (kid); g_st[6 * k_ + 1] = blockIdx.x + 65536ull * blockIdx.y;     \
      g_st[6 * k_ + 2] = a0; g_st[6 * k_ + 3] = a1; g_st[6 * k_ + 4] = a2;             \
      g_st[6 * k_ + 5] = (a3) ? (a3) : __builtin_amdgcn_s_memrealtime();               \
    }                                                                                  \
  }
#else
#define ST_MARK(v)
#define ST_SET(v)
#define ST_FLUSH(kid, a0, a1, a2, a3)
#endif

// Workgroup barrier over LDS only: waits for this wave's LDS operations, not for its global loads
// and stores (a __syncthreads fence waits for every outstanding memory operation: in the step
// kernels that serialised the weight-slice loads behind the list / staging round trips and
// drained each tile's global stores).  Uniform control flow only.
// development bounds checks (-DRNNT_DEC_CHECK: the host emulation, tools/emu, and
// tools/build_variants.sh): a failed check sets its bit in g_dec_err and the access is skipped.
// In the shipping build every check is `true`, so a check may only ever wrap a bounds assertion,
// never a condition the logic needs.
#ifdef RNNT_DEC_CHECK
__device__ unsigned int g_dec_err;
__device__ __forceinline__ bool dec_ok(bool c, int bit) {
  if (!c) atomicOr(&g_dec_err, 1u << bit);
  return c;
}
#else
__device__ __forceinline__ constexpr bool dec_ok(bool, int) { return true; }
#endif

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// XCD-aware decomposition of a 1-D grid of 8 * X * Y8 workgroups into (column group x, row group
// y < 8 * Y8): workgroup id goes to XCD id & 7 (round-robin dispatch), and all X column groups
// of a row group run on one XCD, so a row tile's inputs are fetched into one L2 (measured before:
// the column groups of a row tile spread over every XCD, each fetching the rows).
struct GridXY {
  int x, y, ny;
};
// One row group (a short list: the decode's tail) launches just X workgroups, dealt round-robin
// to the XCDs: the column groups' weight slices (up to 1.6 MB) then stream through all eight L2s
// instead of one, and the single row tile's inputs are small.
__device__ __forceinline__ GridXY xcd_grid(int X) {
  if ((int)gridDim.x == X) return GridXY{(int)blockIdx.x, 0, 1};
  const int id = blockIdx.x, t = id >> 3;
  return GridXY{t % X, (id & 7) + 8 * (t / X), 8 * (int)(gridDim.x / (8 * X))};
}
static inline int xcd_grid_size(int X, int rows) { return rows <= 1 ? X : 8 * X * ((rows + 7) / 8); }

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
constexpr int JT_PITCH = H + 16;  // bf16 per staged W1t row: +32 B, conflict-free ds_read_b128 (16-lane groups)
__global__ void __launch_bounds__(256) joint_trans_kernel(DecWeights w, const uint16_t* __restrict__ fbf,
                                                          const int32_t* __restrict__ f_lens,
                                                          float* __restrict__ F, int Npad, int nrows) {
  extern __shared__ __attribute__((aligned(16))) uint16_t Ws[];  // [64][JT_PITCH]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const GridXY gxy = xcd_grid(J / 64);
  if (gxy.y * JT_ROWS >= nrows) return;
  const int j0 = gxy.x * 64;
  const int row0 = gxy.y * JT_ROWS;
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
      __builtin_nontemporal_store(acc[i][jt], (v4f*)(F + (size_t)row * J + j0 + jt * 16 + 4 * q));
  }
}

// F as a 256 (j) x 256 (frame row) tile GEMM, staged like the encoder's tick kernel: both
// operands DMA'd into LDS as 128-byte row segments (64 k, two MFMA k steps; 8 whole cache lines
// per piece), two 64 KiB buffers, XOR-swizzled image (slot c ^ ((r >> 1) & 7)); 8 waves as
// 4 (j) x 2 (rows), each 64 j x 128 rows = 4 x 8 bf16 MFMA tiles.  Same per-element chain as
// joint_trans_kernel (bias first, natural k in 32-k instructions), so F is bit-identical.
// Grid: the two j tiles of a row tile sit on one XCD (frame rows fetched into one L2).
typedef __attribute__((address_space(3))) void jg_lds_void;
typedef __attribute__((address_space(1))) void jg_glb_void;
constexpr int JG_SMEM = 2 * 65536;
__global__ void __launch_bounds__(512, 1) joint_trans_gemm_kernel(DecWeights w, const uint16_t* __restrict__ fbf,
                                                                 const int32_t* __restrict__ f_lens,
                                                                 float* __restrict__ F, int Npad, int nrt) {
  extern __shared__ __attribute__((aligned(16))) int8_t jsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave & 3, wn = wave >> 2;
  const int q = lane >> 4, col = lane & 15;
  const int id = blockIdx.x, xcd = id & 7, rest = id >> 3;
  const int ct = rest & 1, rt = (rest >> 1) * 8 + xcd;
  if (rt >= nrt) return;
  const int j0 = ct * 256, row0 = rt * 256;
  const int t = row0 / Npad, n0 = row0 % Npad;  // Npad is a multiple of 256: one frame per tile
  const bool my_valid = f_lens[n0 + (tid & 255)] > t;
  if (!__syncthreads_or(my_valid)) return;
  // ---- staging: wave w moves A (W1t) pieces 4w..4w+3 and B (frame) pieces 4w..4w+3, piece p =
  // rows 8p..8p+7 x 128 B; lane l -> row 8p + (l >> 3), LDS slot l & 7 holding 16-B column
  // (l & 7) ^ ((row >> 1) & 7)
  const int r8 = lane >> 3, sl = lane & 7;
  const uint32_t gc0 = (uint32_t)(sl ^ ((r8 >> 1) & 7)) * 16, gc1 = (uint32_t)(sl ^ (((8 + r8) >> 1) & 7)) * 16;
  const uint32_t rl = (uint32_t)(32 * wave + r8);
  const uint32_t o0 = rl * (H * 2) + gc0, o1 = rl * (H * 2) + gc1;  // same row pitch (2 KiB) for both operands
  const char* abase = (const char*)(w.w1t + (size_t)j0 * H);
  const char* bbase = (const char*)(fbf + (size_t)row0 * H);
  auto issueA = [&](int s) __attribute__((always_inline)) {
    int8_t* st = jsm + (s & 1) * 65536 + wave * 4096;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((jg_glb_void*)(abase + (size_t)(8 * j) * (H * 2) + s * 128 + ((j & 1) ? o1 : o0)),
                                       (jg_lds_void*)(st + j * 1024), 16, 0, 0);
  };
  auto issueB = [&](int s) __attribute__((always_inline)) {
    int8_t* st = jsm + (s & 1) * 65536 + 32768 + wave * 4096;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((jg_glb_void*)(bbase + (size_t)(8 * j) * (H * 2) + s * 128 + ((j & 1) ? o1 : o0)),
                                       (jg_lds_void*)(st + j * 1024), 16, 0, 0);
  };
  v4f acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 b = *(const float4*)(w.bt + j0 + wm * 64 + i * 16 + 4 * q);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) acc[i][jj] = v4f{b.x, b.y, b.z, b.w};
  }
  const int sw = col >> 1;
  const int fa0 = (wm * 64 + col) * 128, fb0 = 32768 + (wn * 128 + col) * 128;
  constexpr int NS = H * 2 / 128;  // 16 stages of 64 k
  issueA(0);
  issueB(0);
  for (int s = 0; s < NS; ++s) {
    // this wave's pieces of stage s landed and every wave's reads of stage s-1 retired
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (s + 1 < NS) issueA(s + 1);
    const int8_t* st = jsm + (s & 1) * 65536;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int cs = ((kk * 4 + q) ^ sw) << 4;
      uint4 fra[4], frb[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) fra[i] = *(const uint4*)(st + fa0 + cs + i * 2048);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) frb[jj] = *(const uint4*)(st + fb0 + cs + jj * 2048);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) acc[i][jj] = mfma_bf16(fra[i], frb[jj], acc[i][jj]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (kk == 0 && s + 1 < NS) {
        issueB(s + 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  // F[row][j]: lane holds j = j0 + wm*64 + 16 i + 4q .. +3 of row row0 + wn*128 + 16 jj + col
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const int n = n0 + wn * 128 + jj * 16 + col;
    if (f_lens[n] <= t) continue;
    float* dst = F + (size_t)(row0 + wn * 128 + jj * 16 + col) * J + j0 + wm * 64 + 4 * q;
#pragma unroll
    for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(acc[i][jj], (v4f*)(dst + i * 16));
  }
}

// ---------------------------------------------------------------- greedy decode
// Lock-step over the batch, like the reference's loop (rnnt_model.hpp:92-124), but only the
// rows that emitted at the previous step re-run the prediction network:
//   pred(layer 0) -> pred(layer 1) -> G  for the emit list's rows   (weight-stationary grids)
//   joint + argmax + greedy update for the live list's rows -> next step's emit / live lists

__device__ __forceinline__ float* hc_part(float* hc, int row, int slot, int part) {
  return hc + ((size_t)row * 2 + slot) * 4 * P + part * P;  // parts 0:h0 1:h1 2:c0 3:c1
}
// the h parts hold bf16 (the contract rounds h to bf16 where it is produced): 320 bf16 in the
// first 640 bytes of the part, so the staging loads of the step kernels move half the bytes
__device__ __forceinline__ uint16_t* h_bf(float* hc, int row, int slot, int layer) {
  return (uint16_t*)hc_part(hc, row, slot, layer);
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
    s.list[atomicAdd(&s.count[EMIT_N(0)], 1)] = emit_entry(row, 0, 28);  // every live row needs its first (SOS) prediction
    s.live[atomicAdd(&s.count[LIVE_N(0)], 1)] = live_entry(row, 0, 0, 0, fl, -1);
  }
}

// Server continuous batching (PipelineState, metadata.cpp:97-194): rows are slots that keep their
// greedy state across calls.  A slot flagged in reset starts an utterance (the State::init /
// masked_fill_ values above, its result row refilled with -1); the others keep pre_g, the
// committed prediction state (slot) and res / idx, and only the per-call frame counters restart
// (TorchModel::decode zeroes symbols_added and time_idx every call, rnnt_model.hpp:95-98).  Every
// live slot re-runs the prediction of its committed state on pre_g -- the candidate the previous
// call already held, recomputed bit-identically (a pure function of that state).
__global__ void __launch_bounds__(256) dec_init_stream_kernel(DecArgs a, const int32_t* __restrict__ reset) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= a.Npad) return;
  const int fl = row < a.N ? a.f_lens[row] : 0;
  DecState& s = a.s;
  if (row >= a.N || reset[row]) {
    s.idx[row] = -1; s.preg[row] = SOS; s.slot[row] = 0;
    float* h = hc_part(a.hc, row, 0, 0);
    for (int k = 0; k < 4 * P; ++k) h[k] = 0.0f;
  }
  s.time[row] = 0; s.added[row] = 0;
  s.fin[row] = fl <= 0;
  if (fl > 0) {
    const int pg = s.preg[row];
    s.list[atomicAdd(&s.count[EMIT_N(0)], 1)] = emit_entry(row, s.slot[row], pg < 0 ? 28 : pg);
    s.live[atomicAdd(&s.count[LIVE_N(0)], 1)] = live_entry(row, s.slot[row], 0, 0, fl, s.idx[row]);
  }
}

// result rows of the slots flagged in reset refilled with -1 (one workgroup per row, coalesced)
__global__ void __launch_bounds__(256) dec_reset_res_kernel(int32_t* __restrict__ res, int max_res,
                                                            const int32_t* __restrict__ reset) {
  const int row = blockIdx.x;
  if (!reset[row]) return;
  for (int k = threadIdx.x; k < max_res; k += 256) res[(size_t)row * max_res + k] = -1;
}

// One prediction LSTM layer for the listed rows (lstm_amx_bf16 cell): gates =
// (b_ih + x.W_ih^T) + (b_hh + h.W_hh^T); c fp32, h bf16.  A workgroup (4 waves) owns 4 gate
// tiles, one per wave, whose W_hh (and, layer 1, W_ih) rows stay in registers for the launch
// (10 x 16 B per chain per lane; layer 0's input half comes from the label table).  Every
// launch reloads its weights, and one CU takes in only a few tens of GB/s, so the slice per
// workgroup is kept small (20-40 KB: in-kernel stamps showed 160-320 KB slices costing 12-20 us
// per launch).  Grid: x = 20 gate groups, y = row groups striding over the emit list's tiles.
constexpr int PRED_THREADS = 256;  // 4 waves, one gate tile each: 40 KB of weights per workgroup
// rows per workgroup iteration of the prediction / G kernels: 32 (two MFMA row tiles per weight
// fragment) with 24 / 48 row groups -- isolated greedy 69.5 -> 66.7 ms per query vs 16 rows and
// 48 / 96 groups (64 rows: 82 ms); the joint keeps 16-row tiles (JRT)
constexpr int DEC_RT = 32;
// row groups (grid y) of the prediction / G launches and workgroups of the joint, at most: round-2
// sweeps of 12-96 / 24-96 / 256-512 measured within +-1.5 %
constexpr int PRED_ROW_GROUPS = 24;
constexpr int G_ROW_GROUPS = 48;
constexpr int JOINT_GROUPS = 512;

// ---- stores of data another workgroup of the SAME launch reads (persistent mode, PS = true): written
// through (`sc1`: the line leaves the XCD's L2), 4- or 16-byte, as the MI355X guide's hand-off rows
// require (Guideline 16, the flow encoder's recipe: sc1 stores, every wave's vmcnt(0), a workgroup
// barrier, one relaxed agent-scope counter add; the consumer polls, acquires, meets at a barrier).
// PS = false: plain stores (the step kernels hand off at kernel boundaries).
typedef unsigned int dec_u32x4 __attribute__((ext_vector_type(4)));
#ifndef RNNT_EMU
template <bool PS>
__device__ __forceinline__ void st_b32(void* p, uint32_t v) {
  if (PS) __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *(uint32_t*)p = v;
}
template <bool PS>
__device__ __forceinline__ void st_b128(void* p, uint4 v) {
  if (PS) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, (short)0, 0x7ffffff0, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(dec_u32x4{v.x, v.y, v.z, v.w}, r, 0, 0, 16);  // aux 16 = sc1
  } else {
    *(uint4*)p = v;
  }
}
#else  // host emulation (tools/emu): the step kernels only, plain stores
template <bool PS>
inline void st_b32(void* p, uint32_t v) { *(uint32_t*)p = v; }
template <bool PS>
inline void st_b128(void* p, uint4 v) { *(uint4*)p = v; }
#endif

// One prediction LSTM layer for the emit list's rows (see dec_pred_kernel).  The body runs one
// launch's work: in the step kernel once, in the persistent decode once per step with the weight
// slice kept in registers across steps (wl: loaded).  X / ents_all: the caller's LDS.
template <int LAYER>
struct PredRegs {
  uint4 wh[P / 32], wx[LAYER ? P / 32 : 1];
  float4 bh, bx;
  bool wl = false;
};
constexpr int pred_xp(int layer) { return (layer ? 2 * P : P) + 16; }
template <int LAYER, int NW, bool PS, int RT = DEC_RT>
__device__ __forceinline__ void dec_pred_body(const DecArgs& a, int parity, const GridXY gxy,
                                              uint16_t (*X)[pred_xp(LAYER)], int (*ents_all)[RT], PredRegs<LAYER>& W) {
  constexpr int PRED_THREADS = NW * 64;
  constexpr int KX = LAYER ? 2 * P : P;  // staged k: layer 1 [x | h], layer 0 [h]
  constexpr int NK = PRED_THREADS / RT;  // row tiles whose list entries load up front
  constexpr int DEC_SUB = RT / 16;
  const DecState& s = a.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  ST_MARK(st0);
  const int* list = s.list + parity * a.Npad;
  // the entries of this workgroup's first NK row tiles load beside the list length (one round
  // trip for all of them; indices past Npad -- XCD rounding, long strides -- are guarded)
  const int i0 = (gxy.y + (tid / RT) * gxy.ny) * RT + tid % RT;
  const int e0 = i0 < a.Npad ? list[i0] : -1;
  const int cnt = s.count[EMIT_N(parity)];
  const int ntiles = (cnt + RT - 1) / RT;
  if (gxy.y >= ntiles) return;
  ents_all[tid / RT][tid % RT] = i0 < cnt ? e0 : -1;
  const int t0 = gxy.x * (PRED_THREADS / 64) + wave;  // this wave's gate tile
  for (int rt = gxy.y, it = 0; rt < ntiles; rt += gxy.ny, ++it) {
    int* ents = ents_all[it % NK];
    if (it >= NK && tid < RT)  // past the prefetched tiles (the slot's tile is done)
      ents[tid] = rt * RT + tid < cnt && dec_ok(rt * RT + tid < a.Npad, 3) ? list[rt * RT + tid] : -1;
    lds_barrier();
    ST_MARK(st1);
    // this lane's committed cell states (sub-tile st: row ents[16 st + c]) and, layer 0, its
    // label-table input halves, fetched beside the input staging
    float cp[DEC_SUB];
    float4 xt[DEC_SUB];
#pragma unroll
    for (int st = 0; st < DEC_SUB; ++st) {
      int ec = ents[16 * st + c];
      if (ec >= 0 && !dec_ok(entry_row(ec) < a.Npad && entry_label(ec) <= 28, 0)) ec = -1;
      cp[st] = ec >= 0 ? hc_part(a.hc, entry_row(ec), entry_slot(ec), 2 + LAYER)[t0 * 4 + q] : 0.0f;
      if (!LAYER) xt[st] = *(const float4*)(a.w.xtab + (size_t)(ec >= 0 ? entry_label(ec) : 28) * PG4 + t0 * 16 + 4 * q);
    }
    // stage the listed rows' inputs as bf16: layer 0 h0 (committed slot); layer 1
    // [h0 of the candidate slot | h1 committed]
    // every load of the tile first (one memory round trip); entries past the list end read row
    // 0 (a safe cached address) and stage zeros
    constexpr int NX = RT * (KX / 8), NIT = (NX + PRED_THREADS - 1) / PRED_THREADS;
    uint4 xv[NIT];
    int emv[NIT];
#pragma unroll
    for (int u = 0; u < NIT; ++u) {  // this thread's entries first: one LDS round trip, not one per load
      const int i = tid + PRED_THREADS * u;
      emv[u] = (NX % PRED_THREADS == 0 || i < NX) ? ents[i / (KX / 8)] : -1;
    }
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
      const int i = tid + PRED_THREADS * u;
      if (NX % PRED_THREADS == 0 || i < NX) {
        const int k = (i % (KX / 8)) * 8, em = emv[u];
        const int r = em >= 0 && dec_ok(entry_row(em) < a.Npad, 1) ? entry_row(em) : 0, smm = em >= 0 ? entry_slot(em) : 0;
        const uint16_t* src = LAYER == 0 ? h_bf(a.hc, r, smm, 0) + k
                                         : (k < P ? h_bf(a.hc, r, smm ^ 1, 0) + k : h_bf(a.hc, r, smm, 1) + k - P);
        xv[u] = *(const uint4*)src;
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the weight loads behind the input loads
    if (!W.wl) {
      W.wl = true;
      const uint16_t* wr = a.w.wp[LAYER] + (size_t)(t0 * 16 + c) * 640 + 8 * q;
#pragma unroll
      for (int b = 0; b < P / 32; ++b) W.wh[b] = *(const uint4*)(wr + P + 32 * b);
      if (LAYER) {
#pragma unroll
        for (int b = 0; b < P / 32; ++b) W.wx[b] = *(const uint4*)(wr + 32 * b);
        W.bx = *(const float4*)(a.w.bih_p[LAYER] + t0 * 16 + 4 * q);
      }
      W.bh = *(const float4*)(a.w.bhh_p[LAYER] + t0 * 16 + 4 * q);
    }
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
      const int i = tid + PRED_THREADS * u;
      if (NX % PRED_THREADS == 0 || i < NX) {
        const int m = i / (KX / 8), k = (i % (KX / 8)) * 8;
        *(uint4*)&X[m][k] = emv[u] >= 0 ? xv[u] : uint4{0u, 0u, 0u, 0u};
      }
    }
    lds_barrier();
    ST_MARK(st2);
    // the chains of every sub-tile (h, and x on layer 1) advance together, one k block at a
    // time, so each block's fragment reads overlap the previous block's MFMAs (sub-tiles past the
    // list end run on the staged zeros; their results are not stored).  Each chain is still the
    // contract's natural-k sequence from its bias.
    int ecs[DEC_SUB];
    v4f ahs[DEC_SUB], axs[DEC_SUB];
#pragma unroll
    for (int st = 0; st < DEC_SUB; ++st) {
      ecs[st] = ents[16 * st + c];
      ahs[st] = v4f{W.bh.x, W.bh.y, W.bh.z, W.bh.w};
      axs[st] = LAYER ? v4f{W.bx.x, W.bx.y, W.bx.z, W.bx.w} : v4f{xt[st].x, xt[st].y, xt[st].z, xt[st].w};
    }
#pragma unroll
    for (int b = 0; b < P / 32; ++b) {
#pragma unroll
      for (int st = 0; st < DEC_SUB; ++st) {
        const uint16_t* xr = &X[16 * st + c][8 * q];
        ahs[st] = mfma_bf16(W.wh[b], *(const uint4*)(xr + (LAYER ? P : 0) + 32 * b), ahs[st]);
        if (LAYER) axs[st] = mfma_bf16(W.wx[LAYER ? b : 0], *(const uint4*)(xr + 32 * b), axs[st]);
      }
    }
#pragma unroll
    for (int st = 0; st < DEC_SUB; ++st) {
      const int ec = ecs[st];
      const int row = ec >= 0 && dec_ok(entry_row(ec) < a.Npad, 2) ? entry_row(ec) : -1, sl = ec >= 0 ? entry_slot(ec) : 0;
      const v4f gs = axs[st] + ahs[st];
      const int u = t0 * 4 + q;
      const float ig = det_sigmoid(gs[0]), fg = det_sigmoid(gs[1]), gg = det_tanh(gs[2]), og = det_sigmoid(gs[3]);
      const float cn = fg * cp[st] + ig * gg;
      const float hh = bf_round_ftz(og * det_tanh(cn));
      const uint32_t hb = __float_as_uint(hh) >> 16;  // hh is bf16-exact
      if (PS) {
        // 4-byte write-through stores: units u (q even) and u + 1 (lane + 16, same row) in one word
        const uint32_t hpair = __shfl_xor(hb, 16);
        if (row >= 0) {
          st_b32<true>(hc_part(a.hc, row, sl ^ 1, 2 + LAYER) + u, __float_as_uint(cn));
          if ((q & 1) == 0) st_b32<true>(h_bf(a.hc, row, sl ^ 1, LAYER) + u, hb | (hpair << 16));
        }
      } else if (row >= 0) {
        hc_part(a.hc, row, sl ^ 1, 2 + LAYER)[u] = cn;
        h_bf(a.hc, row, sl ^ 1, LAYER)[u] = (uint16_t)hb;
      }
    }
    lds_barrier();  // X (and this entry slot, NK tiles on) are restaged by the next tile
    ST_FLUSH(LAYER, st0, st1, st2, 0ull);
  }
}

// NW waves per workgroup (NW gate tiles; 4: 8-wave workgroups measured no faster)
template <int LAYER, int NW>
__global__ void __launch_bounds__(NW * 64) dec_pred_kernel(DecArgs a, int parity) {
  // bf16 pitch +32 B per row: every ds_read_b128 lane group ({0-3,12-15,20-27}, ...: rows c, 16-B
  // column q) lands on 16 distinct bank quads; the round-2 +16 B pitch put rows c and c+8 on the same
  // quads (2-way, 36-37 % of the LDS cycles of these kernels in the r02 PMC pass)
  __shared__ __attribute__((aligned(16))) uint16_t X[DEC_RT][pred_xp(LAYER)];
  __shared__ int ents_all[NW * 64 / DEC_RT][DEC_RT];
  PredRegs<LAYER> W;
  dec_pred_body<LAYER, NW, false>(a, parity, xcd_grid(PG4 / (16 * NW)), X, ents_all, W);
}

// G = b_p + g . W1p^T for the listed rows' new candidates.  Workgroups of 4 waves, one 16-column
// tile (10 KB of W1p) per wave in registers: grid x = 8 column groups, y = row groups striding
// over the emit list's tiles.  Also clears the next step's emit and live lists for the joint
// that follows (reset: the workgroup that does it).
constexpr int GXP = P + 16;  // +32 B: conflict-free fragment reads (see dec_pred_kernel's XP)
constexpr int G_THREADS = 256;  // 4 waves, one 16-column tile each; grid x = 8 column groups
struct GRegs {
  uint4 wv[P / 32];
  float4 b0;
  bool wl = false;
};
template <bool PS, int RT = DEC_RT>
__device__ __forceinline__ void dec_g_body(const DecArgs& a, int parity, const GridXY gxy, bool reset,
                                           uint16_t (*X)[GXP], int (*ents_all)[RT], GRegs& W) {
  constexpr int NK = G_THREADS / RT;  // row tiles whose list entries load up front
  constexpr int DEC_SUB = RT / 16;
  const DecState& s = a.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  ST_MARK(st0);
  if (reset && tid == 0) {
    st_b32<PS>(&s.count[EMIT_N(parity ^ 1)], 0u);
    st_b32<PS>(&s.count[LIVE_N(parity ^ 1)], 0u);
  }
  const int* list = s.list + parity * a.Npad;
  const int i0 = (gxy.y + (tid / RT) * gxy.ny) * RT + tid % RT;
  const int e0 = i0 < a.Npad ? list[i0] : -1;
  const int cnt = s.count[EMIT_N(parity)];
  const int ntiles = (cnt + RT - 1) / RT;
  if (gxy.y >= ntiles) return;
  ents_all[tid / RT][tid % RT] = i0 < cnt ? e0 : -1;
  const int jt = gxy.x * (G_THREADS / 64) + wave;  // this wave's column tile
  for (int rt = gxy.y, it = 0; rt < ntiles; rt += gxy.ny, ++it) {
    int* ents = ents_all[it % NK];
    if (it >= NK && tid < RT) ents[tid] = rt * RT + tid < cnt && dec_ok(rt * RT + tid < a.Npad, 6) ? list[rt * RT + tid] : -1;
    lds_barrier();
    ST_MARK(st1);
    constexpr int NX = RT * (P / 8), NIT = (NX + G_THREADS - 1) / G_THREADS;
    uint4 xv[NIT];
    int emv[NIT];
#pragma unroll
    for (int u = 0; u < NIT; ++u) {  // this thread's entries first (one LDS round trip)
      const int i = tid + G_THREADS * u;
      emv[u] = (NX % G_THREADS == 0 || i < NX) ? ents[i / (P / 8)] : -1;
    }
#pragma unroll
    for (int u = 0; u < NIT; ++u) {  // every load first (one round trip); past the list end: row 0, zeros staged
      const int i = tid + G_THREADS * u;
      if (NX % G_THREADS == 0 || i < NX) {
        const int k = (i % (P / 8)) * 8, em = emv[u];
        const bool okr = em >= 0 && dec_ok(entry_row(em) < a.Npad, 4);
        xv[u] = *(const uint4*)(h_bf(a.hc, okr ? entry_row(em) : 0, okr ? entry_slot(em) ^ 1 : 0, 1) + k);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the weight loads behind the input loads
    if (!W.wl) {
      W.wl = true;
      const uint16_t* w0 = a.w.w1p + (size_t)(jt * 16 + c) * P + 8 * q;
#pragma unroll
      for (int b = 0; b < P / 32; ++b) W.wv[b] = *(const uint4*)(w0 + 32 * b);
      W.b0 = *(const float4*)(a.w.bp + jt * 16 + 4 * q);
    }
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
      const int i = tid + G_THREADS * u;
      if (NX % G_THREADS == 0 || i < NX) {
        const int m = i / (P / 8), k = (i % (P / 8)) * 8;
        *(uint4*)&X[m][k] = emv[u] >= 0 ? xv[u] : uint4{0u, 0u, 0u, 0u};
      }
    }
    lds_barrier();
    ST_MARK(st2);
    // every sub-tile's chain advances one k block at a time (fragment reads overlap MFMAs)
    v4f accs[DEC_SUB];
#pragma unroll
    for (int st = 0; st < DEC_SUB; ++st) accs[st] = v4f{W.b0.x, W.b0.y, W.b0.z, W.b0.w};
#pragma unroll
    for (int b = 0; b < P / 32; ++b)
#pragma unroll
      for (int st = 0; st < DEC_SUB; ++st)
        accs[st] = mfma_bf16(W.wv[b], *(const uint4*)(&X[16 * st + c][8 * q] + 32 * b), accs[st]);
#pragma unroll
    for (int st = 0; st < DEC_SUB; ++st) {
      const int ec = ents[16 * st + c];
      const v4f acc = accs[st];
      if (ec >= 0 && dec_ok(entry_row(ec) < a.Npad, 5))
        st_b128<PS>(a.G + (size_t)entry_row(ec) * J + jt * 16 + 4 * q,
                    uint4{__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])});
    }
    lds_barrier();
    ST_FLUSH(2, st0, st1, st2, 0ull);
  }
}

__global__ void __launch_bounds__(G_THREADS) dec_g_kernel(DecArgs a, int parity) {
  __shared__ __attribute__((aligned(16))) uint16_t X[DEC_RT][GXP];
  __shared__ int ents_all[G_THREADS / DEC_RT][DEC_RT];
  GRegs W;
  dec_g_body<false>(a, parity, xcd_grid(J / (16 * (G_THREADS / 64))), blockIdx.x == 0, X, ents_all, W);
}

// Co-resident step kernels (SLIM): 16-row tiles and a register cap, so a workgroup fits on a CU
// beside a 256x256 encoder tick workgroup (147456 B of LDS, 2 waves x 200 VGPRs per SIMD: 16 KiB of
// LDS and 112 VGPRs per SIMD left).  The same bodies, the same instruction sequence per row: identical
// results.  While an encoder runs, the step kernels above wait for a tick workgroup to give up a CU.
constexpr int SLIM_RT = 16;
#ifndef RNNT_EMU
#define SLIM_BOUNDS __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(56)))  // 112 on gfx950 (the attribute counts half)
#else
#define SLIM_BOUNDS __launch_bounds__(256)
#endif
template <int LAYER>
__global__ void SLIM_BOUNDS dec_pred_slim_kernel(DecArgs a, int parity) {
  __shared__ __attribute__((aligned(16))) uint16_t X[SLIM_RT][pred_xp(LAYER)];
  __shared__ int ents_all[256 / SLIM_RT][SLIM_RT];
  PredRegs<LAYER> W;
  dec_pred_body<LAYER, 4, false, SLIM_RT>(a, parity, xcd_grid(PG4 / 64), X, ents_all, W);
}
// Layer 1 does not fit that way (its [x | h] staging alone is 21 KB at 16 rows, its 640-k weight
// slice 80 VGPRs per wave), so its two chains are split over the two launches: the h chain (b_hh +
// h1.W_hh^T) reads only the committed h1, known before the step, so it runs in the layer-0 launch
// (gate groups 20..39 of that grid) and leaves its sums in PH; the layer-1 launch runs the x chain
// (b_ih + h0'.W_ih^T, h0' = layer 0's new h) and adds PH, x + h as the step kernel adds them.  Each
// role is a 320-k chain like the G kernel's.
enum { SLIM_H1 = 0, SLIM_X1 = 1 };
template <int ROLE>
__device__ __forceinline__ void dec_l1_slim_body(const DecArgs& a, int parity, const GridXY gxy, uint16_t (*X)[GXP],
                                                 int (*ents_all)[SLIM_RT]) {
  constexpr int RT = SLIM_RT, NK = 256 / RT;
  const DecState& s = a.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int* list = s.list + parity * a.Npad;
  const int i0 = (gxy.y + (tid / RT) * gxy.ny) * RT + tid % RT;
  const int e0 = i0 < a.Npad ? list[i0] : -1;
  const int cnt = s.count[EMIT_N(parity)];
  const int ntiles = (cnt + RT - 1) / RT;
  if (gxy.y >= ntiles) return;
  ents_all[tid / RT][tid % RT] = i0 < cnt ? e0 : -1;
  const int t0 = gxy.x * 4 + wave;  // this wave's gate tile
  uint4 wv[P / 32];
  float4 b0 = float4{0.0f, 0.0f, 0.0f, 0.0f};
  bool wl = false;
  for (int rt = gxy.y, it = 0; rt < ntiles; rt += gxy.ny, ++it) {
    int* ents = ents_all[it % NK];
    if (it >= NK && tid < RT) ents[tid] = rt * RT + tid < cnt && dec_ok(rt * RT + tid < a.Npad, 6) ? list[rt * RT + tid] : -1;
    lds_barrier();
    // this lane's row (column c of the tile) and, x chain, its cell state and h-chain sums
    int ec = ents[c];
    if (ec >= 0 && !dec_ok(entry_row(ec) < a.Npad && entry_label(ec) <= 28, 0)) ec = -1;
    const int erow = ec >= 0 ? entry_row(ec) : 0, esl = ec >= 0 ? entry_slot(ec) : 0;
    float cp = 0.0f;
    float4 ph = float4{0.0f, 0.0f, 0.0f, 0.0f};
    if (ROLE == SLIM_X1 && ec >= 0) {
      cp = hc_part(a.hc, erow, esl, 3)[t0 * 4 + q];
      ph = *(const float4*)(a.PH + (size_t)erow * PG4 + t0 * 16 + 4 * q);
    }
    constexpr int NX = RT * (P / 8), NIT = (NX + 255) / 256;
    uint4 xv[NIT];
    int emv[NIT];
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
      const int i = tid + 256 * u;
      emv[u] = (NX % 256 == 0 || i < NX) ? ents[i / (P / 8)] : -1;
    }
#pragma unroll
    for (int u = 0; u < NIT; ++u) {  // every load first (one round trip); past the list end: row 0, zeros staged
      const int i = tid + 256 * u;
      if (NX % 256 == 0 || i < NX) {
        const int k = (i % (P / 8)) * 8, em = emv[u];
        const bool okr = em >= 0 && dec_ok(entry_row(em) < a.Npad, 1);
        const int r = okr ? entry_row(em) : 0, sm = okr ? entry_slot(em) : 0;
        xv[u] = *(const uint4*)((ROLE == SLIM_H1 ? h_bf(a.hc, r, sm, 1) : h_bf(a.hc, r, sm ^ 1, 0)) + k);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the weight loads behind the input loads
    if (!wl) {
      wl = true;
      const uint16_t* wr = a.w.wp[1] + (size_t)(t0 * 16 + c) * 640 + 8 * q + (ROLE == SLIM_H1 ? P : 0);
#pragma unroll
      for (int b = 0; b < P / 32; ++b) wv[b] = *(const uint4*)(wr + 32 * b);
      b0 = *(const float4*)((ROLE == SLIM_H1 ? a.w.bhh_p[1] : a.w.bih_p[1]) + t0 * 16 + 4 * q);
    }
#pragma unroll
    for (int u = 0; u < NIT; ++u) {
      const int i = tid + 256 * u;
      if (NX % 256 == 0 || i < NX) {
        const int m = i / (P / 8), k = (i % (P / 8)) * 8;
        *(uint4*)&X[m][k] = emv[u] >= 0 ? xv[u] : uint4{0u, 0u, 0u, 0u};
      }
    }
    lds_barrier();
    v4f acc = v4f{b0.x, b0.y, b0.z, b0.w};
#pragma unroll
    for (int b = 0; b < P / 32; ++b) acc = mfma_bf16(wv[b], *(const uint4*)(&X[c][8 * q] + 32 * b), acc);
    if (ec >= 0) {
      if (ROLE == SLIM_H1) {
        *(v4f*)(a.PH + (size_t)erow * PG4 + t0 * 16 + 4 * q) = acc;
      } else {
        const v4f gs = acc + v4f{ph.x, ph.y, ph.z, ph.w};
        const int u = t0 * 4 + q;
        const float ig = det_sigmoid(gs[0]), fg = det_sigmoid(gs[1]), gg = det_tanh(gs[2]), og = det_sigmoid(gs[3]);
        const float cn = fg * cp + ig * gg;
        const float hh = bf_round_ftz(og * det_tanh(cn));
        hc_part(a.hc, erow, esl ^ 1, 3)[u] = cn;
        h_bf(a.hc, erow, esl ^ 1, 1)[u] = (uint16_t)(__float_as_uint(hh) >> 16);
      }
    }
    lds_barrier();  // X and this entry slot are restaged by the next tile
  }
}
// layer 0 (gate groups 0..19) and layer 1's h chain (20..39) in one launch
__global__ void SLIM_BOUNDS dec_pred0h_slim_kernel(DecArgs a, int parity) {
  __shared__ __attribute__((aligned(16))) uint16_t X[SLIM_RT][GXP];
  __shared__ int ents_all[256 / SLIM_RT][SLIM_RT];
  GridXY g = xcd_grid(2 * (PG4 / 64));
  if (g.x < PG4 / 64) {
    PredRegs<0> W;
    dec_pred_body<0, 4, false, SLIM_RT>(a, parity, g, X, ents_all, W);
  } else {
    g.x -= PG4 / 64;
    dec_l1_slim_body<SLIM_H1>(a, parity, g, X, ents_all);
  }
}
__global__ void SLIM_BOUNDS dec_pred1x_slim_kernel(DecArgs a, int parity) {
  __shared__ __attribute__((aligned(16))) uint16_t X[SLIM_RT][GXP];
  __shared__ int ents_all[256 / SLIM_RT][SLIM_RT];
  dec_l1_slim_body<SLIM_X1>(a, parity, xcd_grid(PG4 / 64), X, ents_all);
}
__global__ void SLIM_BOUNDS dec_g_slim_kernel(DecArgs a, int parity) {
  __shared__ __attribute__((aligned(16))) uint16_t X[SLIM_RT][GXP];
  __shared__ int ents_all[G_THREADS / SLIM_RT][SLIM_RT];
  GRegs W;
  dec_g_body<false, SLIM_RT>(a, parity, xcd_grid(J / (16 * (G_THREADS / 64))), blockIdx.x == 0, X, ents_all, W);
}

// joint (y1 = bf16(relu(F[t] + G)), logits = b2 + y1.W2^T) + argmax + greedy_decode_update
// (decoder.py:137-167) for JRT live-list rows per workgroup tile.  A blank (or a forced advance
// after max_symbols_per_step) moves the row to its next frame with the SAME prediction, so the
// workgroup evaluates up to JOINT_ITERS frames per launch, stopping a row at its first
// emission (it then needs a new prediction: next step's emit list) or at its last frame; rows
// not finished go to the next step's live list.  Identical results for any cap; the cap
// trades lock-step steps against the length of each step.
constexpr int JOINT_ITERS = 2;  // 1 / 3 / 4 measured slower

constexpr int YP = J + 16;  // +32 B: conflict-free fragment reads (see dec_pred_kernel's XP)
constexpr int JRT = 16;  // joint rows per workgroup tile: the argmax maps 4 waves x 4 rows x 16 lanes onto it
struct JointLds {
  __attribute__((aligned(16))) uint16_t X[JRT][YP];
  float Lp[4][JRT][NLAB_PAD + 1];
  int rows[JRT], walking[JRT], tidx[JRT], emit_e[JRT];
  int slot_[JRT], add_[JRT], flen_[JRT], idx_[JRT];
};
struct JointRegs {
  uint4 wv[8];  // W2 fragments: issued after the first tile's F / G loads (see dec_pred_kernel)
  v4f bias = v4f{0.0f, 0.0f, 0.0f, 0.0f};
  bool wl = false;
};
// jg / njg: this workgroup's index among the joint workgroups and their count (row tiles jg, jg + njg, ...)
template <bool PS>
__device__ __forceinline__ void dec_joint_body(const DecArgs& a, int parity, int jg, int njg, JointLds& L, JointRegs& W) {
  const DecState& s = a.s;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  ST_MARK(st0);
  const int4* llist = s.live + parity * a.Npad;
  int4* nlist = s.live + (parity ^ 1) * a.Npad;
  const int4 r_first = tid < JRT ? llist[jg * JRT + tid] : int4{0, 0, 0, 0};
  const int lcnt = s.count[LIVE_N(parity)];
  const int ntiles = (lcnt + JRT - 1) / JRT;
  if (jg >= ntiles) return;
  // logits = ((s0 + s1) + s2) + s3, s_b = y1[128b : 128b+128] . W2^T (s0 from b2): wave w runs
  // label half w&1 over k blocks 2(w>>1) and 2(w>>1)+1 as two independent 4-instruction chains
  const int lh = wave & 1, kb0 = 2 * (wave >> 1);
  for (int rt = jg; rt < ntiles; rt += njg) {
    if (tid < JRT) {
      const int i = rt * JRT + tid;
      const int4 e = i < lcnt && dec_ok(i < a.Npad, 7) ? (rt == jg ? r_first : llist[i]) : int4{-1, 0, 0, 0};
      int r = e.x < 0 ? -1 : entry_row(e.x);
      if (r >= 0 && !dec_ok(r < a.Npad && (e.y & 0xffff) < ((e.y >> 16) & 0xffff), 8)) r = -1;
      L.rows[tid] = r;
      L.walking[tid] = r >= 0;
      L.emit_e[tid] = -1;
      L.slot_[tid] = (e.x >> 24) & 1;
      L.add_[tid] = (e.x >> 25) & 31;
      L.tidx[tid] = e.y & 0xffff;
      L.flen_[tid] = (e.y >> 16) & 0xffff;
      L.idx_[tid] = e.z;
    }
    lds_barrier();
    ST_MARK(st1);
#ifdef RNNT_DEV_STAMPS
    unsigned long long st2 = 0ull;
#endif
    constexpr int NIT = JRT * (J / 8) / 256;
    float4 gl4[NIT][2];
    for (int it = 0; it < JOINT_ITERS; ++it) {
      bool any = false;
      for (int m = 0; m < JRT; ++m) any |= L.walking[m] != 0;
      if (!any) break;
      // every load of the tile first (one memory round trip), then y1: rows not walking read a
      // safe cached address (row 0 of frame 0) and stage zeros.  G is the same for every frame
      // of the walk (blank keeps the prediction).
      v4f fl4[NIT][2];
      bool wk[NIT];
#pragma unroll
      for (int u = 0; u < NIT; ++u) {
        const int i = tid + 256 * u, m = i / (J / 8), k = (i % (J / 8)) * 8;
        wk[u] = L.walking[m] != 0;
        const int row = wk[u] ? L.rows[m] : 0, tm = wk[u] ? L.tidx[m] : 0;
        const float* fr = a.F + ((size_t)tm * a.Npad + row) * J + k;
        fl4[u][0] = __builtin_nontemporal_load((const v4f*)fr);  // streamed once
        fl4[u][1] = __builtin_nontemporal_load((const v4f*)(fr + 4));
        if (it == 0) {
          const float* gr = a.G + (size_t)row * J + k;
          gl4[u][0] = *(const float4*)gr;
          gl4[u][1] = *(const float4*)(gr + 4);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (!W.wl) {
        W.wl = true;
        const uint16_t* wr = a.w.w2 + (size_t)(lh * 16 + c) * J + 8 * q;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          W.wv[b] = *(const uint4*)(wr + 128 * kb0 + 32 * b);
          W.wv[4 + b] = *(const uint4*)(wr + 128 * (kb0 + 1) + 32 * b);
        }
        if (kb0 == 0) {
          const float4 b0 = *(const float4*)(a.w.b2 + lh * 16 + 4 * q);
          W.bias = v4f{b0.x, b0.y, b0.z, b0.w};
        }
      }
#pragma unroll
      for (int u = 0; u < NIT; ++u) {
        const int i = tid + 256 * u, m = i / (J / 8), k = (i % (J / 8)) * 8;
        float y[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const v4f f4 = fl4[u][h];
          const float4 g4 = gl4[u][h];
          const float s0 = f4[0] + g4.x, s1 = f4[1] + g4.y, s2 = f4[2] + g4.z, s3 = f4[3] + g4.w;
          y[4 * h + 0] = bf_round_ftz(s0 > 0.0f ? s0 : 0.0f);
          y[4 * h + 1] = bf_round_ftz(s1 > 0.0f ? s1 : 0.0f);
          y[4 * h + 2] = bf_round_ftz(s2 > 0.0f ? s2 : 0.0f);
          y[4 * h + 3] = bf_round_ftz(s3 > 0.0f ? s3 : 0.0f);
        }
        *(uint4*)&L.X[m][k] = wk[u] ? pack8(float4{y[0], y[1], y[2], y[3]}, float4{y[4], y[5], y[6], y[7]})
                                    : uint4{0u, 0u, 0u, 0u};
      }
      lds_barrier();
      ST_SET(st2);
      if (__any(L.walking[c] != 0)) {
        const uint16_t* xr = &L.X[c][8 * q];
        v4f s0 = W.bias, s1 = v4f{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          s0 = mfma_bf16(W.wv[b], *(const uint4*)(xr + 128 * kb0 + 32 * b), s0);
          s1 = mfma_bf16(W.wv[4 + b], *(const uint4*)(xr + 128 * (kb0 + 1) + 32 * b), s1);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          L.Lp[kb0][c][lh * 16 + 4 * q + r] = s0[r];
          L.Lp[kb0 + 1][c][lh * 16 + 4 * q + r] = s1[r];
        }
      }
      lds_barrier();
      // logits = ((s0 + s1) + s2) + s3 and the argmax over the 29 real labels: wave w takes rows
      // 4w .. 4w+3, 16 lanes per row with labels 2l, 2l+1, merged by cross-lane moves (larger
      // value, ties to the smaller label: torch.argmax's first maximum); the row's first lane
      // applies greedy_decode_update
      {
        const int m = 4 * wave + (lane >> 4), l2 = 2 * (lane & 15);
        float bv = 0.0f;
        int bl = -1;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int j = l2 + e;
          const float v = ((L.Lp[0][m][j] + L.Lp[1][m][j]) + L.Lp[2][m][j]) + L.Lp[3][m][j];
          if (j < NLAB && (bl < 0 || v > bv)) {
            bv = v;
            bl = j;
          }
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          const float ov = __shfl_xor(bv, off);
          const int ol = __shfl_xor(bl, off);
          if (ol >= 0 && (bl < 0 || ov > bv || (ov == bv && ol < bl))) {
            bv = ov;
            bl = ol;
          }
        }
        if ((lane & 15) == 0) {
          if (L.walking[m]) {
            const int row = L.rows[m], best = bl;
            if (best != BLANK && L.add_[m] != MAXSYM) {
              const int id = L.idx_[m] + 1;
              L.idx_[m] = id;
              // persistent launch: write-through, as a row's next step may run on another XCD
              // whose L2 would otherwise write back its own (newer) copy of the line first
              st_b32<PS>(&s.idx[row], (uint32_t)id);
              if (id < a.max_res) st_b32<PS>(&a.res[(size_t)row * a.max_res + id], (uint32_t)best);
              st_b32<PS>(&s.added[row], (uint32_t)++L.add_[m]);
              st_b32<PS>(&s.preg[row], (uint32_t)best);
              const int nsl = L.slot_[m] ^ 1;  // commit the candidate (hg, cg) as (pre_hg, pre_cg)
              L.slot_[m] = nsl;
              st_b32<PS>(&s.slot[row], (uint32_t)nsl);
              L.emit_e[m] = emit_entry(row, nsl, best);
              L.walking[m] = 0;
            } else {
              const int fl = L.flen_[m];
              int t = L.tidx[m] + 1;
              if (t >= fl) {
                st_b32<PS>(&s.fin[row], 1u);
                L.walking[m] = 0;
                L.rows[m] = -1;  // finished: not in the next live list
                t = fl - 1;
              }
              L.tidx[m] = t;
              st_b32<PS>(&s.time[row], (uint32_t)t);
              st_b32<PS>(&s.added[row], 0u);
              L.add_[m] = 0;
            }
          }
        }
      }
      lds_barrier();
    }
    // the tile's emitting rows -> next emit list, its unfinished rows -> next live list: ONE
    // 64-bit atomic on the adjacent (emit, live) counters of the next parity returns both bases
    if (wave == 0) {
      const int e = lane < JRT ? L.emit_e[lane] : -1;
      const int r = lane < JRT ? L.rows[lane] : -1;
      const unsigned long long me = __ballot(e >= 0), mr = __ballot(r >= 0);
      unsigned long long base = 0;
      if (lane == 0 && (me | mr)) {
        const unsigned long long inc = (unsigned long long)__popcll(me) | ((unsigned long long)__popcll(mr) << 32);
#ifndef RNNT_EMU
        base = PS ? __hip_atomic_fetch_add((unsigned long long*)&s.count[EMIT_N(parity ^ 1)], inc, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)
                  : atomicAdd((unsigned long long*)&s.count[EMIT_N(parity ^ 1)], inc);
#else
        base = atomicAdd((unsigned long long*)&s.count[EMIT_N(parity ^ 1)], inc);
#endif
      }
      base = __shfl(base, 0);
      const unsigned long long below = (1ull << lane) - 1;
      if (lane == 0) dec_ok(false, 31);  // ran (the emulator's check that the joint executed)
      if (e >= 0 && dec_ok((int)(base & 0xffffffffu) + __popcll(me & below) < a.Npad, 9))
        st_b32<PS>(&s.list[(parity ^ 1) * a.Npad + (int)(base & 0xffffffffu) + __popcll(me & below)], (uint32_t)e);
      if (r >= 0 && dec_ok((int)(base >> 32) + __popcll(mr & below) < a.Npad, 10)) {
        const int4 le = live_entry(r, L.slot_[lane], L.add_[lane], L.tidx[lane], L.flen_[lane], L.idx_[lane]);
        st_b128<PS>(&nlist[(int)(base >> 32) + __popcll(mr & below)], uint4{(uint32_t)le.x, (uint32_t)le.y, (uint32_t)le.z, (uint32_t)le.w});
      }
    }
    lds_barrier();  // rows / walking / tidx / X are reused by the next row tile
    ST_FLUSH(3, st0, st1, st2, 0ull);
  }
}

__global__ void __launch_bounds__(256) dec_joint_kernel(DecArgs a, int parity) {
  __shared__ JointLds L;
  JointRegs W;
  dec_joint_body<false>(a, parity, blockIdx.x, gridDim.x, L, W);
}

// Co-resident joint (SLIM): 9 KB of LDS and at most 112 VGPRs, so it fits beside an encoder tick
// workgroup.  No y1 staging: wave w takes k block w (k = 128w .. 128w + 127) for both label halves and
// builds its B fragments in registers straight from F and G (the 8 k of row c that the MFMA's lane
// (q, c) takes: F and G for 16 rows x 128 k per wave, each element loaded once per tile); its two
// chains are s_w of the step kernel (from b2 on block 0, from 0 on the others), so the logits
// ((s0 + s1) + s2) + s3 and everything after them are the step kernel's.  G is re-read each walk
// iteration (the step kernel keeps it in registers).
struct JointSlimLds {
  float Lp[4][JRT][NLAB_PAD + 1];
  int rows[JRT], walking[JRT], tidx[JRT], emit_e[JRT];
  int slot_[JRT], add_[JRT], flen_[JRT], idx_[JRT];
};
__global__ void SLIM_BOUNDS dec_joint_slim_kernel(DecArgs a, int parity) {
  __shared__ JointSlimLds L;
  const DecState& s = a.s;
  const int jg = blockIdx.x, njg = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4, c = lane & 15;
  const int4* llist = s.live + parity * a.Npad;
  int4* nlist = s.live + (parity ^ 1) * a.Npad;
  const int4 r_first = tid < JRT ? llist[jg * JRT + tid] : int4{0, 0, 0, 0};
  const int lcnt = s.count[LIVE_N(parity)];
  const int ntiles = (lcnt + JRT - 1) / JRT;
  if (jg >= ntiles) return;
  for (int rt = jg; rt < ntiles; rt += njg) {
    if (tid < JRT) {
      const int i = rt * JRT + tid;
      const int4 e = i < lcnt && dec_ok(i < a.Npad, 7) ? (rt == jg ? r_first : llist[i]) : int4{-1, 0, 0, 0};
      int r = e.x < 0 ? -1 : entry_row(e.x);
      if (r >= 0 && !dec_ok(r < a.Npad && (e.y & 0xffff) < ((e.y >> 16) & 0xffff), 8)) r = -1;
      L.rows[tid] = r;
      L.walking[tid] = r >= 0;
      L.emit_e[tid] = -1;
      L.slot_[tid] = (e.x >> 24) & 1;
      L.add_[tid] = (e.x >> 25) & 31;
      L.tidx[tid] = e.y & 0xffff;
      L.flen_[tid] = (e.y >> 16) & 0xffff;
      L.idx_[tid] = e.z;
    }
    lds_barrier();
#pragma unroll 1
    for (int it = 0; it < JOINT_ITERS; ++it) {
      bool any = false;
      for (int m = 0; m < JRT; ++m) any |= L.walking[m] != 0;
      if (!any) break;
      // this lane's row: F at its walk frame and G (rows not walking read row 0 of frame 0: their
      // columns are computed and dropped)
      const bool wk = L.walking[c] != 0;
      const int row = wk ? L.rows[c] : 0, tm = wk ? L.tidx[c] : 0;
      const float* fr = a.F + ((size_t)tm * a.Npad + row) * J + 128 * wave + 8 * q;
      const float* gr = a.G + (size_t)row * J + 128 * wave + 8 * q;
      // W2 fragments (label half h, k = 128 wave + 32 b + 8 q; re-read each iteration, L1 / L2
      // hits) and F and G in two halves: the first half goes to bf16 before the second loads --
      // 64 VGPRs of F and G at once would not fit beside the weights
      uint4 wv[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint16_t* wr = a.w.w2 + (size_t)(h * 16 + c) * J + 128 * wave + 8 * q;
#pragma unroll
        for (int b = 0; b < 4; ++b) wv[h][b] = *(const uint4*)(wr + 32 * b);
      }
      // chains from b2 on block 0 (re-read each iteration: registers are the budget here)
      v4f s0 = v4f{0.0f, 0.0f, 0.0f, 0.0f}, s1 = s0;
      if (wave == 0) {
        s0 = *(const v4f*)(a.w.b2 + 4 * q);
        s1 = *(const v4f*)(a.w.b2 + 16 + 4 * q);
      }
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        v4f f4[2][2];
        float4 g4[2][2];
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          const int b = 2 * hb + bb;
          f4[bb][0] = __builtin_nontemporal_load((const v4f*)(fr + 32 * b));  // streamed once
          f4[bb][1] = __builtin_nontemporal_load((const v4f*)(fr + 32 * b + 4));
          g4[bb][0] = *(const float4*)(gr + 32 * b);
          g4[bb][1] = *(const float4*)(gr + 32 * b + 4);
        }
        uint4 yb[2];
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          float y[8];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const v4f f = f4[bb][h];
            const float4 g = g4[bb][h];
            const float t0 = f[0] + g.x, t1 = f[1] + g.y, t2 = f[2] + g.z, t3 = f[3] + g.w;
            y[4 * h + 0] = bf_round_ftz(t0 > 0.0f ? t0 : 0.0f);
            y[4 * h + 1] = bf_round_ftz(t1 > 0.0f ? t1 : 0.0f);
            y[4 * h + 2] = bf_round_ftz(t2 > 0.0f ? t2 : 0.0f);
            y[4 * h + 3] = bf_round_ftz(t3 > 0.0f ? t3 : 0.0f);
          }
          yb[bb] = pack8(float4{y[0], y[1], y[2], y[3]}, float4{y[4], y[5], y[6], y[7]});
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          s0 = mfma_bf16(wv[0][2 * hb + bb], yb[bb], s0);
          s1 = mfma_bf16(wv[1][2 * hb + bb], yb[bb], s1);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        L.Lp[wave][c][4 * q + r] = s0[r];
        L.Lp[wave][c][16 + 4 * q + r] = s1[r];
      }
      lds_barrier();
      // the step kernel's argmax and greedy_decode_update (dec_joint_body)
      {
        const int m = 4 * wave + (lane >> 4), l2 = 2 * (lane & 15);
        float bv = 0.0f;
        int bl = -1;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int j = l2 + e;
          const float v = ((L.Lp[0][m][j] + L.Lp[1][m][j]) + L.Lp[2][m][j]) + L.Lp[3][m][j];
          if (j < NLAB && (bl < 0 || v > bv)) {
            bv = v;
            bl = j;
          }
        }
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          const float ov = __shfl_xor(bv, off);
          const int ol = __shfl_xor(bl, off);
          if (ol >= 0 && (bl < 0 || ov > bv || (ov == bv && ol < bl))) {
            bv = ov;
            bl = ol;
          }
        }
        if ((lane & 15) == 0 && L.walking[m]) {
          const int row = L.rows[m], best = bl;
          if (best != BLANK && L.add_[m] != MAXSYM) {
            const int id = L.idx_[m] + 1;
            L.idx_[m] = id;
            s.idx[row] = id;
            if (id < a.max_res) a.res[(size_t)row * a.max_res + id] = best;
            s.added[row] = ++L.add_[m];
            s.preg[row] = best;
            const int nsl = L.slot_[m] ^ 1;  // commit the candidate (hg, cg) as (pre_hg, pre_cg)
            L.slot_[m] = nsl;
            s.slot[row] = nsl;
            L.emit_e[m] = emit_entry(row, nsl, best);
            L.walking[m] = 0;
          } else {
            const int fl = L.flen_[m];
            int t = L.tidx[m] + 1;
            if (t >= fl) {
              s.fin[row] = 1;
              L.walking[m] = 0;
              L.rows[m] = -1;  // finished: not in the next live list
              t = fl - 1;
            }
            L.tidx[m] = t;
            s.time[row] = t;
            s.added[row] = 0;
            L.add_[m] = 0;
          }
        }
      }
      lds_barrier();
    }
    // the tile's emitting rows -> next emit list, its unfinished rows -> next live list (one 64-bit atomic)
    if (wave == 0) {
      const int e = lane < JRT ? L.emit_e[lane] : -1;
      const int r = lane < JRT ? L.rows[lane] : -1;
      const unsigned long long me = __ballot(e >= 0), mr = __ballot(r >= 0);
      unsigned long long base = 0;
      if (lane == 0 && (me | mr)) {
        const unsigned long long inc = (unsigned long long)__popcll(me) | ((unsigned long long)__popcll(mr) << 32);
        base = atomicAdd((unsigned long long*)&s.count[EMIT_N(parity ^ 1)], inc);
      }
      base = __shfl(base, 0);
      const unsigned long long below = (1ull << lane) - 1;
      if (lane == 0) dec_ok(false, 31);  // ran (the emulator's check that the joint executed)
      if (e >= 0 && dec_ok((int)(base & 0xffffffffu) + __popcll(me & below) < a.Npad, 9))
        s.list[(parity ^ 1) * a.Npad + (int)(base & 0xffffffffu) + __popcll(me & below)] = e;
      if (r >= 0 && dec_ok((int)(base >> 32) + __popcll(mr & below) < a.Npad, 10)) {
        const int4 le = live_entry(r, L.slot_[lane], L.add_[lane], L.tidx[lane], L.flen_[lane], L.idx_[lane]);
        nlist[(int)(base >> 32) + __popcll(mr & below)] = le;
      }
    }
    lds_barrier();  // rows / walking / tidx are reused by the next row tile
  }
}

#ifndef RNNT_EMU
// ---------------------------------------------------------------- persistent tail decode
// Once few rows are live (the long tail of a length-sorted batch, where a step is four dependent
// launches of a handful of workgroups), one launch runs every remaining step: each workgroup takes
// one role for the whole launch -- a prediction layer-0 / layer-1 gate group (20 each), a G column
// group (8) or a joint row group (nj) -- keeps its weight slice in registers across steps, and
// runs that role's step body (the SAME code as the step kernels above: identical results) once
// per step.  Phases hand off through per-role completion counters in device memory (`pc`):
// pred0(k) waits for joint(k-1), pred1(k) for pred0(k), G(k) for pred1(k), joint(k) for G(k); the
// data a phase hands on is stored write-through (PS = true).  Every role reads the same live count
// of step k (written by joint(k-1), complete before any role of step k starts) and stops at 0, or
// after max_steps; each still publishes, so no role waits for one that left.  Every wait is
// bounded: past the timeout it raises the abort word and every workgroup leaves (the host reports
// it).  Control flow around the waits is wave-uniform (wave 0 polls as a whole; see the flow
// encoder).
constexpr int PS_P0 = PG4 / (16 * 4), PS_P1 = PS_P0, PS_G = J / (16 * (G_THREADS / 64));  // 20, 20, 8
enum { PC_P0 = 0, PC_P1 = 1, PC_G = 2, PC_J = 3, PC_ABORT = 4, PC_STEPS = 5, PC_WORDS = 8 };
__device__ __forceinline__ unsigned pc_load(const uint32_t* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// wave 0 (whole wave): wait until counter `who` reaches `need`, then acquire; false on abort
__device__ __forceinline__ bool pc_wait(uint32_t* pc, int who, unsigned need, unsigned long long timeout) {
  const unsigned long long t_end = __builtin_amdgcn_s_memrealtime() + timeout;
  while (pc_load(pc + who) < need) {
    if (pc_load(pc + PC_ABORT)) return false;
    if (__builtin_amdgcn_s_memrealtime() > t_end) {
      __hip_atomic_store(pc + PC_ABORT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return true;
}

// one role's step loop; Body(parity) runs the step body
template <class Body>
__device__ __forceinline__ void ps_loop(const DecArgs& a, uint32_t* pc, int role, int prev, unsigned n_prev, int step0,
                                        int max_steps, unsigned long long timeout, int* lds_flag, int last_j, Body&& body) {
  const bool w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
  for (int k = 0;; ++k) {
    const int parity = (step0 + k) & 1;
    if (w0) {
      bool ok = true;
      if (!(role == PC_P0 && k == 0)) ok = pc_wait(pc, prev, n_prev * (unsigned)(role == PC_P0 ? k : k + 1), timeout);
      // the step's live count (joint(k-1) wrote it; every role reads the same value)
      const int live = ok ? (int)__builtin_amdgcn_readfirstlane(*(volatile const int*)&a.s.count[LIVE_N(parity)]) : 0;
      if (threadIdx.x == 0) lds_flag[0] = (!ok || live <= 0 || k >= max_steps) ? (ok ? 1 : 2) : 0;
    }
    __syncthreads();
    const int stop = __builtin_amdgcn_readfirstlane(lds_flag[0]);
    if (stop == 2) return;  // aborted: leave without publishing (every waiter sees the abort word)
    ST_MARK(ps0);
    if (!stop) body(parity);
    ST_MARK(ps1);
    // publish: every wave's stores have landed, then one count
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
#ifdef RNNT_DEV_STAMPS
      {  // record (16 + role, workgroup | step << 16, ready, body end, stores drained, published)
        const unsigned long long ps2 = __builtin_amdgcn_s_memrealtime();
        const unsigned k_ = atomicAdd(&g_st_n, 1u);
        if (k_ < (1u << 22) / 6) {
          g_st[6 * k_] = 16 + role; g_st[6 * k_ + 1] = blockIdx.x + 65536ull * k;
          g_st[6 * k_ + 2] = ps0; g_st[6 * k_ + 3] = ps1; g_st[6 * k_ + 4] = ps2;
          g_st[6 * k_ + 5] = __builtin_amdgcn_s_memrealtime();
        }
      }
#endif
      __hip_atomic_fetch_add(pc + role, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (stop && last_j) __hip_atomic_store(pc + PC_STEPS, (uint32_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (stop) return;
    __syncthreads();  // lds_flag is rewritten by the next step
  }
}

constexpr size_t ps_lds_bytes() {
  const size_t p1 = sizeof(uint16_t) * DEC_RT * pred_xp(1) + sizeof(int) * (256 / DEC_RT) * DEC_RT;
  const size_t g = sizeof(uint16_t) * DEC_RT * GXP + sizeof(int) * (G_THREADS / DEC_RT) * DEC_RT;
  const size_t j = sizeof(JointLds);
  return (p1 > g ? (p1 > j ? p1 : j) : (g > j ? g : j)) + 16;
}

__global__ void __launch_bounds__(256) dec_persist_kernel(DecArgs a, uint32_t* pc, int step0, int max_steps, int nj,
                                                          unsigned long long timeout) {
  extern __shared__ __attribute__((aligned(16))) uint8_t psm[];
  int* flag = (int*)(psm + ps_lds_bytes() - 16);
  const int b = blockIdx.x;  // roles: [0,20) pred0 gate groups, [20,40) pred1, [40,48) G, [48,48+nj) joint
  if (b < PS_P0) {
    PredRegs<0> W;
    auto X = (uint16_t(*)[pred_xp(0)])psm;
    auto E = (int(*)[DEC_RT])(psm + sizeof(uint16_t) * DEC_RT * pred_xp(0));
    ps_loop(a, pc, PC_P0, PC_J, (unsigned)nj, step0, max_steps, timeout, flag, 0,
            [&](int p) { dec_pred_body<0, 4, true>(a, p, GridXY{b, 0, 1}, X, E, W); });
  } else if (b < PS_P0 + PS_P1) {
    PredRegs<1> W;
    auto X = (uint16_t(*)[pred_xp(1)])psm;
    auto E = (int(*)[DEC_RT])(psm + sizeof(uint16_t) * DEC_RT * pred_xp(1));
    ps_loop(a, pc, PC_P1, PC_P0, (unsigned)PS_P0, step0, max_steps, timeout, flag, 0,
            [&](int p) { dec_pred_body<1, 4, true>(a, p, GridXY{b - PS_P0, 0, 1}, X, E, W); });
  } else if (b < PS_P0 + PS_P1 + PS_G) {
    GRegs W;
    auto X = (uint16_t(*)[GXP])psm;
    auto E = (int(*)[DEC_RT])(psm + sizeof(uint16_t) * DEC_RT * GXP);
    const int g = b - PS_P0 - PS_P1;
    ps_loop(a, pc, PC_G, PC_P1, (unsigned)PS_P1, step0, max_steps, timeout, flag, 0,
            [&](int p) { dec_g_body<true>(a, p, GridXY{g, 0, 1}, g == 0, X, E, W); });
  } else {
    JointRegs W;
    JointLds& L = *(JointLds*)psm;
    const int jg = b - PS_P0 - PS_P1 - PS_G;
    ps_loop(a, pc, PC_J, PC_G, (unsigned)PS_G, step0, max_steps, timeout, flag, jg == 0,
            [&](int p) { dec_joint_body<true>(a, p, jg, nj, L, W); });
  }
}
#endif  // RNNT_EMU

__global__ void dec_finish_kernel(DecArgs a) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row < a.N) a.res_len[row] = a.s.idx[row] + 1;
}

int launch_greedy_decode(const DecArgs& a, int32_t* host_flags, hipEvent_t* evs, hipStream_t st, const int32_t* reset) {
  // every buffer the step kernels address (a missing one is a host error here, not a GPU fault)
  const void* need[] = {a.F, a.f_lens, a.hc, a.G, a.PH, a.res, a.res_len, a.w.xtab, a.w.wp[0], a.w.wp[1], a.w.bih_p[1],
                        a.w.bhh_p[0], a.w.bhh_p[1], a.w.w1p, a.w.bp, a.w.w2, a.w.b2, a.s.time, a.s.added, a.s.idx,
                        a.s.preg, a.s.slot, a.s.fin, a.s.list, a.s.live, a.s.count, a.s.pc};
  for (const void* p : need)
    if (!p) return -1;
  if (a.Npad % DEC_RT || a.N > a.Npad || a.Npad >= (1 << 24)) return -1;
  const int rt = a.Npad / DEC_RT;
  if (hipMemsetAsync(a.s.count, 0, 4 * sizeof(int32_t), st) != hipSuccess) return -1;
  if (reset) {
    hipLaunchKernelGGL(dec_reset_res_kernel, dim3(a.N), dim3(256), 0, st, a.res, a.max_res, reset);
    hipLaunchKernelGGL(dec_init_stream_kernel, dim3((a.Npad + 255) / 256), dim3(256), 0, st, a, reset);
  } else {
    if (hipMemsetAsync(a.res, 0xff, (size_t)a.N * a.max_res * sizeof(int32_t), st) != hipSuccess) return -1;
    hipLaunchKernelGGL(dec_init_kernel, dim3((a.Npad + 255) / 256), dim3(256), 0, st, a);
  }
  // Steps are enqueued in chunks and the host reads the live count one chunk behind, so a decode
  // ends with the rest of the chunk holding its last step plus one more chunk of (cheap, but still
  // ~20 us each: four dependent launches) empty steps.  Once few rows are left -- the long-tail
  // rows whose last emission ends the loop -- chunks shrink (TAIL_CHUNK): less overshoot while the
  // host (~3.5 us per launch) still stays ahead of the GPU.
  constexpr int CHUNK = 32, TAIL_ROWS = 64;
  // Tail chunks of 16 steps: isolated decode of the bench query 93.6 / 94.0 ms vs 94.6 / 94.9 with 8,
  // 95.3-96.0 with 4 (tools/r04_dectail.sh, same box, alternating; fewer polls outweigh the longer
  // overshoot).  Development knobs for that A/B: RNNT_DEC_TAIL_CHUNK steps per tail chunk,
  // RNNT_DEC_SPIN=1 polls the previous chunk's event without yielding (no gain measured).
  static const int TAIL_CHUNK = [] {
    const char* v = dev_env("RNNT_DEC_TAIL_CHUNK");
    const int c = v ? atoi(v) : 16;
    return c >= 1 && c <= CHUNK ? c : 16;
  }();
  static const bool SPIN = [] {
    const char* v = dev_env("RNNT_DEC_SPIN");
    return v && v[0] == '1';
  }();
  // development knob RNNT_DEC_RG="PxGxJ": row-group caps of the step kernels' grids (pred, G, joint)
  static const int* RG = [] {
    static int rg[3] = {PRED_ROW_GROUPS, G_ROW_GROUPS, JOINT_GROUPS};
    if (const char* v = dev_env("RNNT_DEC_RG")) {
      int x[3];
      if (sscanf(v, "%dx%dx%d", &x[0], &x[1], &x[2]) == 3 && x[0] > 0 && x[1] > 0 && x[2] > 0)
        for (int i = 0; i < 3; ++i) rg[i] = x[i];
    }
    return rg;
  }();
  // the co-resident step kernels (SLIM_BOUNDS): pred0 (1), pred1 with layer 1's h chain moved into the
  // layer-0 launch (2), G (4), joint (8) -- all four by default: 121.1-121.6k -> 122.9-123.1k utt/s,
  // overlapped greedy decode 2236 -> 1488 ms per query, isolated 656 -> 726 (MEASUREMENTS section 9).
  // Development knob RNNT_DEC_SLIM=mask selects a subset (0: the step kernels above alone).
  static const int SLIM = [] {
    const char* v = dev_env("RNNT_DEC_SLIM");
    return v ? atoi(v) : 15;
  }();
  // persistent tail (dec_persist_kernel): once the live rows read back fit a.persist_rows, one launch
  // runs every remaining step (0 = off; at most DEC_PERSIST_MAX rows)
#ifndef RNNT_EMU
  const int PERSIST_ROWS = a.persist_rows < 0 ? 0 : (a.persist_rows > DEC_PERSIST_MAX ? DEC_PERSIST_MAX : a.persist_rows);
  static std::atomic<uint64_t> ps_attr{0};
#else
  constexpr int PERSIST_ROWS = 0;
#endif
  int step = 0, chunk = 0;
  int live_bound = a.N;  // unfinished rows at the end of the last chunk read back (an upper bound)
  bool done = false;
  while (!done && step < a.max_iter) {
#ifndef RNNT_EMU
    if (PERSIST_ROWS > 0 && chunk > 0 && live_bound <= PERSIST_ROWS) {
      // the chunks already enqueued run first (stream order); the persistent launch continues at
      // `step` with at most live_bound rows (live counts only fall)
      const int nj = (live_bound + JRT - 1) / JRT > 0 ? (live_bound + JRT - 1) / JRT : 1;
      if (set_smem_attr_once((const void*)dec_persist_kernel, (int)ps_lds_bytes(), ps_attr)) return -1;
      if (hipMemsetAsync(a.s.pc, 0, PC_WORDS * sizeof(uint32_t), st) != hipSuccess) return -1;
      hipLaunchKernelGGL(dec_persist_kernel, dim3(PS_P0 + PS_P1 + PS_G + nj), dim3(256), ps_lds_bytes(), st, a, a.s.pc,
                         step, a.max_iter - step, nj, 200000000ull /* 2 s of s_memrealtime (100 MHz) */);
      if (hipGetLastError() != hipSuccess) return -1;
      if (hipMemcpyAsync(host_flags + 2, a.s.pc + PC_ABORT, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        return -1;
      if (host_flags[2]) return -2;  // a wait timed out: the launch drained without finishing
      step += host_flags[3];  // steps the launch ran (it stopped at step index host_flags[3])
      done = true;
      break;
    }
#endif
    const int csz = live_bound > TAIL_ROWS ? CHUNK : TAIL_CHUNK;
    // row-tile workgroups per launch: one resident round, and no more than the live rows need
    const int lt = (live_bound + DEC_RT - 1) / DEC_RT < rt ? (live_bound + DEC_RT - 1) / DEC_RT : rt;
    const int lt1 = lt > 0 ? lt : 1;
    const int rg_pred = lt1 < RG[0] ? lt1 : RG[0];
    const int rg_g = lt1 < RG[1] ? lt1 : RG[1];
    const int ljt = (live_bound + JRT - 1) / JRT > 0 ? (live_bound + JRT - 1) / JRT : 1;
    const int rg_joint = ljt < RG[2] ? ljt : RG[2];
    // co-resident kernels: 16-row tiles, the same row-group caps (twice as many: 120.4-122.8k vs 122.4-
    // 123.6k utt/s on one box; 6-8 pred groups lose 9 % isolated, MEASUREMENTS section 9)
    const int ls = (live_bound + SLIM_RT - 1) / SLIM_RT < a.Npad / SLIM_RT ? (live_bound + SLIM_RT - 1) / SLIM_RT : a.Npad / SLIM_RT;
    const int ls1 = ls > 0 ? ls : 1;
    const int sg_pred = ls1 < RG[0] ? ls1 : RG[0], sg_g = ls1 < RG[1] ? ls1 : RG[1];
    for (int i = 0; i < csz && step < a.max_iter; ++i, ++step) {
      const int p = step & 1;
      if (SLIM & 2)
        hipLaunchKernelGGL(dec_pred0h_slim_kernel, dim3(xcd_grid_size(2 * (PG4 / 64), sg_pred)), dim3(256), 0, st, a, p);
      else if (SLIM & 1)
        hipLaunchKernelGGL((dec_pred_slim_kernel<0>), dim3(xcd_grid_size(PG4 / 64, sg_pred)), dim3(256), 0, st, a, p);
      else
        hipLaunchKernelGGL((dec_pred_kernel<0, PRED_THREADS / 64>), dim3(xcd_grid_size(PG4 / (16 * (PRED_THREADS / 64)), rg_pred)),
                           dim3(PRED_THREADS), 0, st, a, p);
      if (SLIM & 2)
        hipLaunchKernelGGL(dec_pred1x_slim_kernel, dim3(xcd_grid_size(PG4 / 64, sg_pred)), dim3(256), 0, st, a, p);
      else
        hipLaunchKernelGGL((dec_pred_kernel<1, PRED_THREADS / 64>), dim3(xcd_grid_size(PG4 / (16 * (PRED_THREADS / 64)), rg_pred)),
                           dim3(PRED_THREADS), 0, st, a, p);
      if (SLIM & 4)
        hipLaunchKernelGGL(dec_g_slim_kernel, dim3(xcd_grid_size(J / (16 * (G_THREADS / 64)), sg_g)), dim3(G_THREADS), 0, st, a, p);
      else
        hipLaunchKernelGGL(dec_g_kernel, dim3(xcd_grid_size(J / (16 * (G_THREADS / 64)), rg_g)), dim3(G_THREADS), 0, st, a,
                           p);
      if (SLIM & 8)
        hipLaunchKernelGGL(dec_joint_slim_kernel, dim3(rg_joint), dim3(256), 0, st, a, p);
      else
        hipLaunchKernelGGL(dec_joint_kernel, dim3(rg_joint), dim3(256), 0, st, a, p);
    }
    // poll the live-row count one chunk behind, so the host never drains the queue: the length of
    // the live list the chunk's last joint wrote (parity step & 1; the next step's G kernel resets
    // the other parity's counters)
    if (hipMemcpyAsync(host_flags + (chunk & 1), a.s.count + LIVE_N(step & 1), sizeof(int32_t), hipMemcpyDeviceToHost,
                       st) != hipSuccess)
      return -1;
    if (hipEventRecord(evs[chunk & 1], st) != hipSuccess) return -1;
    if (chunk > 0) {
      if (SPIN) {
        hipError_t q;
        while ((q = hipEventQuery(evs[(chunk - 1) & 1])) == hipErrorNotReady) {
        }
        if (q != hipSuccess) return -1;
      } else if (hipEventSynchronize(evs[(chunk - 1) & 1]) != hipSuccess) {
        return -1;
      }
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
  if (Npad % 256 == 0) {  // the engine's batches; op-level callers with other row counts: 64-column kernel
    static std::atomic<uint64_t> gattr{0};
    if (set_smem_attr_once((const void*)joint_trans_gemm_kernel, JG_SMEM, gattr)) return -1;
    const int nrt = Tp * Npad / 256;
    hipLaunchKernelGGL(joint_trans_gemm_kernel, dim3(16 * ((nrt + 7) / 8)), dim3(512), JG_SMEM, st, w, fbf, f_lens, F,
                       Npad, nrt);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  static std::atomic<uint64_t> attr{0};
  const int smem = 64 * JT_PITCH * 2;
  if (set_smem_attr_once((const void*)joint_trans_kernel, smem, attr)) return -1;
  const int nrows = Tp * Npad;
  hipLaunchKernelGGL(joint_trans_kernel, dim3(xcd_grid_size(J / 64, (nrows + JT_ROWS - 1) / JT_ROWS)), dim3(256), smem,
                     st, w, fbf, f_lens, F, Npad, nrows);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dec_xtab(const DecWeights& w, float* xtab, hipStream_t st) {
  hipLaunchKernelGGL(dec_xtab_kernel, dim3(PG4 / 16), dim3(128), 0, st, w, xtab);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rnnt

#ifdef RNNT_DEV_STAMPS
// development: copy out (and reset) the step kernels' stamp records (6 x u64 each)
extern "C" int rnnt_dev_read_stamps(unsigned long long* out, int max_records) {
  unsigned int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(rnnt::g_st_n), sizeof(n)) != hipSuccess) return -1;
  if (n > (1u << 22) / 6) n = (1u << 22) / 6;
  if ((int)n > max_records) n = max_records;
  if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(rnnt::g_st), (size_t)n * 6 * 8) != hipSuccess) return -1;
  const unsigned int z = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(rnnt::g_st_n), &z, sizeof(z)) != hipSuccess) return -1;
  return (int)n;
}
#endif

#ifdef RNNT_DEC_CHECK
extern "C" int rnnt_dev_read_dec_err(unsigned int* out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rnnt::g_dec_err), sizeof(unsigned int)) != hipSuccess) return -1;
  const unsigned int z = 0;
  return hipMemcpyToSymbol(HIP_SYMBOL(rnnt::g_dec_err), &z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
