// encoder.hip -- int8 transcription (quantised encoder LSTM stack) on CDNA4.
//
// Replaces intel_mlperf::lstm_amx_int8 / stack_time (reference quant_lstm.py:80-102,
// modeling_rnnt.py:326-328).  One launch = one layer x one timestep over the active batch
// tiles: gates^T[4096 x Nb] = W[4096 x (I+H)] . [x_t | h_{t-1}]^T with int8 -> int32 MFMA
// (v_mfma_i32_16x16x64_i8), the whole LSTM cell (dequant + bias, sigmoid/tanh, fp16 cell,
// requantisation of h and y) fused in the epilogue, and StackTime fused into layer 1's
// output addressing.  int32 accumulation is exact, so results are bit-identical to the CPU
// restatement regardless of tiling.
//
// Weight rows are gate-interleaved (packed row 4u+g = original row g*1024+u), so a 16x16
// accumulator tile holds the i,f,g,o pre-activations of one (unit, batch row) in one lane's
// four registers (C/D map: row = 4*(lane>>4)+reg, col = lane&15).
#include "rnnt_device.hpp"
#include "encoder.hpp"

namespace rnnt {

// sigma table of the cell (tools/gen_act_table.py), copied to LDS by every workgroup
__device__ const float4 g_act_tab[128] = {
#include "act_table.inc"
};

// development instrumentation (-DRNNT_DEV_STAMPS, tools/enc_stamps.py): thread 0 of every tile
// records s_memrealtime (100 MHz) at workgroup start, once stage 0 has landed, after the main
// loop and after the epilogue, with the tile and the CU it ran on.
#ifdef RNNT_DEV_STAMPS
__device__ unsigned long long g_est[1 << 22];
__device__ unsigned int g_est_n;
#define EST_MARK(v) v = __builtin_amdgcn_s_memrealtime()
// record slot i of this tile's 8-word record (thread 0 stores at once: nothing stays live)
#define EST_PUT(i, v) \
  if (threadIdx.x == 0 && est_k < (1u << 22) / 8) g_est[8 * est_k + (i)] = (v)
#else
#define EST_MARK(v)
#define EST_PUT(i, v)
#endif

// ---------------------------------------------------------------- feature quantisation
// x_q = q8(x * in_scale[0]) over [T][Npad][256] (layer-0 input quantizer, calibrated on
// cat([x, h]); quant_modules.py:118-121).
__global__ void __launch_bounds__(256) quantize_kernel(const float4* __restrict__ x, int64_t n4, float s,
                                                       uint32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    const uint32_t b0 = (uint8_t)q8(v.x * s), b1 = (uint8_t)q8(v.y * s), b2 = (uint8_t)q8(v.z * s),
                   b3 = (uint8_t)q8(v.w * s);
    out[i] = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
  }
}

// AssembleSamples (rnnt_qsl.cpp:150-188) fused with the quantizer: one thread per 4 output
// channels, a wave covers one (frame, row) pair's 256 channels as 64 x 4 B (the 240 real
// channels are one contiguous 960-byte run of the sample's stored frame).
__global__ void __launch_bounds__(256) quantize_gather_kernel(const float* __restrict__ store,
                                                              const int64_t* __restrict__ offsets,
                                                              const int32_t* __restrict__ lens, int n, int n_pad,
                                                              int64_t words, float s, uint32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (int64_t)gridDim.x * blockDim.x) {
    const int c4 = (int)(i & 63);
    const int64_t rt = i >> 6;  // t * n_pad + row
    const int row = (int)(rt % n_pad), t = (int)(rt / n_pad);
    uint32_t v = 0;
    if (row < n && c4 < 60 && t < lens[row]) {
      const float4 x = *(const float4*)(store + (offsets[row] + t) * 240 + 4 * c4);
      v = (uint32_t)(uint8_t)q8(x.x * s) | ((uint32_t)(uint8_t)q8(x.y * s) << 8) |
          ((uint32_t)(uint8_t)q8(x.z * s) << 16) | ((uint32_t)(uint8_t)q8(x.w * s) << 24);
    }
    out[i] = v;
  }
}

// ---------------------------------------------------------------- LSTM step
// Workgroup tile: 256 packed gate rows (64 units) x 256 batch rows, K swept in 64-byte
// steps.  8 waves as 4 (gate) x 2 (batch); each wave owns 64 gate rows x 128 batch rows =
// 4 x 8 MFMA 16x16x64 tiles.  The 256x256 tile halves the L2->LDS bytes per MFMA of a 128x128
// tile: staging through the per-CU load path (~70 GB/s/CU from L2), not the MFMA, bounds this
// GEMM (DESIGN.md "Encoder kernel").
constexpr int BM = 256;
constexpr int BN = ENC_BATCH_TILE;           // 128 * ENC_WN
constexpr int BK = 64;
constexpr int NWAVE = 4 * ENC_WN;            // 4 gate-row waves x ENC_WN batch-column waves
#ifndef RNNT_NSTAGE
#define RNNT_NSTAGE (ENC_WN == 2 ? 4 : 3)
#endif
#ifndef RNNT_INTERLEAVE
#define RNNT_INTERLEAVE 0
#endif
#ifndef RNNT_STAGGER
#define RNNT_STAGGER 1
#endif
#ifndef RNNT_BK128  // 1: 128-byte-row stages, two buffers (see the main loop); 0: 64-byte stages, 4 buffers
#define RNNT_BK128 (ENC_WN == 2)
#endif
#ifndef RNNT_BK128_ISSUE  // 128-byte stages: 0 all pieces at the stage top; 1 waves 4-7 mid-stage; 2 A top, B mid
#define RNNT_BK128_ISSUE 2
#endif
#ifndef RNNT_PRIO_MODE  // 0: MFMA clusters at priority 1; 1: + late waves at 1 throughout; 2: static, late waves only
#define RNNT_PRIO_MODE 0
#endif
#ifndef RNNT_STAGGER_AT
#define RNNT_STAGGER_AT 2  // MFMA group (of 4) before which the late waves issue their pieces
#endif
constexpr int NSTAGE = RNNT_NSTAGE;          // LDS ring depth: NSTAGE-1 stages in flight
constexpr int A_BYTES = BM * BK;             // 16 KiB
constexpr int STAGE_BYTES = (BM + BN) * BK;  // 32 / 24 KiB
constexpr int APW = (BM / 16) / NWAVE;       // 16-row A pieces (1 KiB LDS-DMA each) per wave: 2 | 4
constexpr int BPW = (BN / 16) / NWAVE;       // B pieces per wave: 2
constexpr int GLDS_PER_STAGE = APW + BPW;
constexpr int C_GLDS = (BN * 128 / 1024) / NWAVE;  // cell-state DMA pieces per wave: 4
#ifndef RNNT_TAB_COPIES  // sigma-table copies in LDS: 16 = one per 16-byte bank slot
#define RNNT_TAB_COPIES 1
#endif
constexpr int TAB_COPIES = RNNT_TAB_COPIES;
constexpr int TAB_OFF = NSTAGE * STAGE_BYTES;   // LDS: sigma table after the ring
#ifndef RNNT_PERSIST
#define RNNT_PERSIST 0
#endif
constexpr int YS_OFF = TAB_OFF + 128 * 16 * TAB_COPIES;  // RNNT_PERSIST 2: the y image (256 x 80 B)
constexpr int SMEM_BYTES = YS_OFF + (RNNT_PERSIST == 2 ? BN * 80 : 0);
static_assert(TAB_COPIES == 1 || TAB_COPIES == 16, "table copies");
static_assert(SMEM_BYTES <= 160 * 1024, "LDS");
static_assert(BPW == 2 && (APW == 2 || APW == 4) && C_GLDS == 4, "staging split");
static_assert(BN * 128 <= STAGE_BYTES, "the cell-state image fits one ring buffer");
static_assert(NSTAGE >= 3 && BN * 80 <= STAGE_BYTES, "the epilogue's h / y images fit two other ring buffers");

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(1))) void glb_void;

// LDS image of a [rows][64 B] tile: 16-byte column c of row r is stored at column
// c ^ h[(r >> 2) & 3] with h = {0, 2, 3, 1}.  A fragment read (lane l: row l&15, column l>>4)
// is a ds_read_b128 whose four 16-lane groups each touch rows {0-3,12-15} at one column and
// rows 4-11 at the next; with this h every group lands on 16 distinct 16-byte bank slots.
__device__ __forceinline__ int swz_h(int row) { return (0x1320 >> (((row >> 2) & 3) * 4)) & 3; }
__device__ __forceinline__ int swz(int row, int col16) { return row * BK + ((col16 ^ swz_h(row)) << 4); }

// Retire this wave's LDS-DMA down to N outstanding, drain LDS ops, then barrier: after it,
// every wave's DMA of the retired stage has landed (each wave waited for its own) and every
// wave's reads of the stage about to be refilled are done.  One asm statement, so its
// "memory" clobber orders it against the compiler's LDS accesses on both sides.
template <int N>
__device__ __forceinline__ void stage_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
// runtime-selected immediate (wave-uniform n in [0, 24])
__device__ __forceinline__ void stage_barrier_n(int n) {
  switch (n) {
#define RNNT_SB(v) \
  case v: stage_barrier<v>(); break;
    RNNT_SB(0) RNNT_SB(2) RNNT_SB(4) RNNT_SB(6) RNNT_SB(8) RNNT_SB(10) RNNT_SB(12) RNNT_SB(14) RNNT_SB(16)
    RNNT_SB(18) RNNT_SB(20) RNNT_SB(22) RNNT_SB(24)
#undef RNNT_SB
    default: stage_barrier<0>(); break;
  }
}

// byte offset of (row r, byte b < 128) in a swizzled [rows][128 B] epilogue image
__device__ __forceinline__ int cimg_off(int r, int b) { return r * 128 + ((((b >> 4) ^ r) & 7) << 4) + (b & 15); }

// RNNT_PERSIST 2 (persistent workgroups, 128-byte stages): the next tile's stage 0 (job nx, tile
// nmt/nnt; nx == nullptr: none) is DMA'd during this tile's epilogue into the buffer the last
// stage used; roff: this tile's ring offset (stage s in buffer (s + roff) & 1); pre0: stage 0
// was issued by the previous tile.
__device__ __forceinline__ void lstm_i8_step(const EncStepArgs& a, int mt, int nt, int8_t* smem,
                                             unsigned long long st_t0 = 0ull, const EncStepArgs* nxp = nullptr,
                                             bool has_nx = false, int nmt = 0, int nnt = 0, int roff = 0,
                                             bool pre0 = false) {
  (void)nxp; (void)has_nx; (void)nmt; (void)nnt; (void)roff; (void)pre0;
  (void)st_t0;
#ifdef RNNT_DEV_STAMPS
  unsigned est_k;
  {
    unsigned v = 0;
    if (threadIdx.x == 0) v = atomicAdd(&g_est_n, 1u);
    est_k = __builtin_amdgcn_readfirstlane(v);  // wave 0 (the only writer) holds thread 0's ticket
  }
  EST_PUT(2, st_t0);
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 3, wn = wave >> 2;
  const int m0 = mt * BM;  // packed gate row base
  const int n0 = nt * BN;  // batch row base
  const int K = a.I + H;
  const int nK = K / BK;

  // ---- epilogue operands, prefetched so their latency hides under the main loop
  const int q = lane >> 4, col = lane & 15;
  const int u0 = (m0 >> 2) + wm * 16 + q * 4;  // this lane's 4 consecutive units
  const int nb = n0 + wn * 128 + col;          // batch row of j = 0 (row j: nb + 16 j)
  // ---- LDS-DMA staging: wave w moves A pieces APW*w .. +APW-1 and B pieces 2w, 2w+1 (16 rows x
  // 64 B each); lane l of piece p lands at LDS slot 64p + l = row*4 + (col16 ^ h(row)), so it
  // fetches row 16p + (l>>2), 16-byte column (l&3) ^ h, where h(row) depends on l>>4 only.
  const int hx = (0x1320 >> ((lane >> 4) * 4)) & 3;
  const int gcol = ((lane & 3) ^ hx) * 16;
  const int rA = wave * APW * 16 + (lane >> 2);  // first row of this wave's A pieces (+16 each)
  const int rB = wave * BPW * 16 + (lane >> 2);  // first row of its B pieces
#ifdef RNNT_DEV_SAME_TILE  // development ablation: every workgroup stages tile (0, 0) (L2-resident)
  const int lm0 = 0, ln0 = 0;
#else
  const int lm0 = m0, ln0 = n0;
#endif
  // per-lane 32-bit offsets from wave-uniform (SGPR) tile bases: global_load_lds with saddr
  const uint32_t oA = (uint32_t)(rA * K + gcol), oX = (uint32_t)(rB * a.I + gcol), oH = (uint32_t)(rB * H + gcol);
  const int8_t* wbase = a.W + (size_t)lm0 * K;
  const int8_t* xbase0 = a.x + (size_t)ln0 * a.I;
  const int8_t* xbase1 = xbase0 + (size_t)16 * a.I;
  const int8_t* hbase0 = a.h_in + (size_t)ln0 * H - a.I;
  const int8_t* hbase1 = hbase0 + (size_t)16 * H;
  lds_char* lds = (lds_char*)(lds_void*)smem;
  const int pa = wave * APW * 1024, pb = A_BYTES + wave * BPW * 1024;

  // piece j (0..GLDS_PER_STAGE-1) of stage ks: A pieces first, then the two B pieces
  auto issue_piece = [&](int ks, int j) __attribute__((always_inline)) {
#ifdef RNNT_DEV_NO_LOAD  // development ablation: no staging (MFMA on stale LDS)
    return;
#endif
    const int k = ks * BK;
    lds_char* st = lds + (ks % NSTAGE) * STAGE_BYTES;
    if (j < APW) {
      __builtin_amdgcn_global_load_lds((glb_void*)(wbase + (size_t)(16 * j) * K + k + oA), (lds_void*)(st + pa + j * 1024), 16,
                                       0, 0);
    } else if (k < a.I) {
      __builtin_amdgcn_global_load_lds((glb_void*)((j == APW ? xbase0 : xbase1) + k + oX),
                                       (lds_void*)(st + pb + (j - APW) * 1024), 16, 0, 0);
    } else {
      __builtin_amdgcn_global_load_lds((glb_void*)((j == APW ? hbase0 : hbase1) + k + oH),
                                       (lds_void*)(st + pb + (j - APW) * 1024), 16, 0, 0);
    }
  };
  auto issue = [&](int ks) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < GLDS_PER_STAGE; ++j) issue_piece(ks, j);
  };

  // the tile's fp16 cell state (BN rows x 64 units x 2 B) DMA'd into the ring buffer of stage
  // nK-NSTAGE once it has been read; piece p, lane l: row 8p + (l>>3), 16-B chunk l&7
#if RNNT_BK128
  // two 64 KiB stages of 128-byte rows; the cell state goes into the buffer the last stage does
  // not occupy (stage nS-2's, issued once that stage's reads are retired)
  const int nS = K / 128;
  const int cbuf = ((nS + roff) & 1) * 65536;
#else
  const int cbuf = ((nK - NSTAGE) % NSTAGE) * STAGE_BYTES;
#endif
  auto issue_c = [&]() __attribute__((always_inline)) {
    // image row r holds logical 16-B chunk ch at chunk slot ch ^ (r & 7) (cimg_off), so the
    // epilogue's per-lane 8-byte accesses of 16 consecutive rows hit 2-way instead of 8-way
    // bank conflicts; lane l of piece p lands in slot l & 7 of row 8p + (l >> 3)
    const uint16_t* cb = a.c + (size_t)n0 * H + (m0 >> 2) + ((lane & 7) ^ ((lane >> 3) & 7)) * 8;
#pragma unroll
    for (int pc = 0; pc < C_GLDS; ++pc) {
      const int p = wave * C_GLDS + pc;
      __builtin_amdgcn_global_load_lds((glb_void*)(cb + (size_t)(8 * p + (lane >> 3)) * H), (lds_void*)(lds + cbuf + p * 1024),
                                       16, 0, 0);
    }
  };

  v4i acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  // fragment reads: A rows wm*64 + i*16 + (lane&15), B rows wn*128 + j*16 + (lane&15), 16-byte
  // column lane>>4; +16 rows is +1 KiB in the image (the swizzle repeats every 16 rows)
  const int fa = swz(wm * 64 + col, q), fb = A_BYTES + swz(wn * 128 + col, q);
  (void)nK; (void)fa; (void)fb; (void)issue;  // the 64-byte-stage loops' helpers (unused with RNNT_BK128)

#if RNNT_BK128
  // 128-byte staging: a stage holds two MFMA k steps (K bytes k0..k0+127) of all 256 A and 256 B
  // rows, so each LDS-DMA piece moves 8 whole 128-byte rows (8 full cache lines) instead of 16
  // half lines -- half the address/tag work per byte on the load path.  Image: 16-byte column c
  // of row r at slot c ^ ((r >> 1) & 7) (rows of 128 B, two per 256-byte bank row): conflict-free
  // for the ds_read_b128 lane groups.  Two buffers: stage s+1 is DMA'd while stage s is consumed.
  static_assert(BM == 256 && BN == 256 && NWAVE == 8, "128-byte staging layout");
  {
    const int r8 = lane >> 3;                                   // row within a piece
    const int sl = lane & 7;                                    // 16-byte slot within the row
    const int gc0 = (sl ^ ((r8 >> 1) & 7)) * 16;                // even pieces: rows 8p + r8, p even
    const int gc1 = (sl ^ (((8 + r8) >> 1) & 7)) * 16;          // odd pieces
    // per-lane 32-bit offsets (even / odd pieces differ in the swizzle) from SGPR tile bases
    const uint32_t rl = (uint32_t)(32 * wave + r8);
    const uint32_t oA0 = rl * K + gc0, oA1 = rl * K + gc1;
    const uint32_t oX0 = rl * a.I + gc0, oX1 = rl * a.I + gc1;
    const uint32_t oH0 = rl * H + gc0, oH1 = rl * H + gc1;
    auto issue128A = [&](int s, int jb = 0, int je = 4) __attribute__((always_inline)) {
      const int k = s * 128;
      lds_char* st = lds + ((s + roff) & 1) * 65536 + wave * 4096;
#pragma unroll
      for (int j = jb; j < je; ++j)  // A pieces 4w..4w+3: rows 32w + 8j + r8
        __builtin_amdgcn_global_load_lds((glb_void*)(wbase + (size_t)(8 * j) * K + k + ((j & 1) ? oA1 : oA0)),
                                         (lds_void*)(st + j * 1024), 16, 0, 0);
    };
    auto issue128B = [&](int s, int jb = 0, int je = 4) __attribute__((always_inline)) {
      const int k = s * 128;
      lds_char* st = lds + ((s + roff) & 1) * 65536 + wave * 4096;
      if (k < a.I) {
#pragma unroll
        for (int j = jb; j < je; ++j)
          __builtin_amdgcn_global_load_lds((glb_void*)(xbase0 + (size_t)(8 * j) * a.I + k + ((j & 1) ? oX1 : oX0)),
                                           (lds_void*)(st + 32768 + j * 1024), 16, 0, 0);
      } else {
#pragma unroll
        for (int j = jb; j < je; ++j)
          __builtin_amdgcn_global_load_lds((glb_void*)(hbase0 + (size_t)(8 * j) * H + k + ((j & 1) ? oH1 : oH0)),
                                           (lds_void*)(st + 32768 + j * 1024), 16, 0, 0);
      }
    };
    auto issue128 = [&](int s) __attribute__((always_inline)) {
      issue128A(s);
      issue128B(s);
    };
    // issue points of stage s+1's pieces inside stage s (RNNT_BK128_ISSUE >= 2): 0 top (after the
    // barrier), 1 after half of the first k step, 2 after the first k step, 3 after half of the
    // second.  2: A@0 B@2;  3: A0-1@0 A2-3@1 B0-1@2 B2-3@3;  4: A@0 B@1;  5: A0-1 B0-1@0 A2-3 B2-3@2
    auto issue_at = [&](int pt, int s) __attribute__((always_inline)) {
      constexpr int M = RNNT_BK128_ISSUE;
      if (M == 2) { if (pt == 0) issue128A(s); if (pt == 2) issue128B(s); }
      if (M == 3) {
        if (pt == 0) issue128A(s, 0, 2);
        if (pt == 1) issue128A(s, 2, 4);
        if (pt == 2) issue128B(s, 0, 2);
        if (pt == 3) issue128B(s, 2, 4);
      }
      if (M == 4) { if (pt == 0) issue128A(s); if (pt == 1) issue128B(s); }
      if (M == 5) {
        if (pt == 0) { issue128A(s, 0, 2); issue128B(s, 0, 2); }
        if (pt == 2) { issue128A(s, 2, 4); issue128B(s, 2, 4); }
      }
    };
    const int sw = col >> 1;  // (row >> 1) & 7 for rows 16i + col
    const int fa0 = (wm * 64 + col) * 128, fb0 = 32768 + (wn * 128 + col) * 128;
    // RNNT_BK128_ISSUE 2: every wave issues its A pieces of stage s+1 at the top of stage s and
    // its B pieces after the first k step's MFMAs (the load path sees two half bursts per stage);
    // 1: waves 4-7 issue all of theirs after the first k step; 0: all at the top
    const bool late = RNNT_BK128_ISSUE == 1 && wn == 1;
    if (!pre0) issue128(0);
#ifdef RNNT_DEV_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stamps only: stage 0 landed (this wave)
    EST_PUT(3, __builtin_amdgcn_s_memrealtime());
    EST_PUT(6, __builtin_amdgcn_s_memtime());
#endif
    for (int s = 0; s < nS; ++s) {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (RNNT_BK128_ISSUE >= 2) {
        if (s + 1 < nS) issue_at(0, s + 1);
        else issue_c();
      } else if (!late) {
        if (s + 1 < nS) issue128(s + 1);
        else issue_c();
      }
      const int8_t* st = smem + ((s + roff) & 1) * 65536;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int cs = ((kk * 4 + q) ^ sw) << 4;
        v4i fra[4], frb[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) fra[i] = *(const v4i*)(st + fa0 + cs + i * 2048);
#pragma unroll
        for (int j = 0; j < 8; ++j) frb[j] = *(const v4i*)(st + fb0 + cs + j * 2048);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if ((RNNT_BK128_ISSUE == 3 || (RNNT_BK128_ISSUE == 4 && kk == 0)) && i == 2 && s + 1 < nS) {
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            issue_at(2 * kk + 1, s + 1);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fra[i], frb[j], acc[i][j], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if ((RNNT_BK128_ISSUE == 2 || RNNT_BK128_ISSUE == 3 || RNNT_BK128_ISSUE == 5) && kk == 0 && s + 1 < nS) {
          issue_at(2, s + 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (late && kk == 0) {
          __builtin_amdgcn_sched_barrier(0);
          if (s + 1 < nS) issue128(s + 1);
          else issue_c();
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
#else
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s) issue(s);  // nK >= 20 for every layer
#if RNNT_PRIO_MODE != 0
  if (RNNT_STAGGER && wn == 1) __builtin_amdgcn_s_setprio(1);
#endif
  for (int ks = 0; ks < nK; ++ks) {
    // LDS-DMA this wave may leave in flight: the stages issued after ks (min(NSTAGE - 2,
    // nK - 1 - ks)) and, once issued (step nK-NSTAGE+1, into stage nK-NSTAGE's buffer), the
    // cell-state pieces
    const int later = nK - 1 - ks < NSTAGE - 2 ? nK - 1 - ks : NSTAGE - 2;
    stage_barrier_n(later * GLDS_PER_STAGE + (ks > nK - NSTAGE + 1 ? C_GLDS : 0));
#ifdef RNNT_DEV_STAMPS
    if (ks == 0) {
      EST_PUT(3, __builtin_amdgcn_s_memrealtime());
      EST_PUT(6, __builtin_amdgcn_s_memtime());
    }
#endif
#if !RNNT_INTERLEAVE
    // RNNT_STAGGER: waves 4-7 (each the SIMD partner of wave w-4) issue their pieces after half
    // of their MFMAs, so one wave of a SIMD issues LDS-DMA while its partner runs MFMAs
    const bool late = RNNT_STAGGER && wn == 1;
    if (!late) {
      if (ks + NSTAGE - 1 < nK) issue(ks + NSTAGE - 1);
      else if (ks + NSTAGE - 1 == nK) issue_c();
    }
#else
    const bool next = ks + NSTAGE - 1 < nK;
    if (ks + NSTAGE - 1 == nK) issue_c();
#endif
    const int8_t* st = smem + (ks % NSTAGE) * STAGE_BYTES;
    v4i fra[4], frb[8];
#ifdef RNNT_DEV_NO_READ  // development ablation: MFMA on register-resident fragments
#pragma unroll
    for (int i = 0; i < 4; ++i) fra[i] = v4i{ks, i, 1, 2};
#pragma unroll
    for (int j = 0; j < 8; ++j) frb[j] = v4i{j, ks, 3, 4};
    asm volatile("" : "+v"(fra[0]), "+v"(frb[0]));
    (void)st;
#else
#pragma unroll
    for (int i = 0; i < 4; ++i) fra[i] = *(const v4i*)(st + fa + i * 1024);
#pragma unroll
    for (int j = 0; j < 8; ++j) frb[j] = *(const v4i*)(st + fb + j * 1024);
#endif
#ifdef RNNT_DEV_NO_MFMA  // development ablation: staging + LDS reads only
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(fra[i]), "v"(frb[i]), "v"(frb[i + 4]));
#else
#if RNNT_PRIO_MODE == 0
    __builtin_amdgcn_s_setprio(1);  // MFMA cluster at raised priority (guide T5)
#elif RNNT_PRIO_MODE == 1
    if (!late) __builtin_amdgcn_s_setprio(1);  // late waves hold priority 1 for the whole loop
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#if RNNT_INTERLEAVE
      // the next stage's LDS-DMA pieces spread between the MFMA groups
#pragma unroll
      for (int pj = i * GLDS_PER_STAGE / 4; pj < (i + 1) * GLDS_PER_STAGE / 4; ++pj)
        if (next) issue_piece(ks + NSTAGE - 1, pj);
      __builtin_amdgcn_sched_barrier(0);
#endif
#if !RNNT_INTERLEAVE
      if (RNNT_STAGGER && i == RNNT_STAGGER_AT) {
        __builtin_amdgcn_sched_barrier(0);
        if (late) {
          if (ks + NSTAGE - 1 < nK) issue(ks + NSTAGE - 1);
          else if (ks + NSTAGE - 1 == nK) issue_c();
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#endif
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fra[i], frb[j], acc[i][j], 0, 0, 0);
#if RNNT_INTERLEAVE
      __builtin_amdgcn_sched_barrier(0);
#endif
    }
#if RNNT_PRIO_MODE == 0
    __builtin_amdgcn_s_setprio(0);
#elif RNNT_PRIO_MODE == 1
    if (!late) __builtin_amdgcn_s_setprio(0);
#endif
#endif
  }
#endif
#if RNNT_PRIO_MODE != 0
  __builtin_amdgcn_s_setprio(0);
#endif
  stage_barrier<0>();  // the cell-state DMA has landed for every wave
#ifdef RNNT_DEV_STAMPS
  EST_PUT(4, __builtin_amdgcn_s_memrealtime());
  EST_PUT(7, __builtin_amdgcn_s_memtime());
#endif
#ifdef RNNT_DEV_NO_EPI  // development ablation: main loop only
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(acc[i][j]));
  return;
#endif

  // ---- fused LSTM cell epilogue (quant_lstm.py:162-183 semantics; oracle_enc_cell)
  const float As = a.rb * 4.0f, Ag = a.rb * 8.0f, ins = a.in_s, outs = a.out_s;
  // table lookups are random gathers: with 16 copies, entry k of copy s at slot 16k + s, lane l
  // reads copy l & 15, so the 16 lanes of each ds_read_b128 lane group ({0-3,12-15,20-27}, ...)
  // sit on 16 distinct bank slots whatever entries they pick (no bank conflicts)
  const float4* tab = (const float4*)(smem + TAB_OFF) + (TAB_COPIES == 16 ? (lane & 15) : 0);
  float4 bq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#ifdef RNNT_DEV_EPI_NOBQ  // development ablation: no bias load
    bq[i] = float4{64.0f, 64.0f, 64.0f, 64.0f};
#else
    bq[i] = *(const float4*)(a.bq + m0 + wm * 64 + i * 16 + q * 4);
#endif
  }
  // results go to LDS first and leave as whole 128-/64-byte row segments (16 B per lane,
  // full cache lines per wave instruction) instead of 4-/8-byte scattered per-lane stores:
  // c_new in place over the c_in image (each lane rewrites exactly what it read), h and y / the
  // bf16 output in two other ring buffers (all free after the main loop)
  const int ul = u0 - (m0 >> 2);  // this lane's first unit within the tile's 64
#if RNNT_BK128
  lds_char* hs = lds + cbuf + 32768;
  // with a next-tile prefetch the last stage's buffer is taken: the int8 y image goes after the
  // table (the caller passes no next tile for ENC_OUT_FINAL, whose bf16 image needs 32 KiB)
  lds_char* ys = (RNNT_PERSIST == 2 && has_nx) ? lds + YS_OFF : lds + ((nS - 1 + roff) & 1) * 65536;
#if RNNT_PERSIST == 2
  if (has_nx) {
    const EncStepArgs* nx = nxp;
    // next tile's stage 0 into the last stage's buffer (its reads retired at the barrier above);
    // issued after the bias loads so waiting for those does not wait for these
    asm volatile("" ::: "memory");
    const int K2 = nx->I + H, I2 = nx->I;
    const int r8 = lane >> 3, sl = lane & 7;
    const uint32_t gc0 = (sl ^ ((r8 >> 1) & 7)) * 16, gc1 = (sl ^ (((8 + r8) >> 1) & 7)) * 16;
    const uint32_t rl = (uint32_t)(32 * wave + r8);
    const int8_t* wb = nx->W + (size_t)nmt * BM * K2;
    const int8_t* xb = nx->x + (size_t)nnt * BN * I2;
    lds_char* st = lds + ((nS - 1 + roff) & 1) * 65536 + wave * 4096;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((glb_void*)(wb + (size_t)(8 * j) * K2 + ((j & 1) ? rl * K2 + gc1 : rl * K2 + gc0)),
                                       (lds_void*)(st + j * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j)  // k = 0 < I2: the x part
      __builtin_amdgcn_global_load_lds((glb_void*)(xb + (size_t)(8 * j) * I2 + ((j & 1) ? rl * I2 + gc1 : rl * I2 + gc0)),
                                       (lds_void*)(st + 32768 + j * 1024), 16, 0, 0);
  }
#endif
#else
  lds_char* hs = lds + ((cbuf / STAGE_BYTES + 1) % NSTAGE) * STAGE_BYTES;
  lds_char* ys = lds + ((cbuf / STAGE_BYTES + 2) % NSTAGE) * STAGE_BYTES;
#endif
  constexpr int HP = 80;  // int8 image pitch (64 B + 16: conflict-free 4-byte writes, 16-B aligned rows)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = nb + 16 * j, r = n - n0;
    const uint2 cv = *(const uint2*)(smem + cbuf + cimg_off(r, ul * 2));
    const float cin[4] = {h2f((uint16_t)(cv.x & 0xffff)), h2f((uint16_t)(cv.x >> 16)), h2f((uint16_t)(cv.y & 0xffff)),
                          h2f((uint16_t)(cv.y >> 16))};
    uint32_t cw[2] = {0u, 0u}, hq = 0, yq = 0;
    float hv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float cn, hh;
      enc_cell<TAB_COPIES>(tab, acc[i][j], bq[i], As, Ag, cin[i], cn, hh);
      cw[i >> 1] |= (uint32_t)f2h(cn) << (16 * (i & 1));
      hv[i] = hh;
      hq |= (uint32_t)(uint8_t)q8(hh * ins) << (8 * i);
      yq |= (uint32_t)(uint8_t)q8(hh * outs) << (8 * i);
    }
#ifdef RNNT_DEV_EPI_NOSTORE  // development ablation: results kept live, nothing stored
    asm volatile("" ::"v"(cw[0]), "v"(cw[1]), "v"(hq), "v"(yq), "v"(hv[0]));
    continue;
#endif
    *(uint2*)(smem + cbuf + cimg_off(r, ul * 2)) = uint2{cw[0], cw[1]};
    *(uint32_t*)(hs + r * HP + ul) = hq;
    if (a.mode == ENC_OUT_FINAL) {
      if (a.y32) *(float4*)(a.y32 + (size_t)n * H + u0) = float4{hv[0], hv[1], hv[2], hv[3]};
      *(uint2*)(ys + cimg_off(r, ul * 2)) = uint2{(uint32_t)f2bf_ftz(hv[0]) | ((uint32_t)f2bf_ftz(hv[1]) << 16),
                                               (uint32_t)f2bf_ftz(hv[2]) | ((uint32_t)f2bf_ftz(hv[3]) << 16)};
    } else {
      *(uint32_t*)(ys + r * HP + ul) = yq;
    }
  }
#ifdef RNNT_DEV_EPI_NOSTORE
  return;
#endif
  // the staged images are complete: LDS writes retired + barrier.  Not __syncthreads(): its
  // fence waits vmcnt(0), i.e. for a next-tile prefetch (RNNT_PERSIST 2) still in flight
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  // copy-out: thread t moves 16-byte chunks; a wave instruction writes 8 (c, bf16 f) or 16 (h, y)
  // whole row segments
  const int um = m0 >> 2;
#pragma unroll
  for (int it = 0; it < BN * 8 / (NWAVE * 64); ++it) {  // c: BN rows x 128 B
    const int idx = it * NWAVE * 64 + tid, r = idx >> 3, ch = idx & 7;
    *(uint4*)(a.c + (size_t)(n0 + r) * H + um + ch * 8) = *(const uint4*)(smem + cbuf + cimg_off(r, ch * 16));
    if (a.mode == ENC_OUT_FINAL)
      *(uint4*)(a.fbf + (size_t)(n0 + r) * H + um + ch * 8) = *(const uint4*)(ys + cimg_off(r, ch * 16));
  }
#pragma unroll
  for (int it = 0; it < BN * 4 / (NWAVE * 64); ++it) {  // h, y: BN rows x 64 B
    const int idx = it * NWAVE * 64 + tid, r = idx >> 2, ch = idx & 3, n = n0 + r;
    *(uint4*)(a.h_out + (size_t)n * H + um + ch * 16) = *(const uint4*)(hs + r * HP + ch * 16);
    if (a.mode == ENC_OUT_I8) {
      *(uint4*)(a.y8 + (size_t)n * H + um + ch * 16) = *(const uint4*)(ys + r * HP + ch * 16);
    } else if (a.mode == ENC_OUT_STACKED) {
      // StackTime (modeling_rnnt.py:314-324): frame t -> stacked frame t/2, half t%2;
      // frames t >= x_lens[n] are zeroed; the odd-T pad frame is zero too.
      int8_t* dst = a.y8 + (size_t)n * (2 * H) + um + ch * 16;
      const uint4 z = uint4{0u, 0u, 0u, 0u};
      *(uint4*)(dst + a.half * H) = (a.t < a.lens[n]) ? *(const uint4*)(ys + r * HP + ch * 16) : z;
      if (a.zero_next) *(uint4*)(dst + H) = z;
    }
  }
#ifdef RNNT_DEV_STAMPS
  EST_PUT(5, __builtin_amdgcn_s_memrealtime());
  EST_PUT(0, (unsigned long long)K | ((unsigned long long)mt << 16) | ((unsigned long long)nt << 24) |
                 ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 32));  // HW_REG_HW_ID
  EST_PUT(1, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20));        // HW_REG_XCC_ID
#endif
}

// One launch = one wavefront tick: up to 5 independent layer-steps (jobs, longest K first).
// XCD-aware tile order: workgroup id -> XCD id % 8 (round-robin dispatch).  XCD x takes gate
// tiles 4(x&3)..4(x&3)+3 and the (x>>2)-th half of each job's active batch tiles, so the 32
// workgroups resident on an XCD share 4 weight tiles and ~8 activation tiles through its L2
// (weights fetched from HBM/MALL 2x, activations 4x per tick, instead of 1x / 8x).
// 2 waves per SIMD either way: one 8-wave workgroup per CU (ENC_WN 2) or two 4-wave ones (1)
#ifndef RNNT_XCD_G  // gate tiles per XCD: 4 (x 1/2 of the batch tiles) or 8 (x 1/4)
#define RNNT_XCD_G 4
#endif
constexpr int XG = RNNT_XCD_G;           // gate tiles per XCD
constexpr int XGG = 16 / XG;             // gate groups
constexpr int XP = 8 / XGG;              // batch parts
static_assert(XG == 4 || XG == 8, "XCD tile map");
// job tile k (0..) of XCD xcd -> (mt, nt); batch part p = tiles [p*nbt/XP, (p+1)*nbt/XP)
__device__ __forceinline__ int xcd_pick(const EncTickArgs& args, int xcd, int k, int& mt, int& nt) {
  const int gsel = xcd % XGG, psel = xcd / XGG;
  for (int j = 0; j < args.njobs; ++j) {
    const int nbt = args.nbt[j];
    const int b0 = XG == 4 ? (psel ? (nbt + 1) >> 1 : 0) : psel * nbt / XP;
    const int b1 = XG == 4 ? (psel ? nbt : (nbt + 1) >> 1) : (psel + 1) * nbt / XP;
    const int cnt = XG * (b1 - b0);
    if (k < cnt) {
      mt = gsel * XG + (k % XG);
      nt = b0 + k / XG;
      return j;
    }
    k -= cnt;
  }
  return -1;
}
constexpr int WG_PER_CU = ENC_WN == 2 ? 1 : 2;
constexpr int SLOTS_PER_XCD = 32 * WG_PER_CU;  // resident workgroups per XCD (32 CUs)
__global__ void __launch_bounds__(NWAVE * 64, WG_PER_CU) lstm_i8_tick_kernel(EncTickArgs args) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  const int xcd = blockIdx.x & 7;
  unsigned long long st_t0 = 0ull;
  EST_MARK(st_t0);
#pragma unroll
  for (int it = 0; it < 128 * TAB_COPIES / (NWAVE * 64); ++it) {
    const int idx = it * NWAVE * 64 + threadIdx.x;
    ((float4*)(smem + TAB_OFF))[idx] = g_act_tab[TAB_COPIES == 16 ? idx >> 4 : idx];
  }
  if (128 * TAB_COPIES < NWAVE * 64 && threadIdx.x < 128 * TAB_COPIES)
    ((float4*)(smem + TAB_OFF))[threadIdx.x] = g_act_tab[TAB_COPIES == 16 ? threadIdx.x >> 4 : threadIdx.x];  // read after the
  // first stage barrier of the main loop (lgkmcnt(0) + s_barrier)
  // RNNT_PERSIST: workgroup (xcd, slot) takes the XCD's tiles slot, slot + SLOTS_PER_XCD, ... in
  // the order one-tile-per-workgroup rounds would run them (a layer-step 4 % shorter alone, but
  // the resident grid then starves the other streams' decode kernels: off by default)
  const int stride = RNNT_PERSIST ? (int)(gridDim.x >> 3) : 1 << 30;
#if RNNT_PERSIST == 2
  static_assert(RNNT_BK128, "next-tile prefetch uses the 128-byte stage ring");
  auto pick = [&](int k, int& mt, int& nt) -> int { return xcd_pick(args, xcd, k, mt, nt); };
  int k0 = blockIdx.x >> 3, mt = 0, nt = 0;
  int jsel = pick(k0, mt, nt);
  int roff = 0;
  bool pre0 = false;
  while (jsel >= 0) {
    int nmt = 0, nnt = 0;
    const int jn = pick(k0 + stride, nmt, nnt);
    // the previous tile's epilogue LDS reads are done (raw barrier: the prefetched stage 0 and
    // the copy-out stores may stay in flight)
    if (k0 != (int)(blockIdx.x >> 3)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const EncStepArgs& cur = args.job[__builtin_amdgcn_readfirstlane(jsel)];
    const bool pf = jn >= 0 && cur.mode != ENC_OUT_FINAL;
    lstm_i8_step(cur, __builtin_amdgcn_readfirstlane(mt), __builtin_amdgcn_readfirstlane(nt), smem, st_t0,
                 &args.job[__builtin_amdgcn_readfirstlane(jn >= 0 ? jn : jsel)], pf,
                 __builtin_amdgcn_readfirstlane(nmt), __builtin_amdgcn_readfirstlane(nnt), roff, pre0);
    roff = ((cur.I + H) / 128 - 1 + roff) & 1;  // the next tile starts in the last stage's buffer
    pre0 = pf;
    jsel = jn;
    mt = nmt;
    nt = nnt;
    k0 += stride;
  }
  return;
#endif
  for (int k0 = blockIdx.x >> 3;; k0 += stride) {
    int mt = 0, nt = 0;
    const int jsel = xcd_pick(args, xcd, k0, mt, nt);
    if (jsel < 0) return;
    if (k0 != (int)(blockIdx.x >> 3)) __syncthreads();  // the previous tile's epilogue LDS reads are done
    // wave-uniform runtime index into the kernarg segment: the job's fields stay scalar loads
    lstm_i8_step(args.job[__builtin_amdgcn_readfirstlane(jsel)], __builtin_amdgcn_readfirstlane(mt),
                 __builtin_amdgcn_readfirstlane(nt), smem, st_t0);
  }
}

// ---------------------------------------------------------------- host launchers
int launch_quantize(const float* feat, int64_t n, float s, int8_t* out, hipStream_t st) {
  const int64_t n4 = n / 4;
  int grid = (int)((n4 + 255) / 256);
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(quantize_kernel, dim3(grid), dim3(256), 0, st, (const float4*)feat, n4, s, (uint32_t*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_quantize_gather(const float* store, const int64_t* offsets, const int32_t* lens, int T, int n, int n_pad,
                           float s, int8_t* out, hipStream_t st) {
  const int64_t words = (int64_t)T * n_pad * 64;
  int grid = (int)((words + 255) / 256);
  if (grid > 16384) grid = 16384;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(quantize_gather_kernel, dim3(grid), dim3(256), 0, st, store, offsets, lens, n, n_pad, words, s,
                     (uint32_t*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_lstm_i8_tick(const EncTickArgs& a, hipStream_t st) {
  static std::atomic<uint64_t> attr{0};
  if (set_smem_attr_once((const void*)lstm_i8_tick_kernel, SMEM_BYTES, attr)) return -1;
  // shapes the kernel's staging assumes (checked on the host: a mismatch would read out of bounds)
  for (int j = 0; j < a.njobs; ++j) {
    const int K = a.job[j].I + H;
    if (a.job[j].I % (RNNT_BK128 ? 128 : BK) != 0 || K % (RNNT_BK128 ? 128 : BK) != 0 || a.nbt[j] < 0) return -1;
  }
  int per_xcd = 0;  // the batch-half-0 XCDs carry the larger half
  for (int j = 0; j < a.njobs; ++j) per_xcd += XG * ((a.nbt[j] + XP - 1) / XP);  // the largest part
  if (per_xcd <= 0) return 0;
#ifndef RNNT_PERSIST_FREE  // persistent grids: workgroup slots per XCD left to other streams
#define RNNT_PERSIST_FREE 0
#endif
  constexpr int PSLOTS = SLOTS_PER_XCD - RNNT_PERSIST_FREE;
  const int grid = 8 * (RNNT_PERSIST && per_xcd > PSLOTS ? PSLOTS : per_xcd);
  hipLaunchKernelGGL(lstm_i8_tick_kernel, dim3(grid), dim3(NWAVE * 64), SMEM_BYTES, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rnnt

#ifdef RNNT_DEV_STAMPS
// development: copy out (and reset) the tick kernel's per-tile stamp records (8 x u64 each)
extern "C" int rnnt_dev_read_enc_stamps(unsigned long long* out, int max_records) {
  unsigned int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(rnnt::g_est_n), sizeof(n)) != hipSuccess) return -1;
  if (n > (1u << 22) / 8) n = (1u << 22) / 8;
  if ((int)n > max_records) n = max_records;
  if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(rnnt::g_est), (size_t)n * 8 * 8) != hipSuccess) return -1;
  const unsigned int z = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(rnnt::g_est_n), &z, sizeof(z)) != hipSuccess) return -1;
  return (int)n;
}
#endif
