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
#include <stdlib.h>
#include <string.h>

#include "rnnt_device.hpp"
#include "encoder.hpp"

namespace rnnt {

// sigma table of the cell (tools/gen_act_table.py), copied to LDS by every workgroup
__device__ const __attribute__((aligned(16))) float2 g_act_tab[ENC_TAB_N] = {
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
// 16-word records: 0-7 the tile's timeline; 8, 9, 10: shader clocks of the main loop spent at the stage
// barriers (wait_stage), from a barrier to the end of the stage's MFMA issue, and stages
#define EST_W 16
#define EST_PUT(i, v) \
  if (threadIdx.x == 0 && est_k < (1u << 22) / EST_W) g_est[EST_W * est_k + (i)] = (v)
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
// Workgroup tile: BM packed gate rows (BM/4 units) x BN batch rows, K swept in 128-byte stages;
// 8 waves as 4 (gate) x 2 (batch), each wave WMT x WNT MFMA 16x16x64 tiles (BM = 64 WMT,
// BN = 32 WNT).  Two shapes:
//   * 256 x 256 (WMT 4, WNT 8): 128 accumulator VGPRs per lane at 2 waves/SIMD, one workgroup
//     per CU -- the largest tile whose int32 accumulators fit the register file; it balances the
//     per-CU L2->LDS load path against the MFMA.  Ticks with many tiles.
//   * 128 x 128 (WMT 2, WNT 4): 32 accumulator VGPRs, 80 KiB of LDS, two workgroups per CU --
//     8x the tiles of a layer-step, each with a quarter of the bytes per stage.  Ticks that would
//     leave CUs idle with the large tile: small batches, the tail ticks of a length-sorted batch.
constexpr int NWAVE = 8;
template <int WMT, int WNT, int NBUF_ = 2>
struct TileCfg {
  static constexpr int BM = 64 * WMT, BN = 32 * WNT;
  static constexpr int NBUF = NBUF_;             // stage ring depth (NBUF - 1 stages in flight)
  static constexpr int STAGE = (BM + BN) * 128;  // one stage: 128 K bytes of BM A + BN B rows
  static constexpr int TAB_OFF = NBUF * STAGE;   // LDS: sigma table after the stage ring
  static constexpr int SMEM = TAB_OFF + ENC_TAB_N * 8;
  static constexpr int PA = BM / 64, PB = BN / 64;  // 1 KiB DMA pieces per wave per stage (A, B)
  static constexpr int CROW = BM / 2;            // fp16 cell-state bytes per batch row of the tile
  static constexpr int CPR = CROW / 16;          // 16-byte chunks per cell-state row
  static constexpr int HC = BM / 64;             // 16-byte chunks per int8 h / y row
  static constexpr int HP = BM / 4 + 16;         // int8 image pitch (16-B aligned rows, offset banks)
  static constexpr int NGT = G4 / BM;            // gate tiles per layer-step
  static constexpr int GPX = NGT / 4;            // gate tiles per XCD group
  static_assert(NGT % 8 == 0, "one-batch-tile jobs deal their gate tiles to 8 XCDs");
  static_assert(BM >= 64 && BN >= 128, "one A piece (8 rows) per wave at least");
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static_assert(BN * CROW + BN * HP <= STAGE, "c and h images share one stage buffer");
  static constexpr int CPIECES = BN * CPR / 64;   // 1 KiB DMA pieces of the tile's fp16 cell state
  static_assert(CPIECES % NWAVE == 0 || CPIECES < NWAVE, "c DMA pieces per wave");
};
using BigTile = TileCfg<4, 8>;
using SmallTile = TileCfg<2, 4>;
// 64 gate rows x 128 batch rows, 4-deep ring (112 KiB): ticks whose jobs all have one batch tile
// (batches of <= 128 rows, config 3) -- twice the workgroups of the small tile, each moving
// (64 + 128) K instead of (128 + 128) K bytes, so the K loop of the widest job is a quarter shorter
using MiniTile = TileCfg<1, 4, 4>;
// the small tile with a 4-deep ring (144 KiB, one workgroup per CU) for ticks of at most one
// workgroup per CU: a K loop with one stage in flight is latency-bound there (weights stream
// from MALL / HBM at small batch)
using TinyTile = TileCfg<2, 4, 4>;
// the flow kernel's task tile: 128 gate x 128 batch rows, 4-deep ring (one workgroup per CU)
using FlowTile = TinyTile;
static_assert(BigTile::BN == ENC_BATCH_TILE && SmallTile::BN == ENC_ROW_TILE, "engine batch tiles");

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(1))) void glb_void;

// byte offset of (row r, byte b < ROWB) in a swizzled [rows][ROWB] image: 16-byte chunk c of
// row r sits at chunk slot c ^ (r mod chunks-per-row)
template <int ROWB>
__device__ __forceinline__ int cimg_off(int r, int b) {
  return r * ROWB + ((((b >> 4) ^ r) & (ROWB / 16 - 1)) << 4) + (b & 15);
}

// Top of main-loop iteration s: wait until this wave's pieces of stage s have landed -- at most
// min(NBUF - 2, stages left after s) later stages (PPS pieces each) may still be in flight --
// drain its LDS reads, and meet the other waves at the barrier.
template <int PPS, int NBUF>
__device__ __forceinline__ void wait_stage(int later) {
  if (NBUF <= 2 || later <= 0) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else if (NBUF == 3 || later == 1) {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(PPS) : "memory");
  } else {
    static_assert(NBUF <= 4, "ring depth");
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(2 * PPS) : "memory");
  }
  // the same lgkmcnt(0) as a real instruction (0xC07F: lgkmcnt 0, the other counters untouched): the
  // compiler does not read inline asm, and without it assumes scalar loads from before the loop may
  // still be outstanding -- its fragment waits then all become lgkmcnt(0) instead of counted ones
  __builtin_amdgcn_s_waitcnt(0xC07F);
}

// 16-byte copy-out store: plain, or write-through (WT: `sc1`, the line leaves the XCD's L2 at
// once) for outputs another workgroup of the same launch reads -- the flow kernel's hand-offs,
// which then need no release fence before the completion count (guide R1 publish)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
template <bool WT>
__device__ __forceinline__ void st16(void* base, size_t off, uint4 v) {
  if (WT) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7ffffff0, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, r, (int)off, 0, 16);  // aux 16 = sc1
  } else {
    *(uint4*)((char*)base + off) = v;
  }
}
// a wave-uniform pointer the compiler can prove uniform (a buffer resource built from it then needs no
// waterfall loop around every access)
__device__ __forceinline__ void* uniform_ptr(const void* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
struct NoWait {
  __device__ void operator()() const {}
};

// One (gate tile mt, batch tile nt) of a layer-step.  WT: write-through hand-off stores (flow
// kernel); hwait() runs (uniformly, every wave) right before the first stage of the recurrent
// half [h_{t-1}] is issued -- the flow kernel's wait for the previous step of the layer.
template <int WMT, int WNT, int NBUF, bool WT = false, class HWait = NoWait>
__device__ __forceinline__ void lstm_i8_step(const EncStepArgs& a, int mt, int nt, int8_t* smem,
                                             unsigned long long st_t0, HWait&& hwait = HWait{},
                                             unsigned long long st_t1 = 0ull, unsigned long long st_tag = 0ull) {
  using C = TileCfg<WMT, WNT, NBUF>;
  constexpr int BM = C::BM, BN = C::BN, STAGE = C::STAGE;
  (void)st_t0;
  (void)st_t1;
  (void)st_tag;
#ifdef RNNT_DEV_STAMPS
  unsigned est_k;
  {
    unsigned v = 0;
    if (threadIdx.x == 0) v = atomicAdd(&g_est_n, 1u);
    est_k = __builtin_amdgcn_readfirstlane(v);  // wave 0 (the only writer) holds thread 0's ticket
  }
  EST_PUT(2, st_t0);
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // SGPR
  const int wm = wave & 3, wn = wave >> 2;
  const int m0 = mt * BM;  // packed gate row base
  const int n0 = nt * BN;  // batch row base
  const int K = a.I + H;
  const int nS = K / 128;  // stages
  const int q = lane >> 4, col = lane & 15;
  // this lane's WMT consecutive units: packed rows of the wave start at R = m0 + 16 WMT wm, in
  // 64-row block R >> 6 at MFMA tile (R & 63) >> 4 (enc_packed_row)
  const int R = m0 + wm * 16 * WMT;
  const int u0 = 16 * (R >> 6) + 4 * q + ((R & 63) >> 4);
  const int nb = n0 + wn * 16 * WNT + col;  // batch row of accumulator column j = 0 (row j: nb + 16 j)
  lds_char* lds = (lds_char*)(lds_void*)smem;

  // ---- staging.  A stage holds K bytes k0..k0+127 (two MFMA k steps) of all BM A and BN B
  // rows; each 1 KiB LDS-DMA piece moves 8 whole 128-byte rows (8 full cache lines).  Image:
  // 16-byte column c of row r at slot c ^ ((r >> 1) & 7) (two 128-B rows per 256-B bank row), so
  // the ds_read_b128 fragment reads are conflict-free; the swizzle is applied on the DMA source
  // address.  Wave w moves A rows 8 PA w .. and B rows 8 PB w .. (PA / PB pieces each); lane l of
  // piece j lands at row 8 PA w + 8j + (l >> 3), slot l & 7.  SGPR tile bases + 32-bit lane offsets.
  const int r8 = lane >> 3, sl = lane & 7;
  // slot of row r = 8 P w + 8 j + r8 is (r >> 1) & 7 = (4 P w + 4 j + (r8 >> 1)) & 7: even / odd pieces
  const int swA = (4 * C::PA * wave) & 7, swB = (4 * C::PB * wave) & 7;  // 0 unless P is odd
  const int gA0 = (sl ^ ((swA + (r8 >> 1)) & 7)) * 16, gA1 = (sl ^ ((swA + 4 + (r8 >> 1)) & 7)) * 16;
  const int gB0 = (sl ^ ((swB + (r8 >> 1)) & 7)) * 16, gB1 = (sl ^ ((swB + 4 + (r8 >> 1)) & 7)) * 16;
  const uint32_t rlA = (uint32_t)(8 * C::PA * wave + r8), rlB = (uint32_t)(8 * C::PB * wave + r8);
  const uint32_t oA0 = rlA * K + gA0, oA1 = rlA * K + gA1;
  const uint32_t oX0 = rlB * a.I + gB0, oX1 = rlB * a.I + gB1;
  const uint32_t oH0 = rlB * H + gB0, oH1 = rlB * H + gB1;
  const int8_t* wbase = a.W + (size_t)m0 * K;
  const int8_t* xbase = a.x + (size_t)n0 * a.I;
  const int8_t* hbase = a.h_in + (size_t)n0 * H - a.I;  // k >= I indexes h at k - I
  // LDS-DMA through buffer resources (buffer_load_dwordx4 ... lds): wave-uniform bases in SGPRs,
  // loop-invariant 32-bit lane offsets, the stage's k in soffset.  Unlike global_load_lds (a FLAT
  // instruction the compiler must assume may also touch LDS through the LGKM counter), these are
  // plain vector-memory loads to it, so the fragment waits below stay counted (lgkmcnt(N)).
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)wbase, (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc((void*)xbase, (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsH = __builtin_amdgcn_make_buffer_rsrc((void*)hbase, (short)0, 0x7ffffff0, 0x00020000);
  auto issueA = [&](int s) __attribute__((always_inline)) {
    const int k = s * 128;
    lds_char* st = lds + (s % NBUF) * STAGE + wave * (C::PA * 1024);
#pragma unroll
    for (int j = 0; j < C::PA; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)(st + j * 1024), 16, (j & 1) ? oA1 : oA0,
                                               k + 8 * j * K, 0, 0);
  };
  auto issueB = [&](int s) __attribute__((always_inline)) {
    const int k = s * 128;
    lds_char* st = lds + (s % NBUF) * STAGE + BM * 128 + wave * (C::PB * 1024);
    if (k < a.I) {
#pragma unroll
      for (int j = 0; j < C::PB; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsX, (lds_void*)(st + j * 1024), 16, (j & 1) ? oX1 : oX0,
                                                 k + 8 * j * a.I, 0, 0);
    } else {
      if (k == a.I) {
        hwait();
        if (WT) EST_PUT(7, __builtin_amdgcn_s_memrealtime());  // flow: its recurrent state was ready
      }
#pragma unroll
      for (int j = 0; j < C::PB; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsH, (lds_void*)(st + j * 1024), 16, (j & 1) ? oH1 : oH0,
                                                 k + 8 * j * H, 0, 0);
    }
  };
  // the tile's fp16 cell state (BN rows x CROW bytes), DMA'd into the buffer the last stage does
  // not occupy once its reads are retired; piece p, lane l: row p (64 / CPR) + l / CPR, chunk
  // (l % CPR) ^ (row % CPR) at slot l % CPR (cimg_off: 2-way instead of 8-way epilogue conflicts)
  const int cbuf = (nS % NBUF) * STAGE;
  const __amdgpu_buffer_rsrc_t rsC =
      __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(a.c + (size_t)n0 * H + (m0 >> 2)), (short)0, 0x7ffffff0, 0x00020000);
  auto issue_c = [&]() __attribute__((always_inline)) {
    constexpr int RPP = 64 / C::CPR, NPC = C::CPIECES >= NWAVE ? C::CPIECES / NWAVE : 1;
    const int cr = lane / C::CPR, cc = lane % C::CPR;
    const uint32_t vo = (uint32_t)(cr * H + (cc ^ (cr & (C::CPR - 1))) * 8) * 2;  // bytes
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc) {
      const int p = wave * NPC + pc;
      if (C::CPIECES < NWAVE && p >= C::CPIECES) break;  // wave-uniform
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsC, (lds_void*)(lds + cbuf + p * 1024), 16, vo, RPP * p * H * 2, 0, 0);
    }
  };

  v4i acc[WMT][WNT];
#pragma unroll
  for (int i = 0; i < WMT; ++i)
#pragma unroll
    for (int j = 0; j < WNT; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  // ---- main loop.  Stages s+1 .. s+NBUF-1 are DMA'd into the other ring buffers while stage s
  // is consumed: every wave issues its A pieces of stage s+NBUF-1 right after the stage barrier
  // and its B pieces after the first k step's MFMAs (two half bursts per stage on the load path;
  // measured best of the issue points tried), MFMA clusters at s_setprio 1.
  // Fragment reads: A rows 16 WMT wm + 16i + col, B rows 16 WNT wn + 16j + col, 16-byte column
  // 4kk + q.
  const int sw = col >> 1;  // (row >> 1) & 7 for rows 16i + col
  const int fa0 = (wm * 16 * WMT + col) * 128, fb0 = BM * 128 + (wn * 16 * WNT + col) * 128;
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s)
    if (s < nS) {
      issueA(s);
      issueB(s);
    }
#ifdef RNNT_DEV_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stamps only: stage 0 landed (this wave)
  EST_PUT(3, __builtin_amdgcn_s_memrealtime());
  EST_PUT(6, WT ? st_t1 : __builtin_amdgcn_s_memtime());  // flow: its input frame was ready
#endif
#ifdef RNNT_DEV_STAMPS
  unsigned long long est_wait = 0, est_work = 0;
#endif
  for (int s = 0; s < nS; ++s) {
    // this wave's DMA of stage s has landed (only later stages' pieces may be outstanding) and
    // its LDS reads are drained; after the barrier every wave's has, and every wave is done
    // reading the buffer stage s+NBUF-1 refills
#ifdef RNNT_DEV_STAMPS
    unsigned long long w0, w1;  // no LDS read is outstanding here (the stage's last MFMAs waited for all)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(w0)::"memory");
    __builtin_amdgcn_sched_barrier(0);
#endif
    wait_stage<C::PA + C::PB, NBUF>(nS - 1 - s);
#ifdef RNNT_DEV_STAMPS
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(w1)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    est_wait += w1 - w0;
#endif
    const int8_t* st = smem + (s % NBUF) * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int cs = ((kk * 4 + q) ^ sw) << 4;
      // fragment reads in the order the MFMAs consume them (A0, all B, then A1..): LDS returns in
      // order, so the first MFMA waits for two reads instead of all of them
      v4i fra[WMT], frb[WNT];
      fra[0] = *(const v4i*)(st + fa0 + cs);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < WNT; ++j) frb[j] = *(const v4i*)(st + fb0 + cs + j * 2048);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 1; i < WMT; ++i) fra[i] = *(const v4i*)(st + fa0 + cs + i * 2048);
      __builtin_amdgcn_sched_barrier(0);
      // the next stage's DMA is issued while these reads are in flight: A after stage s's first
      // reads, B after its second k step's (the B half lands half a stage later, as measured best)
      if (kk == 0) {
        if (s + NBUF - 1 < nS) issueA(s + NBUF - 1);
        else if (s == nS - 1) issue_c();
      } else if (s + NBUF - 1 < nS) {
        issueB(s + NBUF - 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < WMT; ++i)
#pragma unroll
        for (int j = 0; j < WNT; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fra[i], frb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    }
#ifdef RNNT_DEV_STAMPS
    {
      unsigned long long w2;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(w2)::"memory");
      __builtin_amdgcn_sched_barrier(0);
      est_work += w2 - w1;
    }
#endif
  }
#ifdef RNNT_DEV_STAMPS
  EST_PUT(8, est_wait);
  EST_PUT(9, est_work);
  EST_PUT(10, (unsigned long long)nS);
#endif
  // the cell-state DMA has landed for every wave, all fragment reads are done
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#ifdef RNNT_DEV_STAMPS
  EST_PUT(4, __builtin_amdgcn_s_memrealtime());
  if (!WT) EST_PUT(7, __builtin_amdgcn_s_memtime());
#endif

  // ---- fused LSTM cell epilogue (quant_lstm.py:162-183 semantics; oracle_enc_cell)
  const float As = a.rb * 64.0f, Ag = a.rb * 128.0f, ins = a.in_s, outs = a.out_s;
  const float2* tab = (const float2*)(smem + C::TAB_OFF);
  float4 bq[WMT];
#pragma unroll
  for (int i = 0; i < WMT; ++i) bq[i] = *(const float4*)(a.bq + R + i * 16 + q * 4);
  // results go to LDS first and leave as whole row segments (16 B per lane, full cache lines per
  // wave instruction) instead of scattered per-lane stores: c_new in place over the c_in image
  // (each lane rewrites exactly what it read), h and y / the bf16 output in the other stage
  // buffer (free after the main loop)
  const int ul = u0 - (m0 >> 2);  // this lane's first unit within the tile's BM / 4
  lds_char* hs = lds + cbuf + BN * C::CROW;
  lds_char* ys = lds + ((nS - 1) % NBUF) * STAGE;
  constexpr int HP = C::HP;
#pragma unroll
  for (int j = 0; j < WNT; ++j) {
    const int n = nb + 16 * j, r = n - n0;
    float cin[WMT];
    if (WMT == 4) {
      const uint2 cv = *(const uint2*)(smem + cbuf + cimg_off<C::CROW>(r, ul * 2));
      cin[0] = h2f((uint16_t)(cv.x & 0xffff)); cin[1 % WMT] = h2f((uint16_t)(cv.x >> 16));
      cin[2 % WMT] = h2f((uint16_t)(cv.y & 0xffff)); cin[3 % WMT] = h2f((uint16_t)(cv.y >> 16));
    } else if (WMT == 1) {
      cin[0] = h2f(*(const uint16_t*)(smem + cbuf + cimg_off<C::CROW>(r, ul * 2)));
    } else {
      const uint32_t cv = *(const uint32_t*)(smem + cbuf + cimg_off<C::CROW>(r, ul * 2));
      cin[0] = h2f((uint16_t)(cv & 0xffff)); cin[1 % WMT] = h2f((uint16_t)(cv >> 16));
    }
    uint32_t cw[2] = {0u, 0u}, hb[4] = {0u, 0u, 0u, 0u}, yb[4] = {0u, 0u, 0u, 0u};
    float hv[WMT];
#pragma unroll
    for (int i = 0; i < WMT; ++i) {
      float cn, hh;
      enc_cell(tab, acc[i][j], bq[i], As, Ag, cin[i], cn, hh);
      cw[i >> 1] |= (uint32_t)f2h(cn) << (16 * (i & 1));
      hv[i] = hh;
      hb[i] = q8_biased(hh * ins);
      yb[i] = q8_biased(hh * outs);
    }
    const uint32_t hq = pack_q8(hb[0], hb[1], hb[2], hb[3]), yq = pack_q8(yb[0], yb[1], yb[2], yb[3]);
    if (WMT == 4) {
      *(uint2*)(smem + cbuf + cimg_off<C::CROW>(r, ul * 2)) = uint2{cw[0], cw[1]};
      *(uint32_t*)(hs + r * HP + ul) = hq;
    } else if (WMT == 1) {
      *(uint16_t*)(smem + cbuf + cimg_off<C::CROW>(r, ul * 2)) = (uint16_t)cw[0];
      *(uint8_t*)(hs + r * HP + ul) = (uint8_t)hq;
    } else {
      *(uint32_t*)(smem + cbuf + cimg_off<C::CROW>(r, ul * 2)) = cw[0];
      *(uint16_t*)(hs + r * HP + ul) = (uint16_t)hq;
    }
    if (a.mode == ENC_OUT_FINAL) {
      if (a.y32) {
        if (WMT == 4) *(float4*)(a.y32 + (size_t)n * H + u0) = float4{hv[0], hv[1 % WMT], hv[2 % WMT], hv[3 % WMT]};
        else if (WMT == 1) a.y32[(size_t)n * H + u0] = hv[0];
        else *(float2*)(a.y32 + (size_t)n * H + u0) = float2{hv[0], hv[1 % WMT]};
      }
      const uint32_t f01 = (uint32_t)f2bf_ftz(hv[0]) | ((uint32_t)f2bf_ftz(hv[1 % WMT]) << 16);
      if (WMT == 4)
        *(uint2*)(ys + cimg_off<C::CROW>(r, ul * 2)) =
            uint2{f01, (uint32_t)f2bf_ftz(hv[2 % WMT]) | ((uint32_t)f2bf_ftz(hv[3 % WMT]) << 16)};
      else if (WMT == 1)
        *(uint16_t*)(ys + cimg_off<C::CROW>(r, ul * 2)) = (uint16_t)f01;
      else
        *(uint32_t*)(ys + cimg_off<C::CROW>(r, ul * 2)) = f01;
    } else if (WMT == 4) {
      *(uint32_t*)(ys + r * HP + ul) = yq;
    } else if (WMT == 1) {
      *(uint8_t*)(ys + r * HP + ul) = (uint8_t)yq;
    } else {
      *(uint16_t*)(ys + r * HP + ul) = (uint16_t)yq;
    }
  }
  __syncthreads();  // the staged images are complete
  // copy-out: thread t moves 16-byte chunks; a wave instruction writes whole row segments
  const int um = m0 >> 2;
#pragma unroll
  for (int it = 0; it < (BN * C::CPR + NWAVE * 64 - 1) / (NWAVE * 64); ++it) {  // c (and bf16 f): BN rows x CROW bytes
    const int idx = it * NWAVE * 64 + tid, r = idx / C::CPR, ch = idx % C::CPR;
    if ((BN * C::CPR) % (NWAVE * 64) != 0 && idx >= BN * C::CPR) break;
    st16<WT>(a.c, ((size_t)(n0 + r) * H + um + ch * 8) * 2, *(const uint4*)(smem + cbuf + cimg_off<C::CROW>(r, ch * 16)));
    if (a.mode == ENC_OUT_FINAL)  // read after the launch only: plain
      *(uint4*)(a.fbf + (size_t)(n0 + r) * H + um + ch * 8) = *(const uint4*)(ys + cimg_off<C::CROW>(r, ch * 16));
  }
#pragma unroll
  for (int it = 0; it < (BN * C::HC + NWAVE * 64 - 1) / (NWAVE * 64); ++it) {  // h, y: BN rows x BM / 4 bytes
    const int idx = it * NWAVE * 64 + tid, r = idx / C::HC, ch = idx % C::HC, n = n0 + r;
    if ((BN * C::HC) % (NWAVE * 64) != 0 && idx >= BN * C::HC) break;
    st16<WT>(a.h_out, (size_t)n * H + um + ch * 16, *(const uint4*)(hs + r * HP + ch * 16));
    if (a.mode == ENC_OUT_I8) {
      st16<WT>(a.y8, (size_t)n * H + um + ch * 16, *(const uint4*)(ys + r * HP + ch * 16));
    } else if (a.mode == ENC_OUT_STACKED) {
      // StackTime (modeling_rnnt.py:314-324): frame t -> stacked frame t/2, half t%2;
      // frames t >= x_lens[n] are zeroed; the odd-T pad frame is zero too.
      const size_t dst = (size_t)n * (2 * H) + um + ch * 16;
      uint4 v = *(const uint4*)(ys + r * HP + ch * 16);
      if (a.t >= a.lens[n]) v = uint4{0u, 0u, 0u, 0u};  // a value select: no pointer select into a stack temporary
      st16<WT>(a.y8, dst + a.half * H, v);
      if (a.zero_next) st16<WT>(a.y8, dst + H, uint4{0u, 0u, 0u, 0u});
    }
  }
#ifdef RNNT_DEV_STAMPS
  EST_PUT(5, __builtin_amdgcn_s_memrealtime());
  EST_PUT(0, (unsigned long long)K | ((unsigned long long)mt << 16) | ((unsigned long long)nt << 24) |
                 ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 32));  // HW_REG_HW_ID
  EST_PUT(1, WT ? st_tag : (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20));  // flow: step; XCC_ID
#endif
}

// One launch = one wavefront tick: up to 5 independent layer-steps (jobs, longest K first).
// XCD-aware tile order: workgroup id -> XCD id % 8 (round-robin dispatch).  XCD x takes gate
// tiles GPX (x&3) .. GPX (x&3) + GPX - 1 and the (x>>2)-th half of each job's active batch tiles,
// so the workgroups resident on an XCD share a quarter of the weight tiles and half the
// activation tiles through its L2 (weights fetched from HBM/MALL 2x, activations 4x per tick,
// instead of 1x / 8x).  Batch tiles of a job: its active 128-row tiles in the tile's rows.
template <class C>
__host__ __device__ __forceinline__ int job_tiles(const EncTickArgs& args, int j) {
  if (args.bmask[j]) return __builtin_popcountll(enc_tile_mask(args.bmask[j], C::BN));
  return C::BN == 256 ? (args.nbt[j] + 1) >> 1 : args.nbt[j];
}
// batch tile of compact index i (0 .. job_tiles - 1): the i-th active tile
template <class C>
__device__ __forceinline__ int job_tile(const EncTickArgs& args, int j, int i) {
  uint64_t m = args.bmask[j];
  if (!m) return i;
  m = enc_tile_mask(m, C::BN);
  for (; i > 0; --i) m &= m - 1;  // drop the i lowest set bits
  return __builtin_ctzll(m);
}
// job tile k (0..) of XCD xcd -> (mt, nt); -1 past the XCD's last tile.  A job with ONE batch tile
// (small batches: config 3, short Server rounds, the tail of a sorted batch) spreads its gate tiles
// over all 8 XCDs instead (the 4 x 2 split would leave XCDs 4-7 without work for it).
template <class C>
__device__ __forceinline__ int xcd_pick(const EncTickArgs& args, int xcd, int k, int& mt, int& nt) {
  const int gsel = xcd & 3, psel = xcd >> 2;
  for (int j = 0; j < args.njobs; ++j) {
    const int nbt = job_tiles<C>(args, j);
    if (nbt == 1) {
      constexpr int G8 = C::NGT / 8;
      if (k < G8) {
        mt = xcd * G8 + k;
        nt = job_tile<C>(args, j, 0);
        return j;
      }
      k -= G8;
      continue;
    }
    const int b0 = psel ? (nbt + 1) >> 1 : 0;
    const int b1 = psel ? nbt : (nbt + 1) >> 1;
    const int cnt = C::GPX * (b1 - b0);
    if (k < cnt) {
      mt = gsel * C::GPX + k % C::GPX;
      nt = job_tile<C>(args, j, b0 + k / C::GPX);
      return j;
    }
    k -= cnt;
  }
  return -1;
}
template <int WMT, int WNT, int NBUF>
__global__ void __launch_bounds__(NWAVE * 64) lstm_i8_tick_kernel(EncTickArgs args) {
  using C = TileCfg<WMT, WNT, NBUF>;
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  unsigned long long st_t0 = 0ull;
  EST_MARK(st_t0);
  // sigma table into LDS (read after the main loop's first stage barrier)
#pragma unroll
  for (int i = 0; i < ENC_TAB_N / (2 * NWAVE * 64); ++i)
    ((float4*)(smem + C::TAB_OFF))[i * NWAVE * 64 + threadIdx.x] = ((const float4*)g_act_tab)[i * NWAVE * 64 + threadIdx.x];
  int mt = 0, nt = 0;
  const int jsel = xcd_pick<C>(args, blockIdx.x & 7, blockIdx.x >> 3, mt, nt);
  if (jsel < 0) return;
  // wave-uniform runtime index into the kernarg segment: the job's fields stay scalar loads
  lstm_i8_step<WMT, WNT, NBUF>(args.job[__builtin_amdgcn_readfirstlane(jsel)], __builtin_amdgcn_readfirstlane(mt),
                         __builtin_amdgcn_readfirstlane(nt), smem, st_t0);
}

// ---------------------------------------------------------------- persistent dataflow encoder
// Small batches (config 3: N = 128, T <= 500) are latency-bound on the tick path: ~505 dependent
// launches whose every workgroup re-stages its operands from a cold start.  Here one launch holds
// one workgroup per CU; each takes tasks (layer-step, 128-row gate tile, 128-row batch tile) from a
// device queue in tick order and runs the tick kernel's step body on them.  A task waits for the
// completion counter of the step that wrote its input frame before it starts, and for the counter
// of its layer's previous step only right before the first recurrent [h_{t-1}] stage is issued, so
// the input half of the K loop runs while the previous step finishes.
// Hand-offs (MI355X guide, Guideline 16): outputs read inside the launch (h, c, the int8 frame)
// are stored write-through (`sc1`); every wave drains its stores, the workgroup meets at a
// barrier and lane 0 adds 1 to the step's counter (relaxed, agent scope).  A waiting workgroup
// polls one counter from one lane (relaxed, `s_sleep` between polls), then ONE agent-scope
// acquire, its drain and a barrier, before any load of the handed-off bytes.
// Progress needs no dispatch-order assumption: a task depends only on steps of earlier ticks,
// whose tasks were dequeued earlier by workgroups that are running.  Every wait is bounded: past
// the timeout it raises the launch's abort word and every workgroup drains (the host reports it).
// Control flow around the waits is wave-uniform: wave 0 polls as a whole (every lane loads the
// same word; the value is made uniform with readfirstlane), so no lane-divergent branch encloses a
// barrier or the task loop's back edge (a lane-0-only branch there let the compiler's CFG
// structurizer run lanes 1-63 of wave 0 into the next iteration's barrier ahead of lane 0).
__device__ __forceinline__ unsigned flow_load(const uint32_t* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// wave 0: poll until step dep has `need` completed tasks (or the launch aborts / this wait times out)
__device__ __forceinline__ void flow_spin(const EncFlowArgs& f, int dep, unsigned need) {
  uint32_t* abort_w = f.ctr + f.n_steps + 1;
  const unsigned long long t_end = __builtin_amdgcn_s_memrealtime() + f.timeout;
  while (flow_load(f.ctr + dep) < need) {
    if (flow_load(abort_w)) return;
    if (__builtin_amdgcn_s_memrealtime() > t_end) {
      __hip_atomic_store(abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}
__device__ __forceinline__ void flow_acquire() {  // wave 0; the other waves meet it at a barrier
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int WMT, int WNT, int NBUF>
__global__ void __launch_bounds__(NWAVE * 64) lstm_i8_flow_kernel(EncFlowArgs f) {
  using C = TileCfg<WMT, WNT, NBUF>;
  static_assert(C::NGT == ENC_FLOW_NGT || C::NGT == ENC_FLOW_BIG_NGT, "flow task blocks");
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  // [0] task index, [1] recurrent input ready (an LDS pointer: ds ops, not flat)
  volatile __attribute__((address_space(3))) int* slot =
      (volatile __attribute__((address_space(3))) int*)((lds_char*)(lds_void*)smem + C::SMEM);
  const bool w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;  // wave-uniform
  const bool l0 = (threadIdx.x & 63) == 0;
#pragma unroll
  for (int i = 0; i < ENC_TAB_N / (2 * NWAVE * 64); ++i)  // sigma table: once per workgroup
    ((float4*)(smem + C::TAB_OFF))[i * NWAVE * 64 + threadIdx.x] = ((const float4*)g_act_tab)[i * NWAVE * 64 + threadIdx.x];
  uint32_t* head = f.ctr + f.n_steps;
  // the next task index is taken from the queue while the current task runs (wave 0, lane 0)
  unsigned nxt = 0;
  if (w0 && l0) nxt = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    if (w0) slot[0] = flow_load(head + 1) ? f.n_tasks : (int)__builtin_amdgcn_readfirstlane(nxt);
    __syncthreads();
    const int ti = __builtin_amdgcn_readfirstlane(slot[0]);
    if (ti >= f.n_tasks) return;
    unsigned long long t_deq = 0ull, t_x = 0ull;
    EST_MARK(t_deq);
    const uint32_t blk = f.blocks[ti / C::NGT];
    const int si = __builtin_amdgcn_readfirstlane((int)(blk & 0xffffu));
    const int nt = __builtin_amdgcn_readfirstlane((int)(blk >> 16)), mt = ti % C::NGT;
    const EncFlowStep S = f.steps[si];
    // the input frame: wait; the recurrent state: note whether it is ready already (then one
    // acquire covers both and the mid-loop wait is skipped)
    if (w0) {
      if (S.dep_x >= 0) flow_spin(f, S.dep_x, S.need_x);
      const bool hr = S.dep_h < 0 || flow_load(f.ctr + S.dep_h) >= S.need_h;
      if (S.dep_x >= 0 || (S.dep_h >= 0 && hr)) flow_acquire();
      slot[1] = hr;
    }
    __syncthreads();
    const bool h_ready = __builtin_amdgcn_readfirstlane(slot[1]) != 0;
    EST_MARK(t_x);
    if (w0 && l0) nxt = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lstm_i8_step<WMT, WNT, NBUF, true>(S.a, mt, nt, smem, t_deq, [&]() {
      if (h_ready) return;
      if (w0) {
        flow_spin(f, S.dep_h, S.need_h);
        flow_acquire();
      }
      __builtin_amdgcn_s_barrier();  // no LDS / memory wait: the other waves' stage DMA stays in flight
    }, t_x, (unsigned long long)si);
    // publish: every wave's write-through stores have landed, then one count
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (w0 && l0) __hip_atomic_fetch_add(f.ctr + si, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------- host launchers
int launch_lstm_i8_flow(const EncFlowArgs& f, int grid, hipStream_t st, bool big) {
  if (big) {
    using C = BigTile;
    static_assert(C::NGT == ENC_FLOW_BIG_NGT && C::BN == ENC_FLOW_BIG_ROWS, "big flow tile");
    static std::atomic<uint64_t> attr{0};
    const void* fn = (const void*)lstm_i8_flow_kernel<C::BM / 64, C::BN / 32, C::NBUF>;
    if (set_smem_attr_once(fn, C::SMEM + 16, attr)) return -1;
    hipLaunchKernelGGL((lstm_i8_flow_kernel<C::BM / 64, C::BN / 32, C::NBUF>), dim3(grid), dim3(NWAVE * 64),
                       C::SMEM + 16, st, f);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  using C = FlowTile;
  static_assert(C::NGT == ENC_FLOW_NGT, "flow tile");
  static std::atomic<uint64_t> attr{0};
  const void* fn = (const void*)lstm_i8_flow_kernel<C::BM / 64, C::BN / 32, C::NBUF>;
  if (set_smem_attr_once(fn, C::SMEM + 16, attr)) return -1;
  hipLaunchKernelGGL((lstm_i8_flow_kernel<C::BM / 64, C::BN / 32, C::NBUF>), dim3(grid), dim3(NWAVE * 64), C::SMEM + 16,
                     st, f);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

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

// Per tick: the 256 x 256 tile unless its last round of workgroups would leave many CUs idle
// and the 128 x 128 tile (two per CU, 8x the tiles) finishes sooner.  Cost model in units of a
// large-tile round (one 256 x 256 tile per CU), measured at N=8192 / 2048 / 256 (DESIGN.md
// section 4): a full round of small tiles (two per CU) costs ENC_SMALL_ROUND of it, and a
// small-tile launch takes at least ENC_SMALL_FLOOR (its K loop's latency); the small tile must
// win by ENC_SMALL_MARGIN (its co-resident workgroups also leave room for the overlapped
// decode's, which slows the encoder).  `forced` (the engine's rnnt_engine_set_tile) pins a shape.
constexpr int ENC_CUS = 256;
constexpr float ENC_SMALL_ROUND = 0.59f, ENC_SMALL_FLOOR = 0.5f, ENC_SMALL_MARGIN = 0.9f;
template <class C>
static int tick_grid(const EncTickArgs& a) {  // workgroups: 8 XCDs x the batch-half-0 XCDs' (larger) share
  int per_xcd = 0;
  for (int j = 0; j < a.njobs; ++j) {
    const int nbt = job_tiles<C>(a, j);
    per_xcd += nbt == 1 ? C::NGT / 8 : C::GPX * ((nbt + 1) / 2);  // as xcd_pick
  }
  return 8 * per_xcd;
}
template <class C>
static int launch_tick(const EncTickArgs& a, int grid, hipStream_t st) {
  static std::atomic<uint64_t> attr{0};
  const void* fn = (const void*)lstm_i8_tick_kernel<C::BM / 64, C::BN / 32, C::NBUF>;
  if (set_smem_attr_once(fn, C::SMEM, attr)) return -1;
  hipLaunchKernelGGL((lstm_i8_tick_kernel<C::BM / 64, C::BN / 32, C::NBUF>), dim3(grid), dim3(NWAVE * 64), C::SMEM, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_lstm_i8_tick(const EncTickArgs& a, hipStream_t st, int forced) {
  // shapes the kernel's staging assumes (checked on the host: a mismatch would read out of bounds)
  for (int j = 0; j < a.njobs; ++j)
    if (a.job[j].I % 128 != 0 || a.nbt[j] < 0 || (a.bmask[j] && __builtin_popcountll(a.bmask[j]) != a.nbt[j])) return -1;
  const int gb = tick_grid<BigTile>(a), gs = tick_grid<SmallTile>(a), gm = tick_grid<MiniTile>(a);
  if (gb <= 0) return 0;
  int choice = forced == ENC_TILE_FLOW || forced == ENC_TILE_TICKS ? ENC_TILE_AUTO : forced;  // (flow: engine-level)
  if (choice == ENC_TILE_AUTO) {
    const float rb = (float)((gb + ENC_CUS - 1) / ENC_CUS);
    const float rs = fmaxf((float)gs / (2 * ENC_CUS) * ENC_SMALL_ROUND, ENC_SMALL_FLOOR);
    choice = rs < ENC_SMALL_MARGIN * rb ? ENC_TILE_SMALL : ENC_TILE_BIG;
    if (choice == ENC_TILE_SMALL && gs <= ENC_CUS) {  // at most one small workgroup per CU: a deep ring
      bool one_tile = true;
      for (int j = 0; j < a.njobs; ++j) one_tile = one_tile && a.nbt[j] <= 1;
      choice = one_tile && gm <= ENC_CUS ? ENC_TILE_MINI : ENC_TILE_TINY;  // one per CU with half the gate rows: mini
    }
  }
  if (choice == ENC_TILE_BIG) return launch_tick<BigTile>(a, gb, st);
  if (choice == ENC_TILE_MINI) return launch_tick<MiniTile>(a, gm, st);
  return choice == ENC_TILE_TINY ? launch_tick<TinyTile>(a, gs, st) : launch_tick<SmallTile>(a, gs, st);
}

}  // namespace rnnt

#ifdef RNNT_DEV_STAMPS
// development: copy out (and reset) the tick kernel's per-tile stamp records (8 x u64 each)
extern "C" int rnnt_dev_read_enc_stamps(unsigned long long* out, int max_records) {
  unsigned int n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(rnnt::g_est_n), sizeof(n)) != hipSuccess) return -1;
  if (n > (1u << 22) / EST_W) n = (1u << 22) / EST_W;
  if ((int)n > max_records) n = max_records;
  if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(rnnt::g_est), (size_t)n * EST_W * 8) != hipSuccess) return -1;
  const unsigned int z = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(rnnt::g_est_n), &z, sizeof(z)) != hipSuccess) return -1;
  return (int)n;
}
#endif
