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
// Workgroup tile: 256 packed gate rows (64 units) x 256 batch rows, K swept in 128-byte stages.
// 8 waves as 4 (gate) x 2 (batch); each wave owns 64 gate rows x 128 batch rows = 4 x 8 MFMA
// 16x16x64 tiles (128 accumulator VGPRs).  The 256x256 tile is the largest whose int32
// accumulators fit the register file at 2 waves/SIMD; it balances the per-CU L2->LDS load path
// against the MFMA.
constexpr int BM = 256;
constexpr int BN = ENC_BATCH_TILE;
constexpr int NWAVE = 8;
constexpr int STAGE = 65536;                  // one stage: 128 K bytes of 256 A + 256 B rows
constexpr int TAB_OFF = 2 * STAGE;            // LDS: sigma table after the two stage buffers
constexpr int SMEM_BYTES = TAB_OFF + ENC_TAB_N * 8;
static_assert(BN == 256 && SMEM_BYTES <= 160 * 1024, "tile / LDS budget");
static_assert(BN * 128 <= STAGE && BN * 80 <= STAGE, "the epilogue images fit one stage buffer each");

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(1))) void glb_void;

// byte offset of (row r, byte b < 128) in a swizzled [rows][128 B] image: 16-byte chunk c of
// row r sits at chunk slot c ^ (r & 7)
__device__ __forceinline__ int cimg_off(int r, int b) { return r * 128 + ((((b >> 4) ^ r) & 7) << 4) + (b & 15); }

__device__ __forceinline__ void lstm_i8_step(const EncStepArgs& a, int mt, int nt, int8_t* smem,
                                             unsigned long long st_t0) {
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
  const int nS = K / 128;  // stages
  const int q = lane >> 4, col = lane & 15;
  const int u0 = (m0 >> 2) + wm * 16 + q * 4;  // this lane's 4 consecutive units
  const int nb = n0 + wn * 128 + col;          // batch row of accumulator column j = 0 (row j: nb + 16 j)
  lds_char* lds = (lds_char*)(lds_void*)smem;

  // ---- staging.  A stage holds K bytes k0..k0+127 (two MFMA k steps) of all 256 A and 256 B
  // rows; each 1 KiB LDS-DMA piece moves 8 whole 128-byte rows (8 full cache lines).  Image:
  // 16-byte column c of row r at slot c ^ ((r >> 1) & 7) (two 128-B rows per 256-B bank row), so
  // the ds_read_b128 fragment reads are conflict-free; the swizzle is applied on the DMA source
  // address.  Wave w moves A rows 32w..32w+31 and B rows 32w..32w+31 (4 pieces each); lane l of
  // piece j lands at row 32w + 8j + (l >> 3), slot l & 7.  SGPR tile bases + 32-bit lane offsets.
  const int r8 = lane >> 3, sl = lane & 7;
  const int gc0 = (sl ^ ((r8 >> 1) & 7)) * 16;        // even pieces (rows 8j + r8, j even)
  const int gc1 = (sl ^ (((8 + r8) >> 1) & 7)) * 16;  // odd pieces
  const uint32_t rl = (uint32_t)(32 * wave + r8);
  const uint32_t oA0 = rl * K + gc0, oA1 = rl * K + gc1;
  const uint32_t oX0 = rl * a.I + gc0, oX1 = rl * a.I + gc1;
  const uint32_t oH0 = rl * H + gc0, oH1 = rl * H + gc1;
  const int8_t* wbase = a.W + (size_t)m0 * K;
  const int8_t* xbase = a.x + (size_t)n0 * a.I;
  const int8_t* hbase = a.h_in + (size_t)n0 * H - a.I;  // k >= I indexes h at k - I
  auto issueA = [&](int s) __attribute__((always_inline)) {
    const int k = s * 128;
    lds_char* st = lds + (s & 1) * STAGE + wave * 4096;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((glb_void*)(wbase + (size_t)(8 * j) * K + k + ((j & 1) ? oA1 : oA0)),
                                       (lds_void*)(st + j * 1024), 16, 0, 0);
  };
  auto issueB = [&](int s) __attribute__((always_inline)) {
    const int k = s * 128;
    lds_char* st = lds + (s & 1) * STAGE + 32768 + wave * 4096;
    if (k < a.I) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_global_load_lds((glb_void*)(xbase + (size_t)(8 * j) * a.I + k + ((j & 1) ? oX1 : oX0)),
                                         (lds_void*)(st + j * 1024), 16, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_global_load_lds((glb_void*)(hbase + (size_t)(8 * j) * H + k + ((j & 1) ? oH1 : oH0)),
                                         (lds_void*)(st + j * 1024), 16, 0, 0);
    }
  };
  // the tile's fp16 cell state (BN rows x 64 units x 2 B = 32 KiB), DMA'd into the buffer the last
  // stage does not occupy once its reads are retired; piece p, lane l: row 8p + (l >> 3), chunk
  // l & 7 at slot (l & 7) ^ (row & 7) (cimg_off: 2-way instead of 8-way epilogue conflicts)
  const int cbuf = (nS & 1) * STAGE;
  auto issue_c = [&]() __attribute__((always_inline)) {
    const uint16_t* cb = a.c + (size_t)n0 * H + (m0 >> 2) + ((lane & 7) ^ ((lane >> 3) & 7)) * 8;
#pragma unroll
    for (int pc = 0; pc < 4; ++pc) {
      const int p = wave * 4 + pc;
      __builtin_amdgcn_global_load_lds((glb_void*)(cb + (size_t)(8 * p + (lane >> 3)) * H), (lds_void*)(lds + cbuf + p * 1024),
                                       16, 0, 0);
    }
  };

  v4i acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  // ---- main loop.  Stage s+1 is DMA'd into the other buffer while stage s is consumed: every
  // wave issues its A pieces right after the stage barrier and its B pieces after the first k
  // step's 32 MFMAs (two half bursts per stage on the load path; measured best of the issue
  // points tried), MFMA clusters at s_setprio 1.  Fragment reads: A rows
  // wm*64 + 16i + col, B rows wn*128 + 16j + col, 16-byte column 4kk + q.
  const int sw = col >> 1;  // (row >> 1) & 7 for rows 16i + col
  const int fa0 = (wm * 64 + col) * 128, fb0 = 32768 + (wn * 128 + col) * 128;
  issueA(0);
  issueB(0);
#ifdef RNNT_DEV_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stamps only: stage 0 landed (this wave)
  EST_PUT(3, __builtin_amdgcn_s_memrealtime());
  EST_PUT(6, __builtin_amdgcn_s_memtime());
#endif
  for (int s = 0; s < nS; ++s) {
    // this wave's DMA of stage s has landed and its LDS reads are drained; after the barrier
    // every wave's has, and every wave is done reading the buffer stage s+1 refills
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (s + 1 < nS) issueA(s + 1);
    else issue_c();
    const int8_t* st = smem + (s & 1) * STAGE;
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
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fra[i], frb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (kk == 0 && s + 1 < nS) {
        issueB(s + 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  // the cell-state DMA has landed for every wave, all fragment reads are done
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#ifdef RNNT_DEV_STAMPS
  EST_PUT(4, __builtin_amdgcn_s_memrealtime());
  EST_PUT(7, __builtin_amdgcn_s_memtime());
#endif

  // ---- fused LSTM cell epilogue (quant_lstm.py:162-183 semantics; oracle_enc_cell)
  const float As = a.rb * 64.0f, Ag = a.rb * 128.0f, ins = a.in_s, outs = a.out_s;
  const float2* tab = (const float2*)(smem + TAB_OFF);
  float4 bq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bq[i] = *(const float4*)(a.bq + m0 + wm * 64 + i * 16 + q * 4);
  // results go to LDS first and leave as whole 128-/64-byte row segments (16 B per lane, full
  // cache lines per wave instruction) instead of 4-/8-byte scattered per-lane stores: c_new in
  // place over the c_in image (each lane rewrites exactly what it read), h and y / the bf16
  // output in the other stage buffer (free after the main loop)
  const int ul = u0 - (m0 >> 2);  // this lane's first unit within the tile's 64
  lds_char* hs = lds + cbuf + 32768;
  lds_char* ys = lds + ((nS - 1) & 1) * STAGE;
  constexpr int HP = 80;  // int8 image pitch (64 B + 16: conflict-free 4-byte writes, 16-B aligned rows)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = nb + 16 * j, r = n - n0;
    const uint2 cv = *(const uint2*)(smem + cbuf + cimg_off(r, ul * 2));
    const float cin[4] = {h2f((uint16_t)(cv.x & 0xffff)), h2f((uint16_t)(cv.x >> 16)), h2f((uint16_t)(cv.y & 0xffff)),
                          h2f((uint16_t)(cv.y >> 16))};
    uint32_t cw[2] = {0u, 0u}, hb[4], yb[4];
    float hv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float cn, hh;
      enc_cell(tab, acc[i][j], bq[i], As, Ag, cin[i], cn, hh);
      cw[i >> 1] |= (uint32_t)f2h(cn) << (16 * (i & 1));
      hv[i] = hh;
      hb[i] = q8_biased(hh * ins);
      yb[i] = q8_biased(hh * outs);
    }
    const uint32_t hq = pack_q8(hb[0], hb[1], hb[2], hb[3]), yq = pack_q8(yb[0], yb[1], yb[2], yb[3]);
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
  __syncthreads();  // the staged images are complete
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
      uint4 v = *(const uint4*)(ys + r * HP + ch * 16);
      if (a.t >= a.lens[n]) v = uint4{0u, 0u, 0u, 0u};  // a value select: no pointer select into a stack temporary
      *(uint4*)(dst + a.half * H) = v;
      if (a.zero_next) *(uint4*)(dst + H) = uint4{0u, 0u, 0u, 0u};
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
// job tile k (0..) of XCD xcd -> (mt, nt); -1 past the XCD's last tile
__device__ __forceinline__ int xcd_pick(const EncTickArgs& args, int xcd, int k, int& mt, int& nt) {
  const int gsel = xcd & 3, psel = xcd >> 2;
  for (int j = 0; j < args.njobs; ++j) {
    const int nbt = args.nbt[j];
    const int b0 = psel ? (nbt + 1) >> 1 : 0;
    const int b1 = psel ? nbt : (nbt + 1) >> 1;
    const int cnt = 4 * (b1 - b0);
    if (k < cnt) {
      mt = gsel * 4 + (k & 3);
      nt = b0 + (k >> 2);
      return j;
    }
    k -= cnt;
  }
  return -1;
}
__global__ void __launch_bounds__(NWAVE * 64, 1) lstm_i8_tick_kernel(EncTickArgs args) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  unsigned long long st_t0 = 0ull;
  EST_MARK(st_t0);
  // sigma table into LDS (read after the main loop's first stage barrier)
#pragma unroll
  for (int i = 0; i < ENC_TAB_N / (2 * NWAVE * 64); ++i)
    ((float4*)(smem + TAB_OFF))[i * NWAVE * 64 + threadIdx.x] = ((const float4*)g_act_tab)[i * NWAVE * 64 + threadIdx.x];
  int mt = 0, nt = 0;
  const int jsel = xcd_pick(args, blockIdx.x & 7, blockIdx.x >> 3, mt, nt);
  if (jsel < 0) return;
  // wave-uniform runtime index into the kernarg segment: the job's fields stay scalar loads
  lstm_i8_step(args.job[__builtin_amdgcn_readfirstlane(jsel)], __builtin_amdgcn_readfirstlane(mt),
               __builtin_amdgcn_readfirstlane(nt), smem, st_t0);
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
  for (int j = 0; j < a.njobs; ++j)
    if (a.job[j].I % 128 != 0 || a.nbt[j] < 0) return -1;
  int per_xcd = 0;  // the batch-half-0 XCDs carry the larger half
  for (int j = 0; j < a.njobs; ++j) per_xcd += 4 * ((a.nbt[j] + 1) / 2);
  if (per_xcd <= 0) return 0;
  hipLaunchKernelGGL(lstm_i8_tick_kernel, dim3(8 * per_xcd), dim3(NWAVE * 64), SMEM_BYTES, st, a);
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
