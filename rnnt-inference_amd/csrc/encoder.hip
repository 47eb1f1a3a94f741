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

// ---------------------------------------------------------------- LSTM step
constexpr int BM = 128;  // gate rows per workgroup (32 units x 4 gates)
constexpr int BN = 128;  // batch rows per workgroup
constexpr int BK = 64;   // k bytes per stage (one 16x16x64 MFMA depth)
constexpr int NSTAGE = 3;                       // LDS ring depth (2 stages in flight)
constexpr int STAGE_BYTES = (BM + BN) * BK;     // 16 KiB: A image then B image
constexpr int GLDS_PER_STAGE = 4;               // per wave: 2 x 1 KiB pieces of A, 2 of B

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// LDS image of a [128][64 B] tile: 16-byte column c of row r is stored at column
// c ^ h[(r >> 2) & 3] with h = {0, 2, 3, 1}.  A fragment read (lane l: row l&15, column l>>4)
// is a ds_read_b128 whose four 16-lane groups each touch rows {0-3,12-15} at one column and
// rows 4-11 at the next; with this h every group lands on 16 distinct 16-byte bank slots.
__device__ __forceinline__ int swz_h(int row) { return (0x1320 >> (((row >> 2) & 3) * 4)) & 3; }
__device__ __forceinline__ int swz(int row, int col16) { return row * BK + ((col16 ^ swz_h(row)) << 4); }

// Retire this wave's LDS-DMA down to N outstanding, drain LDS ops, then barrier: after it,
// every wave's DMA of the retired stage has landed (each wave waited for its own) and every
// wave's reads of the previous stage are done.  One asm statement so the "memory" clobber
// orders it against the compiler's LDS accesses on both sides.
template <int N>
__device__ __forceinline__ void stage_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lstm_i8_step(const EncStepArgs& a, int tile, int8_t* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.x * BM;  // packed gate row base
  const int n0 = tile * BN;        // batch row base
  const int K = a.I + H;
  const int nK = K / BK;

  // ---- epilogue operands, prefetched so their latency hides under the main loop
  const int q = lane >> 4, col = lane & 15;
  const int u0 = (m0 >> 2) + wm * 16 + q * 4;  // this lane's 4 consecutive units
  int nrow[4];
  uint2 cpre[4];
  int lpre[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    nrow[j] = n0 + wn * 64 + j * 16 + col;
    cpre[j] = *(const uint2*)(a.c + (size_t)nrow[j] * H + u0);
    lpre[j] = a.lens ? a.lens[nrow[j]] : 0;
  }
  float4 bq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) bq[i] = *(const float4*)(a.bq + m0 + wm * 64 + i * 16 + q * 4);

  // ---- LDS-DMA staging: wave w moves pieces 2w, 2w+1 (16 rows x 64 B each) of A and of B;
  // lane l of a piece lands at LDS slot 64p + l = row*4 + (col16 ^ h(row)), so it fetches
  // row 16p + (l>>2), column (l&3) ^ h (h depends on l>>4 only).
  const int hx = (0x1320 >> ((lane >> 4) * 4)) & 3;  // h(row): (row>>2)&3 == lane>>4
  const int gcol = ((lane & 3) ^ hx) * 16;
  const int ra = wave * 32 + (lane >> 2), rb = ra + 16;  // rows of this wave's two pieces
  const int8_t* wa0 = a.W + (size_t)(m0 + ra) * K + gcol;
  const int8_t* wa1 = a.W + (size_t)(m0 + rb) * K + gcol;
  const int8_t* xb0 = a.x + (size_t)(n0 + ra) * a.I + gcol;
  const int8_t* xb1 = a.x + (size_t)(n0 + rb) * a.I + gcol;
  const int8_t* hb0 = a.h_in + (size_t)(n0 + ra) * H + gcol - a.I;
  const int8_t* hb1 = a.h_in + (size_t)(n0 + rb) * H + gcol - a.I;
  lds_void* lds_base = (lds_void*)smem;

  auto issue = [&](int ks) __attribute__((always_inline)) {
    const int k = ks * BK;
    char __attribute__((address_space(3)))* st = (char __attribute__((address_space(3)))*)lds_base + (ks % NSTAGE) * STAGE_BYTES;
    __builtin_amdgcn_global_load_lds((glb_void*)(wa0 + k), (lds_void*)(st + (wave * 2) * 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((glb_void*)(wa1 + k), (lds_void*)(st + (wave * 2 + 1) * 1024), 16, 0, 0);
    const int8_t* b0 = k < a.I ? xb0 + k : hb0 + k;
    const int8_t* b1 = k < a.I ? xb1 + k : hb1 + k;
    __builtin_amdgcn_global_load_lds((glb_void*)b0, (lds_void*)(st + BM * BK + (wave * 2) * 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((glb_void*)b1, (lds_void*)(st + BM * BK + (wave * 2 + 1) * 1024), 16, 0, 0);
  };

  v4i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  // fragment read offsets (rows wm*64 + i*16 + (lane&15), 16-byte column lane>>4)
  int fa_off[4], fb_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    fa_off[i] = swz(wm * 64 + i * 16 + col, q);
    fb_off[i] = BM * BK + swz(wn * 64 + i * 16 + col, q);
  }

  issue(0);
  issue(1);  // nK >= 20 for every layer
  for (int ks = 0; ks < nK; ++ks) {
    if (ks + 1 < nK) stage_barrier<GLDS_PER_STAGE>();
    else stage_barrier<0>();
    if (ks + 2 < nK) issue(ks + 2);
    const int8_t* st = smem + (ks % NSTAGE) * STAGE_BYTES;
    v4i fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = *(const v4i*)(st + fa_off[i]);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = *(const v4i*)(st + fb_off[j]);
#ifdef RNNT_DEV_NO_MFMA  // development ablation: staging + LDS reads only
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(fa[i]), "v"(fb[i]));
#else
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
#endif
  }
#ifdef RNNT_DEV_NO_EPI  // development ablation: main loop only
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
  asm volatile("" ::"v"(cpre[0].x), "v"(cpre[3].y), "v"(bq[0].x), "v"(bq[3].w), "v"(lpre[0]));
  return;
#endif

  // ---- fused LSTM cell epilogue (quant_lstm.py:162-183 semantics; see oracle_lstm_i8_layer)
  const float rbs = a.rb, ins = a.in_s, outs = a.out_s;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = nrow[j];
    const uint16_t cin[4] = {(uint16_t)(cpre[j].x & 0xffff), (uint16_t)(cpre[j].x >> 16),
                             (uint16_t)(cpre[j].y & 0xffff), (uint16_t)(cpre[j].y >> 16)};
    uint16_t cout[4];
    uint32_t hq = 0, yq = 0;
    float hv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float pi = ((float)acc[i][j][0] + bq[i].x) * rbs;
      const float pf = ((float)acc[i][j][1] + bq[i].y) * rbs;
      const float pg = ((float)acc[i][j][2] + bq[i].z) * rbs;
      const float po = ((float)acc[i][j][3] + bq[i].w) * rbs;
      const float ig = det_sigmoid(pi), fg = det_sigmoid(pf), gg = det_tanh(pg), og = det_sigmoid(po);
      const float cn = fg * h2f(cin[i]) + ig * gg;
      cout[i] = f2h(cn);
      const float hh = og * det_tanh(cn);
      hv[i] = hh;
      hq |= (uint32_t)(uint8_t)q8(hh * ins) << (8 * i);
      yq |= (uint32_t)(uint8_t)q8(hh * outs) << (8 * i);
    }
    *(uint2*)(a.c + (size_t)n * H + u0) =
        uint2{(uint32_t)cout[0] | ((uint32_t)cout[1] << 16), (uint32_t)cout[2] | ((uint32_t)cout[3] << 16)};
    *(uint32_t*)(a.h_out + (size_t)n * H + u0) = hq;
    if (a.mode == ENC_OUT_I8) {
      *(uint32_t*)(a.y8 + (size_t)n * H + u0) = yq;
    } else if (a.mode == ENC_OUT_STACKED) {
      // StackTime (modeling_rnnt.py:314-324): frame t -> stacked frame t/2, half t%2;
      // frames t >= x_lens[n] are zeroed; the odd-T pad frame is zero too.
      int8_t* dst = a.y8 + (size_t)n * (2 * H) + u0;
      *(uint32_t*)(dst + a.half * H) = (a.t < lpre[j]) ? yq : 0u;
      if (a.zero_next) *(uint32_t*)(dst + H) = 0u;
    } else {
      if (a.y32) *(float4*)(a.y32 + (size_t)n * H + u0) = float4{hv[0], hv[1], hv[2], hv[3]};
#pragma unroll
      for (int i = 0; i < 4; ++i) a.fperm[(size_t)n * H + chain_pos(u0 + i)] = f2bf(hv[i]);
    }
  }
}

__global__ void __launch_bounds__(256, 2) lstm_i8_tick_kernel(EncTickArgs args) {
  __shared__ __attribute__((aligned(16))) int8_t smem[NSTAGE * STAGE_BYTES];
  const int y = blockIdx.y;
  // wave-uniform job lookup; each case inlines the body with a constant job index so the
  // job's arguments stay in the kernarg segment (scalar loads, no private copy)
  if (y < args.tile_start[1]) {
    lstm_i8_step(args.job[0], y, smem);
  } else if (y < args.tile_start[2]) {
    lstm_i8_step(args.job[1], y - args.tile_start[1], smem);
  } else if (y < args.tile_start[3]) {
    lstm_i8_step(args.job[2], y - args.tile_start[2], smem);
  } else if (y < args.tile_start[4]) {
    lstm_i8_step(args.job[3], y - args.tile_start[3], smem);
  } else {
    lstm_i8_step(args.job[4], y - args.tile_start[4], smem);
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

int launch_lstm_i8_tick(const EncTickArgs& a, hipStream_t st) {
  const int tiles = a.tile_start[a.njobs];
  if (tiles <= 0) return 0;
  hipLaunchKernelGGL(lstm_i8_tick_kernel, dim3(G4 / BM, tiles), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rnnt
