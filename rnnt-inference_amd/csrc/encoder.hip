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

// LDS image of a [128][64 B] tile: 16-byte column c of row r is stored at column
// c ^ h[(r >> 2) & 3] with h = {0, 2, 3, 1}.  A fragment read (lane l: row l&15, column l>>4)
// is a ds_read_b128 whose four 16-lane groups each touch rows {0-3,12-15} at one column and
// rows 4-11 at the next; with this h every group lands on 16 distinct 16-byte bank slots
// (the plain c ^ ((r>>2)&3) swizzle leaves them 2-way conflicted).
__device__ __forceinline__ int swz(int row, int col16) {
  const int h = (0x1320 >> (((row >> 2) & 3) * 4)) & 3;  // nibbles: h[0]=0 h[1]=2 h[2]=3 h[3]=1
  return row * BK + ((col16 ^ h) << 4);
}

__device__ __forceinline__ void lstm_i8_step(const EncStepArgs& a, int tile, int8_t* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.x * BM;  // packed gate row base
  const int n0 = tile * BN;        // batch row base
  const int K = a.I + H;
  const int nK = K / BK;

  // staging assignment: chunk ch = tid (+256): row ch>>2, 16-byte column ch&3
  const int r0 = tid >> 2, r1 = r0 + 64, cc = tid & 3;
  const int8_t* wa0 = a.W + (size_t)(m0 + r0) * K + cc * 16;
  const int8_t* wa1 = a.W + (size_t)(m0 + r1) * K + cc * 16;
  const int8_t* xb0 = a.x + (size_t)(n0 + r0) * a.I + cc * 16;
  const int8_t* xb1 = a.x + (size_t)(n0 + r1) * a.I + cc * 16;
  const int8_t* hb0 = a.h_in + (size_t)(n0 + r0) * H + cc * 16 - a.I;
  const int8_t* hb1 = a.h_in + (size_t)(n0 + r1) * H + cc * 16 - a.I;
  const int sa0 = swz(r0, cc), sa1 = swz(r1, cc);

  v4i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  uint4 ra0 = *(const uint4*)(wa0), ra1 = *(const uint4*)(wa1);
  uint4 rb0 = *(const uint4*)(a.I > 0 ? xb0 : hb0), rb1 = *(const uint4*)(a.I > 0 ? xb1 : hb1);
  {
    int8_t* As = smem;
    int8_t* Bs = smem + BM * BK;
    *(uint4*)(As + sa0) = ra0; *(uint4*)(As + sa1) = ra1;
    *(uint4*)(Bs + sa0) = rb0; *(uint4*)(Bs + sa1) = rb1;
  }
  __syncthreads();

  // fragment read offsets (rows wm*64 + i*16 + (lane&15), 16-byte column lane>>4)
  int fa_off[4], fb_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    fa_off[i] = swz(wm * 64 + i * 16 + (lane & 15), lane >> 4);
    fb_off[i] = swz(wn * 64 + i * 16 + (lane & 15), lane >> 4);
  }

  for (int ks = 0; ks < nK; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nK;
    if (more) {
      const int k1 = (ks + 1) * BK;
      ra0 = *(const uint4*)(wa0 + k1);
      ra1 = *(const uint4*)(wa1 + k1);
      if (k1 < a.I) {
        rb0 = *(const uint4*)(xb0 + k1);
        rb1 = *(const uint4*)(xb1 + k1);
      } else {
        rb0 = *(const uint4*)(hb0 + k1);
        rb1 = *(const uint4*)(hb1 + k1);
      }
    }
    const int8_t* As = smem + cur * (BM + BN) * BK;
    const int8_t* Bs = As + BM * BK;
    v4i fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = *(const v4i*)(As + fa_off[i]);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = *(const v4i*)(Bs + fb_off[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (more) {
      int8_t* An = smem + (cur ^ 1) * (BM + BN) * BK;
      int8_t* Bn = An + BM * BK;
      *(uint4*)(An + sa0) = ra0; *(uint4*)(An + sa1) = ra1;
      *(uint4*)(Bn + sa0) = rb0; *(uint4*)(Bn + sa1) = rb1;
    }
    __syncthreads();
  }

  // ---- fused LSTM cell epilogue (quant_lstm.py:162-183 semantics; see oracle_lstm_i8_layer)
  const float rbs = a.rb, ins = a.in_s, outs = a.out_s;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = (m0 >> 2) + wm * 16 + i * 4 + (lane >> 4);
    const float4 bq = *(const float4*)(a.bq + 4 * u);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
      const float pi = ((float)acc[i][j][0] + bq.x) * rbs;
      const float pf = ((float)acc[i][j][1] + bq.y) * rbs;
      const float pg = ((float)acc[i][j][2] + bq.z) * rbs;
      const float po = ((float)acc[i][j][3] + bq.w) * rbs;
      const float ig = det_sigmoid(pi), fg = det_sigmoid(pf), gg = det_tanh(pg), og = det_sigmoid(po);
      uint16_t* cptr = a.c + (size_t)n * H + u;
      const float cp = h2f(*cptr);
      const float cn = fg * cp + ig * gg;
      *cptr = f2h(cn);
      const float hh = og * det_tanh(cn);
      a.h_out[(size_t)n * H + u] = q8(hh * ins);
      if (a.mode == ENC_OUT_I8) {
        a.y8[(size_t)n * H + u] = q8(hh * outs);
      } else if (a.mode == ENC_OUT_STACKED) {
        // StackTime (modeling_rnnt.py:314-324): frame t -> stacked frame t/2, half t%2;
        // frames t >= x_lens[n] are zeroed; the odd-T pad frame is zero too.
        int8_t* dst = a.y8 + (size_t)n * (2 * H) + u;
        dst[a.half * H] = (a.t < a.lens[n]) ? q8(hh * outs) : (int8_t)0;
        if (a.zero_next) dst[H] = 0;
      } else {
        if (a.y32) a.y32[(size_t)n * H + u] = hh;
        a.fperm[(size_t)n * H + chain_pos(u)] = f2bf(hh);
      }
    }
  }
}

__global__ void __launch_bounds__(256, 2) lstm_i8_tick_kernel(EncTickArgs args) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * (BM + BN) * BK];
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
