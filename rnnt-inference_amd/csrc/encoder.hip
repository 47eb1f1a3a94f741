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
constexpr int BM = 128;        // gate rows per workgroup (32 units x 4 gates)
constexpr int BN = 128;        // batch rows per workgroup
constexpr int BK = 64;         // k bytes per stage (one 16x16x64 MFMA depth)
constexpr int PITCH = BK + 16; // LDS row pitch (bytes): breaks the 64-B power-of-two stride

__global__ void __launch_bounds__(256, 2) lstm_i8_step_kernel(EncStepArgs a) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * 2 * BM * PITCH];
  int8_t* As = smem;                    // [2][BM][PITCH]
  int8_t* Bs = smem + 2 * BM * PITCH;   // [2][BN][PITCH]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.x * BM;       // packed gate row base
  const int n0 = blockIdx.y * BN;       // batch row base
  const int K = a.I + H;
  const int nK = K / BK;

  // global -> register staging: 2 A chunks + 2 B chunks of 16 B per thread per stage
  uint4 ra[2], rb[2];
  auto load_stage = [&](int ks) {
    const int k0 = ks * BK;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int ch = tid + c * 256, row = ch >> 2, col = (ch & 3) * 16;
      ra[c] = *(const uint4*)(a.W + (size_t)(m0 + row) * K + k0 + col);
      const int n = n0 + row;
      const int8_t* src = (k0 < a.I) ? a.x + (size_t)n * a.I + k0 + col
                                      : a.h_in + (size_t)n * H + (k0 - a.I) + col;
      rb[c] = *(const uint4*)src;
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int ch = tid + c * 256, row = ch >> 2, col = (ch & 3) * 16;
      *(uint4*)(As + (buf * BM + row) * PITCH + col) = ra[c];
      *(uint4*)(Bs + (buf * BN + row) * PITCH + col) = rb[c];
    }
  };

  v4i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  load_stage(0);
  store_stage(0);
  __syncthreads();
  int cur = 0;
  for (int ks = 0; ks < nK; ++ks) {
    if (ks + 1 < nK) load_stage(ks + 1);
    v4i fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      fa[i] = *(const v4i*)(As + (cur * BM + wm * 64 + i * 16 + (lane & 15)) * PITCH + (lane >> 4) * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      fb[j] = *(const v4i*)(Bs + (cur * BN + wn * 64 + j * 16 + (lane & 15)) * PITCH + (lane >> 4) * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (ks + 1 < nK) store_stage(cur ^ 1);
    __syncthreads();
    cur ^= 1;
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

// ---------------------------------------------------------------- host launchers
int launch_quantize(const float* feat, int64_t n, float s, int8_t* out, hipStream_t st) {
  const int64_t n4 = n / 4;
  int grid = (int)((n4 + 255) / 256);
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(quantize_kernel, dim3(grid), dim3(256), 0, st, (const float4*)feat, n4, s, (uint32_t*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_lstm_i8_step(const EncStepArgs& a, int n_tiles, hipStream_t st) {
  if (n_tiles <= 0) return 0;
  hipLaunchKernelGGL(lstm_i8_step_kernel, dim3(G4 / BM, n_tiles), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rnnt
