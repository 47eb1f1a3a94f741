// encoder.hpp -- launch interface of the int8 encoder kernels (internal to the engine).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rnnt {

constexpr int ENC_BATCH_TILE = 128;  // batch rows per encoder workgroup (buffers padded to it)

// Packed row of (unit u, gate g) in the encoder weight image.  A 128-row workgroup tile
// holds 32 units; inside it, wave half wm = (u>>4)&1, MFMA tile i = u&3, lane group
// q = (u>>2)&3 and accumulator register g: row = 128*(u>>5) + 64*wm + 16*i + 4*q + g.  One
// lane then owns the four gates of units u0..u0+3 (u0 = 32*(u>>5) + 16*wm + 4*q) for its
// batch row, so the cell epilogue reads/writes 4 consecutive units per access.
__host__ __device__ __forceinline__ int enc_packed_row(int u, int g) {
  return ((u >> 5) << 7) + (((u >> 4) & 1) << 6) + ((u & 3) << 4) + (((u >> 2) & 3) << 2) + g;
}

enum EncOutMode { ENC_OUT_I8 = 0, ENC_OUT_STACKED = 1, ENC_OUT_FINAL = 2 };

struct EncStepArgs {
  const int8_t* W;     // packed [4096][I+1024], gate-interleaved rows
  const float* bq;     // packed [4096]
  const int8_t* x;     // this frame's input rows: [Npad][I]
  const int8_t* h_in;  // [Npad][1024] h_{t-1} (quantised with in_s)
  int8_t* h_out;       // [Npad][1024] h_t
  uint16_t* c;         // [Npad][1024] fp16 cell state, in place
  int8_t* y8;          // I8: [Npad][1024] frame rows; STACKED: [Npad][2048] stacked frame rows
  float* y32;          // FINAL: optional fp32 f rows [Npad][1024]
  uint16_t* fperm;     // FINAL: bf16 f rows [Npad][1024] in chain-permuted k order
  const int32_t* lens; // [Npad] feature lengths (STACKED masking)
  int I;               // input width (256 / 1024 / 2048)
  int mode;            // EncOutMode
  int t;               // frame index (STACKED)
  int half;            // t % 2 (STACKED)
  int zero_next;       // STACKED: also zero the odd-T pad half
  float rb, in_s, out_s;
};

// One launch runs up to ENC_MAX_JOBS independent layer-steps (the wavefront schedule of
// engine.hip: layer l at its own frame); grid.y enumerates (job, batch tile) pairs.
constexpr int ENC_MAX_JOBS = 5;
struct EncTickArgs {
  EncStepArgs job[ENC_MAX_JOBS];
  int tile_start[ENC_MAX_JOBS + 1];  // prefix sums of each job's active batch tiles
  int njobs;
};

int launch_quantize(const float* feat, int64_t n, float s, int8_t* out, hipStream_t st);
int launch_lstm_i8_tick(const EncTickArgs& a, hipStream_t st);

}  // namespace rnnt
