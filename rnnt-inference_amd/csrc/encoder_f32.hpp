// encoder_f32.hpp -- launch interface of the fp32 encoder kernels (engine-internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rnnt {

enum EncF32Mode { ENC_F32_NEXT = 0, ENC_F32_STACKED = 1, ENC_F32_FINAL = 2 };

struct EncF32StepArgs {
  const float* wih;     // [4096][Ip] packed rows (4u+g), chain-permuted k, zero past I
  const float* whh;     // [4096][1024] packed rows, chain-permuted k
  const float* bih;     // [4096] packed
  const float* bhh;     // [4096] packed
  const float* x;       // this frame's input rows [n_pad][Ip], chain-permuted
  const float* h_in;    // [n_pad][1024] chain-permuted
  float* h_out;         // [n_pad][1024] chain-permuted
  float* c;             // [n_pad][1024] natural
  float* y;             // NEXT: [n_pad][1024] chain-permuted; STACKED: [n_pad][2048] chain-permuted;
                        // FINAL: [n_pad][1024] natural (f)
  float* y2;            // FINAL: optional second copy of f, [n_pad][1024] chain-permuted (fp32 decoder input)
  uint16_t* ybf;        // FINAL: optional bf16 copy of f, [n_pad][1024] natural, subnormals flushed
                        // (the f32 + enable_bf16 decoder input, decoder.py:121-122)
  const int32_t* lens;  // STACKED masking
  int I, Ip;            // real / padded input width (240/256, 1024/1024, 2048/2048)
  int n;                // rows to compute (multiple-of-64 tiles launched; rows >= n skipped)
  int mode, t, half, zero_next;
};

// The fp32 contract's chain segment (oracle_lstm_f32_layer): a gate's x and h dot products are
// k-ordered fma chains over 512-k segments, summed in segment order, the first from the bias.
constexpr int ENC_F32_SEG = 512;

// One launch = one wavefront tick of the fp32 stack (the int8 encoder's schedule, engine.hip):
// up to 5 independent layer-steps over the same n rows (n_pad a multiple of 64).
constexpr int ENC_F32_MAX_JOBS = 5;
struct EncF32TickArgs {
  EncF32StepArgs job[ENC_F32_MAX_JOBS];  // longest K first
  int njobs;
};
int launch_lstm_f32_tick(const EncF32TickArgs& a, hipStream_t st);
int launch_permute_feats(const float* x, int64_t rows, float* y, hipStream_t st);

}  // namespace rnnt
