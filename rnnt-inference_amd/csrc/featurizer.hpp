// featurizer.hpp -- log-mel front end kernels (engine-internal launch interface).
//
// The reference's AudioProcessing / FilterbankFeatures.forward (datasets/parts/features.py:185-252,
// datasets/process_librispeech.py:100-111) with the rnnt.toml [input_eval] geometry:
// 16 kHz, n_fft 512, hop 160, hann window 320, 80 mel filters, frame splicing 3, per-feature
// normalisation, channel pad 240 -> 256.  Numerics contract: DESIGN.md "Featurizer".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace rnnt {

constexpr int FZ_NFFT = 512;                  // n_fft
constexpr int FZ_NBIN = FZ_NFFT / 2 + 1;      // 257 one-sided bins
constexpr int FZ_HOP = 160;                   // window_stride 0.01 s
constexpr int FZ_WIN = 320;                   // window_size 0.02 s (hann, periodic=False)
constexpr int FZ_NMEL = 80;                   // features
constexpr int FZ_SPLICE = 3;                  // frame_splicing
constexpr int FZ_FEAT = FZ_NMEL * FZ_SPLICE;  // 240 = TRANS_INPUT_SIZE (metadata.hpp:22)
constexpr int FZ_FEAT_PAD = 256;              // PADDED_INPUT_SIZE (metadata.hpp:33)
constexpr int FZ_CHUNK = 16;                  // STFT frames per workgroup (one mel MFMA row tile)
constexpr int FZ_MEL_COLS = FZ_NMEL / 16;     // 5 filter column tiles

struct FzConsts {           // device constants built at rnnt_featurizer_create
  const float* window;      // [320]
  const float2* twiddle;    // [512] (cos, -sin)(2 pi t / 512)
  const float* fbB;         // [sum col_steps][64] v_mfma_f32_16x16x4f32 B fragments of fb^T:
                            // lane l of step s of column tile c = fb[16c + l%16][col_k0[c] + 4s + l/16]
  int col_k0[FZ_MEL_COLS];  // first bin of column tile c's non-zero span
  int col_steps[FZ_MEL_COLS];
  int col_off[FZ_MEL_COLS]; // first step of column tile c in fbB
  int wave_cols[4];         // column tiles (bitmask) each wave projects, balanced on the host
  float preemph, dither_sq, log_guard, eps;
};

struct FzArgs {
  FzConsts k;
  const float* wav;         // samples of row n at wav + off[n] (or n * stride)
  const int64_t* off;       // [n] or nullptr
  int64_t stride;
  const int32_t* wav_lens;  // [n]
  float* feats;             // [T_out][n_pad][256], or ragged rows (row_off)
  const int64_t* row_off;   // ragged output: frame t of row n at feats + (row_off[n] + t) * 240 (nullptr: padded)
  int32_t* feat_lens;       // [n_pad] ([n] ragged)
  int2* plan;               // [chunks] (utterance, chunk) per fz_logmel workgroup (fz_plan_kernel)
  int n, n_pad, T_out;
  int n_chunks;             // plan entries (fz_logmel sub-groups past it idle)
};

}  // namespace rnnt

// shared with engine.hip: records msg as rnnt_last_error() and returns code
int rnnt_internal_fail(int code, const std::string& msg);
