// decoder_f32.hpp -- launch interface of the fp32 prediction / joint / greedy kernels
// (engine-internal; the run_mode="f32" decoder without enable_bf16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rnnt {

struct DecF32Weights {
  const float* emb;             // [29][320] chain-permuted k; row 28 = 0 (SOS, modeling_rnnt.py:195-200)
  const float* wih[2];          // [1280][320] gate-interleaved rows (4u+g), chain-permuted k
  const float* whh[2];          // [1280][320]
  const float* bih[2];          // [1280] gate-interleaved
  const float* bhh[2];          // [1280]
  const float* w1t;             // [512][1024] chain-permuted k (joint.linear1_trans)
  const float* w1p;             // [512][320]  chain-permuted k (joint.linear1_pred)
  const float* bt;              // [512]
  const float* bp;              // [512]
  const float* w2;              // [32][512] chain-permuted k, rows 29..31 zero
  const float* b2;              // [32], 29..31 zero
};

struct DecF32State {            // device arrays, rows [Npad]
  float* ph;                    // [2][Npad][320] committed prediction h (chain-permuted)
  float* pc;                    // [2][Npad][320] committed c (natural)
  float* gh;                    // [2][Npad][320] candidate h (chain-permuted)
  float* gc;                    // [2][Npad][320] candidate c (natural)
  int32_t *time, *added, *idx, *preg, *fin;
  int32_t* unfinished;          // [1]
};

struct DecF32Args {
  DecF32Weights w;
  DecF32State s;
  const float* F;               // [Tp][Npad][512] natural: b_t + f.W1t^T
  const int32_t* f_lens;        // [Npad] (0 for batch padding)
  int32_t* res;                 // [N][max_res]
  int32_t* res_len;             // [N]
  int N, Npad, max_res, max_iter;
};

// F = b_t + fc . W1t^T for every frame and row (fc: encoder output [Tp][Npad][1024] chain-permuted).
int launch_f32_joint_trans(const DecF32Weights& w, const float* fc, float* F, int Tp, int Npad, hipStream_t st);
// Lock-step greedy loop over the whole batch; polls the unfinished-row counter one 32-step
// chunk behind (host_flags: 2 pinned words, evs: 2 events).  Returns the steps enqueued or -1.
int launch_greedy_decode_f32(const DecF32Args& a, int32_t* host_flags, hipEvent_t* evs, hipStream_t st);
// One fp32 prediction LSTM layer (intel_mlperf::lstm) over n_pad rows (a multiple of 64), natural
// layouts: x / h_in / c_in / h_out / c_out fp32 [n_pad][320]; h_out, c_out must not alias inputs.
int launch_op_lstm_f32(const DecF32Weights& w, int layer, const float* x, const float* h_in, const float* c_in,
                       float* h_out, float* c_out, int n_pad, hipStream_t st);

}  // namespace rnnt
