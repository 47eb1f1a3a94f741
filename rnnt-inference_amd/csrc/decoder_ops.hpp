// decoder_ops.hpp -- launch interface of the operator-level decode kernels (engine-internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "decoder.hpp"

namespace rnnt {

struct GreedyUpdateArgs {
  const int32_t* symbols;  // [n] argmax of the joint
  int32_t* symbols_added;  // [n]
  int32_t* res;            // [n][max_res]
  int32_t* res_idx;        // [n]
  const float* f;          // [Tp][n_pad][1024] encoder output
  const int32_t* f_lens;   // [n]
  int32_t* time_idx;       // [n]
  float* fi;               // [n_pad][1024] current frame rows
  int32_t* pre_g;          // [n]
  uint16_t* pre_hg;        // bf16 [2][n_pad][320]
  float* pre_cg;           // [2][n_pad][320]
  const uint16_t* hg;      // bf16 [2][n_pad][320] candidate state
  const float* cg;         // [2][n_pad][320]
  int32_t* finish;         // [n] (decoder.py:106 `self.finish`)
  int32_t* unfinished;     // device counter of rows not finished (decremented here)
  int n, n_pad, max_res;
};

int launch_op_lstm_bf16(const DecWeights& w, int layer, const uint16_t* x, const uint16_t* h_in, const float* c_in,
                        uint16_t* h_out, float* c_out, int n_pad, hipStream_t st);
int launch_op_joint_hidden(const DecWeights& w, const float* f, const uint16_t* g, uint16_t* y1, int n_pad,
                           hipStream_t st);
int launch_op_joint_logits(const DecWeights& w, const uint16_t* y1, float* logits, int n_pad, hipStream_t st);
int launch_op_greedy_update(const GreedyUpdateArgs& a, hipStream_t st);

}  // namespace rnnt
