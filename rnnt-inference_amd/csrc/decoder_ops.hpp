// decoder_ops.hpp -- launch interface of the operator-level decode kernels (engine-internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "decoder.hpp"

namespace rnnt {

// greedy_decode_update's operands in the reference's own shapes (modeling_rnnt.py:351-365,
// rnnt_model.hpp:92-124): per-layer state tensors, f [Tp][f_batch][1024].  The spec's per-row
// `finish` flag (decoder.py:106) is not an operand of the reference op; it is carried in
// time_idx: a row is finished once time_idx >= f_lens (time_idx is left unclamped when the row
// finishes, so f_lens == 0 rows are finished from the start, as decoder.py:106 has it).
struct GreedyUpdateArgs {
  const void* symbols;     // [n] argmax of the joint (int64 from torch.argmax, or int32)
  bool sym64;
  int32_t* symbols_added;  // [n]
  int32_t* res;            // [n][max_res]
  int32_t* res_idx;        // [n]
  const float* f;          // [Tp][f_batch][1024] encoder output
  int f_batch;
  const int32_t* f_lens;   // [n]
  int32_t* time_idx;       // [n]
  float* fi;               // [n][1024] current frame rows
  int32_t* pre_g;          // [n]
  uint16_t* pre_hg[2];     // bf16 [n][320] per layer
  float* pre_cg[2];        // [n][320]
  const uint16_t* hg[2];   // bf16 [n][320] candidate state
  const float* cg[2];      // [n][320]
  int n, max_res;
};

int launch_op_lstm_bf16(const DecWeights& w, int layer, const uint16_t* x, const uint16_t* h_in, const float* c_in,
                        uint16_t* h_out, float* c_out, int n_pad, hipStream_t st);
int launch_op_joint_hidden(const DecWeights& w, const float* f, const uint16_t* g, uint16_t* y1, int n_pad,
                           hipStream_t st);
int launch_op_joint_logits(const DecWeights& w, const uint16_t* y1, float* logits, int n_pad, hipStream_t st);
int launch_op_greedy_update(const GreedyUpdateArgs& a, hipStream_t st);

}  // namespace rnnt
