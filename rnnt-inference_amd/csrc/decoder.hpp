// decoder.hpp -- launch interface of the prediction / joint / greedy kernels (engine-internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rnnt {


struct DecWeights {
  const uint16_t* embed;   // bf16 [28][320] natural
  const uint16_t* wp[2];   // bf16 [1280][640] gate-interleaved rows (4u+g), natural k ([W_ih | W_hh])
  const float* bih_p[2];   // fp32 [1280] b_ih, gate-interleaved
  const float* bhh_p[2];   // fp32 [1280] b_hh, gate-interleaved
  const uint16_t* w1t;     // bf16 [512][1024] natural k
  const uint16_t* w1p;     // bf16 [512][320]  natural k
  const float* bt;         // [512]
  const float* bp;         // [512]
  const uint16_t* w2;      // bf16 [32][512] natural k (rows 29..31 zero)
  const float* b2;         // [32] (29..31 zero)
  const float* xtab;       // [29][1280] layer-0 input half b_ih + emb[g].W_ih^T, gate-interleaved (28 = SOS)
};

struct DecState {           // per-row greedy state, device arrays [Npad]
  int32_t *time, *added, *idx, *preg, *slot, *fin;
  int32_t* list;             // [2][Npad] emit lists (by step parity): row | slot << 24 | label index << 25
  int4* live;                // [2][Npad] unfinished rows (by step parity) with their greedy state:
                             // {row | slot << 24 | symbols_added << 25, time | f_len << 16, idx, 0}
  int32_t* count;            // [4] list lengths {emit p0, live p0, emit p1, live p1} (8-byte aligned)
  int32_t* unfinished;       // [4] live-row counter (the fp32 decode loop)
  uint32_t* pc;              // [8] persistent tail decode: per-role completion counters, abort word, steps run
};

// the persistent tail decode takes at most this many live rows (32 joint workgroups)
constexpr int DEC_PERSIST_MAX = 512;

struct DecArgs {
  DecWeights w;
  const float* F;          // [Tp][Npad][512] joint trans half, F = b_t + bf16(f).W1t^T
  const int32_t* f_lens;   // [Npad]
  float* hc;               // [Npad][2 slots][4][320] (h0, h1, c0, c1) prediction state
  float* G;                // [Npad][512] joint pred half of the current candidate
  float* PH;               // [Npad][1280] layer-1 h-chain gate sums (b_hh + h1.W_hh^T) of the emitting rows
  int32_t* res;            // [N][max_res]
  int32_t* res_len;        // [N]
  DecState s;
  int N, Npad, max_res, max_iter;
  int persist_rows;        // live rows at or below which one persistent launch runs the rest (0 = off, <= DEC_PERSIST_MAX)
};

// F = b_t + bf16(f) . W1t^T for every frame t < Tp and row tile holding a row with f_len > t
// (fbf: the encoder output as bf16 [Tp][Npad][1024], natural k).
int launch_joint_trans(const DecWeights& w, const uint16_t* fbf, const int32_t* f_lens, float* F, int Tp,
                       int Npad, hipStream_t st);
// xtab (device [29][1280] f32) from w.embed / w.wp[0] / w.bih_p[0]; w.xtab is not read.
int launch_dec_xtab(const DecWeights& w, float* xtab, hipStream_t st);
// Host-driven lock-step loop; polls the live-row counter (host_flags: 2 pinned words, evs: 2
// events) one 32-step chunk behind.
// Returns the number of steps enqueued (>= 0) or -1.
// reset != nullptr: Server continuous batching -- slots keep their greedy state across calls and
// reset[row] != 0 starts a new utterance in that slot (dec_init_stream_kernel).
int launch_greedy_decode(const DecArgs& a, int32_t* host_flags, hipEvent_t* evs, hipStream_t st,
                         const int32_t* reset = nullptr);

}  // namespace rnnt
