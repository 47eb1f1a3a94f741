/*
 * rnnt_oracle.h -- CPU restatement of the reference RNN-T hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker the HIP engine is compared against; it is
 * never linked into, loaded by, or called from the product path (rnnt-inference_amd/).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 *
 * The reference's native kernels live in the un-vendored `mlperf_plugins` submodule
 * (reference .gitmodules:1-3; no pinned SHA), so each function restates the *Python*
 * semantics the reference documents for its op (file:line cited per function) and pins
 * the choices the absent plugin leaves open (DESIGN.md "Numerics contract").
 *
 * Layouts are the reference's natural ones (row r of a gate matrix = gate*H + unit, gate
 * order i,f,g,o as in quant_lstm.py:174), not the engine's packed MFMA layouts.
 */
#ifndef RNNT_ORACLE_H
#define RNNT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- scalar numerics (exported so tests can check them against libm / torch) ---- */
float oracle_exp(float x);
float oracle_sigmoid(float x);
float oracle_tanh(float x);
float oracle_act_sig_t(float t);  /* table sigma at t = 64x + 1024 (int8 cell, see rnnt_oracle.c) */
float oracle_enc_bias(float bq, float rb, int gate);
void oracle_enc_cell(const int32_t acc[4], const float B[4], float rb, float c_prev,
                     float* c_out, float* h_out);
uint16_t oracle_f2h(float x);      /* f32 -> f16 bits, round-half-even */
float oracle_h2f(uint16_t h);
uint16_t oracle_f2bf(float x);     /* f32 -> bf16 bits, round-half-even */
float oracle_bf2f(uint16_t b);
/* bf16 MFMA dot (v_mfma_f32_16x16x32_bf16 accumulation model, see rnnt_oracle.c):
 * out[n] = acc[n] (+) a[n][0:K] . b[n][0:K], K a multiple of 8, a/b bf16-exact floats. */
void oracle_mfma_bf16_dot(int N, int K, const float* acc, const float* a, const float* b, float* out);
int8_t oracle_q8(float v);         /* clamp(round_half_even(v), -128, 127): quant_modules.py:8-9,118-121 */

/* Elementwise quantisation x_q = q8(x * scale). */
void oracle_quantize(const float* x, int64_t n, float scale, int8_t* out);

/* One int8 LSTM layer over T steps (quant_lstm.py:162-183 cell, :193-215 quantised params).
 * x: [T][N][I] int8 (already quantised with in_s); W: [4H][I+H] int8 = [W_ih | W_hh];
 * bq: [4H] fused bias (b_ih+b_hh)*in_s*s_w; h: [N][H] int8 state (in_s) in/out;
 * c: [N][H] fp16-bits cell state in/out; outputs y8 [T][N][H] (q8(h*out_s)) or y32 (h). */
void oracle_lstm_i8_layer(int T, int N, int I, int H, const int8_t* x, const int8_t* W,
                          const float* bq, float rb, float in_s, float out_s, int skip_quant_y,
                          int8_t* h, uint16_t* c, int8_t* y8, float* y32);

/* StackTime (modeling_rnnt.py:314-324): zero frames t >= lens[n], pad T to even, concat
 * pairs: y[t'][n] = [x[2t'][n], x[2t'+1][n]].  x: [T][N][C] -> y: [ceil(T/2)][N][2C]. */
void oracle_stack_time_i8(int T, int N, int C, const int8_t* x, const int32_t* lens, int8_t* y);
void oracle_stack_time_f32(int T, int N, int C, const float* x, const int32_t* lens, float* y);

/* Whole int8 transcription (modeling_rnnt.py:116-144): quantise features with in_s[0],
 * pre_rnn 2 layers, stack_time(2), post_rnn 3 layers (last skip_quant_y).
 * feat: [T][N][256] f32 (240 real channels + 16 zero pad, metadata.hpp:33);
 * W[l]: [4096][I_l+1024] with I = 256,1024,2048,1024,1024; f_out: [ceil(T/2)][N][1024].
 * h_state [5][N][1024] int8 / c_state [5][N][1024] fp16 may be NULL (zero initial state,
 * no state out) or point at carried state (chunked encode, rnnt_model.hpp:62-90). */
void oracle_encoder_i8(int T, int N, const float* feat, const int32_t* lens,
                       const int8_t* const* W, const float* const* bq, const float* rb,
                       const float* in_s, const float* out_s, float* f_out,
                       int8_t* h_state, uint16_t* c_state);

/* fp32 LSTM layer (QuantLSTMLayer.forward with no quantizers, quant_lstm.py:162-183):
 * gates = (b_ih + x.W_ih^T) + (b_hh + h.W_hh^T), each dot k-ordered fmaf chains over 512-k
 * segments summed in segment order (the GPU fp32 encoder's contract). */
void oracle_lstm_f32_layer(int T, int N, int I, int H, const float* x, const float* Wih,
                           const float* Whh, const float* bih, const float* bhh, float* h,
                           float* c, float* y);

/* Whole fp32 transcription: feat [T][N][240 or 256] (I0 = 240 or 256 channels). */
void oracle_encoder_f32(int T, int N, int I0, const float* feat, const int32_t* lens,
                        const float* const* Wih, const float* const* Whh,
                        const float* const* bih, const float* const* bhh, float* f_out);

/* Prediction + joint + greedy decode (modeling_rnnt.py:147-289, decoder.py:102-169).
 * bf16 != 0 reproduces the enable_bf16 path: weights/embedding hold bf16-exact values,
 * h of the prediction LSTM, the encoder frame fed to the joint and the joint hidden are
 * rounded to bf16; every dot product is a k-ordered fmaf chain with fp32 accumulation.
 *   embed [28][320]; pWih/pWhh [2][1280][320]; pbih/pbhh [2][1280];
 *   W1t [512][1024], W1p [512][320], bt/bp [512]; W2 [29][512], b2 [29].
 * f: [Tp][N][1024] encoder output; f_lens [N] (= ceil(feature_len/2)).
 * res [N][max_res] (filled with -1 first), res_len [N]; steps [N][2] (advance, emit)
 * counts may be NULL. */
void oracle_greedy_decode(int Tp, int N, const float* f, const int32_t* f_lens, int bf16,
                          const float* embed, const float* const* pWih,
                          const float* const* pWhh, const float* const* pbih,
                          const float* const* pbhh, const float* W1t, const float* W1p,
                          const float* bt, const float* bp, const float* W2, const float* b2,
                          int32_t* res, int32_t* res_len, int max_res, int32_t* steps);
void oracle_greedy_decode_caps(int Tp, int N, const float* f, const int32_t* f_lens, int bf16,
                          const float* embed, const float* const* pWih,
                          const float* const* pWhh, const float* const* pbih,
                          const float* const* pbhh, const float* W1t, const float* W1p,
                          const float* bt, const float* bp, const float* W2, const float* b2,
                          int32_t* res, int32_t* res_len, int max_res, int32_t* steps, int32_t* caps);
void oracle_greedy_decode_walks(int Tp, int N, const float* f, const int32_t* f_lens, int bf16,
                          const float* embed, const float* const* pWih,
                          const float* const* pWhh, const float* const* pbih,
                          const float* const* pbhh, const float* W1t, const float* W1p,
                          const float* bt, const float* bp, const float* W2, const float* b2,
                          int32_t* res, int32_t* res_len, int max_res, int32_t* steps, int32_t* caps,
                                int32_t* walks);

/* Joint logits for explicit inputs (amx_linear_bf16_accum_relu + amx_linear_i16o32,
 * modeling_rnnt.py:259-289): f [N][1024], g [N][320] -> logits [N][29]. */
void oracle_joint(int N, const float* f, const float* g, int bf16, const float* W1t,
                  const float* W1p, const float* bt, const float* bp, const float* W2,
                  const float* b2, float* logits);

/* One prediction step for a batch (lstm_amx_bf16 / lstm): pre_g [N] int32 (SOS=-1),
 * h [2][N][320], c [2][N][320] in; g_out [N][320], h_out/c_out [2][N][320]. */
void oracle_prediction(int N, const int32_t* pre_g, const float* h, const float* c, int bf16,
                       const float* embed, const float* const* pWih, const float* const* pWhh,
                       const float* const* pbih, const float* const* pbhh, float* g_out,
                       float* h_out, float* c_out);

int oracle_num_threads(void);
int oracle_pin_threads(int n, const int* cpus);
int oracle_bind_master(int cpu);

#ifdef __cplusplus
}
#endif
#endif
